#!/bin/bash
# round 3 evidence pass: bash tools/gpu_r03_final.sh TAG [skip-tests] — full GPU
# suite, the driver's bench command, rocprofv3 kernel stats + the two PMC passes
# (profile_round.sh, summary -> gpurun_out/r03_pmc_traffic.json), one step's
# launch timeline, C2 / C5 lines, the transport snapshot timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "${2:-}" != "skip-tests" ]; then
  DWHMC_TSCAN_RECORD=$O/tscan_record.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
    --timeout 450 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
  tail -3 "$O/tests.log"
fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" \
  || { tail -20 "$O/bench_driver.err"; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 \
  > "$O/bench_C3_200.json" 2> "$O/bench_C3_200.err" || exit 1
bash tools/profile_round.sh "$TAG" r03 || exit 1
python3 tools/trace_step.py "$R/gpurun_out/prof_$TAG/stats/run_kernel_trace.csv" > "$O/step.txt" || exit 1
rm -f "$R/gpurun_out/prof_$TAG/stats/run_kernel_trace.csv"
timeout -k 10 300 python -u bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 \
  > "$O/bench_C2.json" 2> "$O/bench_C2.err" || exit 1
timeout -k 10 300 python -u bench.py --config C5 --steps 40 --warmup 8 --no-cpu-baseline --no-c1 \
  > "$O/bench_C5.json" 2> "$O/bench_C5.err" || exit 1
timeout -k 10 200 python -u tests/bench_transport.py --steps 3 --snapshots 4,8,16 > "$O/transport.json" 2> "$O/transport.err" || exit 1
python - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(os.path.basename(f), round(d["value"], 1), "steps/s", "poles", d["config"]["poles"],
              "frac", round((d.get("roofline") or {}).get("frac") or 0, 3), "alg_frac", d.get("alg_frac_of_peak"))
    except Exception as e:
        print(f, e)
PY
