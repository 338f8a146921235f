#!/bin/bash
# round 3 GPU pass: bash tools/gpu_r03.sh TAG [skip-tests] — GPU suite (incl. the
# published T-scan pin), the driver's bench command with both pole tables, C2 / C5
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
for tab in budget strict; do
  DWHMC_POLE_TABLE=$tab timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
    > "$O/bench_C3_$tab.json" 2> "$O/bench_C3_$tab.err" || { tail -20 "$O/bench_C3_$tab.err"; exit 1; }
  DWHMC_POLE_TABLE=$tab timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 \
    > "$O/bench_C3_200_$tab.json" 2> "$O/bench_C3_200_$tab.err" || { tail -20 "$O/bench_C3_200_$tab.err"; exit 1; }
  DWHMC_POLE_TABLE=$tab timeout -k 10 300 python -u bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 \
    > "$O/bench_C2_$tab.json" 2> "$O/bench_C2_$tab.err" || { tail -20 "$O/bench_C2_$tab.err"; exit 1; }
  DWHMC_POLE_TABLE=$tab timeout -k 10 300 python -u bench.py --config C5 --steps 40 --warmup 8 --no-cpu-baseline --no-c1 \
    > "$O/bench_C5_$tab.json" 2> "$O/bench_C5_$tab.err" || { tail -20 "$O/bench_C5_$tab.err"; exit 1; }
done
python - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(os.path.basename(f), round(d["value"], 1), "steps/s", "poles", d["config"]["poles"],
              "frac", round((d.get("roofline") or {}).get("frac") or 0, 3), "alg_tflops", round(d.get("alg_tflops", 0), 2))
    except Exception as e:
        print(f, e)
PY
