#!/bin/bash
# quick GPU check (via gpurun): bash tools/gpu_quick.sh TAG — the CR/sweep parity
# subset, the driver's bench command, C2 and C5 lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_assembly.py tests/test_simulation.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "not low_temperature and not beta5000" > "$O/tests.log" 2>&1 \
  || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_driver.json" 2> "$O/bench_driver.err" \
  || { tail -20 "$O/bench_driver.err"; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 > "$O/bench_C3_200.json" 2> "$O/bench_C3_200.err" || exit 1
timeout -k 10 300 python -u bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline --no-c1 > "$O/bench_C2.json" 2> "$O/bench_C2.err" || exit 1
timeout -k 10 300 python -u bench.py --config C5 --steps 40 --warmup 8 --no-cpu-baseline --no-c1 > "$O/bench_C5.json" 2> "$O/bench_C5.err" || exit 1
python - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), round(d["value"], 1), "steps/s", round(d["ms_per_step"], 4), "ms/step")
PY
