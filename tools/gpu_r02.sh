#!/bin/bash
# Round-2 GPU pass: parity suite, the driver's exact bench command, profiles,
# the other BASELINE configs, SQ counters.
# Usage (via gpurun): bash tools/gpu_r02.sh TAG [skip-tests]
set -eo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest "$R/tests" -m gpu -x -v --timeout 300 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > "$O/tests.log" 2>&1
fi
timeout -k 10 400 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err"
bash "$R/tools/profile_round.sh" "$TAG"
python3 "$R/tools/trace_step.py" "$R/gpurun_out/prof_$TAG/stats/run_kernel_trace.csv" > "$O/step.txt" || true
rm -f "$R/gpurun_out/prof_$TAG/stats/run_kernel_trace.csv"
timeout -k 10 300 python3 "$R/bench.py" --config C2 --no-c1 > "$O/bench_C2.json" 2> "$O/bench_C2.err"
timeout -k 10 300 python3 "$R/bench.py" --config C5 --no-c1 --no-cpu-baseline > "$O/bench_C5.json" 2> "$O/bench_C5.err"
bash "$R/tools/pmc_sq.sh" "$TAG"
