#!/bin/bash
# Full GPU parity suite + CR plan dump + traced bench (via gpurun).
# Usage: bash tools/gpu_round.sh TAG [extra bench args]
set -eo pipefail
TAG=${1:?tag}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest "$R/tests" -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$O/tests.log" 2>&1
DWHMC_CR_PLAN_DUMP=1 timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline "$@" > "$O/bench.json" 2> "$O/plan.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 10 --no-cpu-baseline --no-timing "$@" > "$O/prof_bench.json" 2> "$O/prof.err"
python3 "$R/tools/trace_step.py" "$O/prof/run_kernel_trace.csv" > "$O/step.txt"
rm -f "$O/prof/run_kernel_trace.csv"
