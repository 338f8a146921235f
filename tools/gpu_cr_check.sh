#!/bin/bash
# Quick GPU check of the CR path (via gpurun): CR parity subset, bench without
# and with kernel timers, and a rocprofv3 kernel trace of a short bench.
# Usage: bash tools/gpu_cr_check.sh TAG [extra bench args]
set -eo pipefail
TAG=${1:?tag}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest "$R/tests/test_gpu_parity.py" -x -q --timeout 120 --timeout-method thread \
  -k "cr" > "$O/tests.log" 2>&1
timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --no-timing "$@" > "$O/bench_notiming.json" 2> "$O/bench.err"
timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline "$@" > "$O/bench.json" 2>> "$O/bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 10 --no-cpu-baseline --no-timing "$@" > "$O/prof_bench.json" 2> "$O/prof.err"
python3 "$R/tools/trace_step.py" "$O/prof/run_kernel_trace.csv" > "$O/step.txt"
