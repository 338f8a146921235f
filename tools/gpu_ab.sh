#!/bin/bash
# GPU A/B pass (via gpurun): the CR parity subset, then tools/ab_bench.py on
# the given variants.  Usage: bash tools/gpu_ab.sh TAG "VAR=1" "VAR=0" [...]
set -o pipefail
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_parity.py" "$R/tests/test_gpu_assembly.py" -x -q \
  --timeout 120 --timeout-method thread -k "not low_temperature and not beta5000" > "$O/tests.log" 2>&1 \
  || { echo TESTS_FAILED; tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 300 python -u "$R/tools/ab_bench.py" --L 32 --beta 16 --Nt 7 --sweeps 4 --rounds 4 \
  --variants "$@" > "$O/ab.txt" 2>&1
rc=$?
cat "$O/ab.txt"
[ $rc -eq 0 ] || exit $rc
# one-step launch timeline of the default build (TRACE=0 skips)
if [ "${TRACE:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o run -- \
    python3 "$R/bench.py" --steps 14 --warmup 7 --no-cpu-baseline --no-c1 --no-timing > "$O/prof_bench.json" 2> "$O/prof.err" \
    || { echo TRACE_FAILED; tail -5 "$O/prof.err"; exit 1; }
  python3 "$R/tools/trace_step.py" "$O/prof/run_kernel_trace.csv" > "$O/step.txt"
  cat "$O/step.txt"
fi
