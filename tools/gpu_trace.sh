#!/bin/bash
# One step's launch timeline + plan dump for a config: bash tools/gpu_trace.sh TAG CONFIG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}; CFG=${2:?config}; shift 2
O=$R/gpurun_out/$TAG
mkdir -p "$O"
DWHMC_CR_PLAN_DUMP=1 timeout -k 10 200 python3 "$R/bench.py" --config "$CFG" --steps 50 --warmup 10 --no-cpu-baseline --no-c1 "$@" \
  > "$O/bench_$CFG.json" 2> "$O/plan_$CFG.txt" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$CFG" -o run -- \
  python3 "$R/bench.py" --config "$CFG" --steps 20 --warmup 10 --no-cpu-baseline --no-c1 --no-timing "$@" \
  > "$O/prof_bench_$CFG.json" 2> "$O/prof_$CFG.err" || exit 1
python3 "$R/tools/trace_step.py" "$O/prof_$CFG/run_kernel_trace.csv" > "$O/step_$CFG.txt"
rm -f "$O/prof_$CFG/run_kernel_trace.csv"
