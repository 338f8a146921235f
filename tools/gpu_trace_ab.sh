#!/bin/bash
# Stage-by-stage A/B under rocprofv3 --kernel-trace (via gpurun):
#   bash tools/gpu_trace_ab.sh TAG "ENV1" "ENV2" ...   (each "K=V,K=V" or "-": the default)
# runs bench.py (C3 unless TRACE_ARGS) once per variant and prints
# tools/trace_steps_avg.py for each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i + 1))
  envs=()
  [ "$v" != "-" ] && IFS=, read -ra envs <<< "$v"
  ([ ${#envs[@]} -gt 0 ] && export "${envs[@]}"; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr$i" -o run -- \
    python3 "$R/bench.py" ${TRACE_ARGS:---steps 40 --warmup 5 --therm 20 --no-c1 --no-cpu-baseline --no-timing} \
    > "$O/tr$i.json" 2> "$O/tr$i.err") || { tail -20 "$O/tr$i.err"; exit 1; }
  f=$(ls "$O"/tr$i/run_kernel_trace.csv "$O"/tr$i/*/run_kernel_trace.csv 2>/dev/null | head -1)
  echo "== variant $i: $v"
  python3 "$R/tools/trace_steps_avg.py" "$f" | tee "$O/tr$i.txt" || exit 1
  rm -f "$f"
done
