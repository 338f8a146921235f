#!/bin/bash
# A/B of the block-product stage configurations (via gpurun): CR parity subset,
# then for each forced DWHMC_CR_GEMM=TS:KSPLIT (and the model's choice) a short
# kernel-traced bench; per-launch step timelines in gpurun_out/TAG/step_<cfg>.txt.
# Usage: bash tools/cr_cfg_sweep.sh TAG [cfg ...]
set -eo pipefail
TAG=${1:?tag}; shift || true
CFGS=${*:-auto 32:1 16:1 16:2 16:4 32:2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest "$R/tests/test_gpu_parity.py" -x -q --timeout 120 --timeout-method thread \
  -k "cr" > "$O/tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
for c in $CFGS; do
  n=${c/:/_}
  if [ "$c" = auto ]; then unset DWHMC_CR_GEMM; else export DWHMC_CR_GEMM=$c; fi
  DWHMC_CR_PLAN_DUMP=1 timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline --no-timing --steps 20 \
    > "$O/bench_$n.json" 2> "$O/plan_$n.txt"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$n" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 10 --no-cpu-baseline --no-timing > /dev/null 2> "$O/prof_$n.err"
  python3 "$R/tools/trace_step.py" "$O/prof_$n/run_kernel_trace.csv" > "$O/step_$n.txt"
  rm -rf "$O/prof_$n"
done
