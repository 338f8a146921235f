#!/bin/bash
# Second SQ/TCC PMC pass (via gpurun): LDS stalls and bank conflicts, L2 hit
# rate, per dispatch (tools/pmc_sq.sh layout).  Usage: bash tools/pmc_sq2.sh TAG
set -eo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d "$O/sq2" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 10 --therm 0 --no-c1 --no-cpu-baseline --no-timing > "$O/sq2.log" 2>&1
