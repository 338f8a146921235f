#!/bin/bash
# One SQ/GRBM PMC pass over a short bench (via gpurun): wave cycles split into
# active / issue-stall / parked, for the per-dispatch analysis of the CR
# stages (tools/pmc_stage.py).  Usage: bash tools/pmc_sq.sh TAG
set -eo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$O/sq" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 10 --therm 0 --no-c1 --no-cpu-baseline --no-timing > "$O/sq.log" 2>&1
python3 "$R/tools/pmc_stage.py" "$O/sq" > "$O/sq_stage.txt"
