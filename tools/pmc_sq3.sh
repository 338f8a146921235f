#!/bin/bash
# Instruction-class / issue split of the CR kernels (round 5, via gpurun):
# lists the gfx950 counters (rocprofv3 -L), keeps the requested SQ counters
# that exist, and runs one --pmc pass per group (<= 8 SQ counters each) over a
# short bench.  Usage: bash tools/pmc_sq3.sh TAG [bench args...]
set -o pipefail
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$O/counters_avail.txt" 2>&1 || true
ARGS=${*:-"--steps 10 --warmup 10 --therm 0 --no-c1 --no-cpu-baseline --no-timing"}
have() { grep -qw "$1" "$O/counters_avail.txt"; }
run_group() {   # name counters...
  local name=$1; shift
  local keep=()
  for c in "$@"; do have "$c" && keep+=("$c"); done
  echo "pass $name: ${keep[*]}"
  [ ${#keep[@]} -gt 0 ] || return 0
  timeout -s KILL 90 rocprofv3 --pmc "${keep[@]}" --output-format csv -d "$O/sq3_$name" -o run -- \
    python3 "$R/bench.py" $ARGS > "$O/sq3_$name.log" 2>&1
}
run_group A SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS || exit 1
run_group B SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC || exit 1
run_group C SQ_WAVE_CYCLES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR || exit 1
run_group D SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_TRANS_F64 SQ_INST_LEVEL_VMEM SQ_IFETCH || exit 1
[ -n "${SQ3_MEM:-}" ] && { run_group E SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum || exit 1; }
echo "sq3 done"
