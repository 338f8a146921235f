#!/bin/bash
# In-order A/B of library builds with the eigensolver's phase times:
#   bash tools/ab_libs_phase.sh TAG "ARGS" PHASE lib1 lib2 ...   (lib "-" = the in-tree build)
set -o pipefail
TAG=${1:?tag}; ARGS=${2:?args}; PH=${3:?phase}; shift 3
O=gpurun_out/$TAG
mkdir -p "$O"
for r in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then L=""; else L="DWHMC_LIB=$lib"; fi
    env $L DWHMC_EIG_DEBUG=1 timeout -k 10 120 python tools/transport_single.py $ARGS > "$O/x.txt" 2>&1 || exit 1
    echo "$lib: $(grep "$PH" "$O/x.txt" | tail -1) | $(tail -1 "$O/x.txt")"
  done
done
