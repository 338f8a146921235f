#!/bin/bash
# In-order A/B of library builds on one workload: bash tools/ab_libs.sh TAG "ARGS" lib1 lib2 ...
# (lib "-" = the in-tree build); tools/transport_single.py ARGS per lib, two rounds
set -o pipefail
TAG=${1:?tag}; ARGS=${2:?args}; shift 2
O=gpurun_out/$TAG
mkdir -p "$O"
for r in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then
      timeout -k 10 120 python tools/transport_single.py $ARGS > "$O/x.txt" 2>&1 || exit 1
    else
      DWHMC_LIB=$lib timeout -k 10 120 python tools/transport_single.py $ARGS > "$O/x.txt" 2>&1 || exit 1
    fi
    echo "$lib: $(cat "$O/x.txt")"
  done
done
