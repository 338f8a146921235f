#!/bin/bash
# In-order A/B of environment settings on one workload:
#   bash tools/ab_env.sh TAG "ARGS" "VAR=a" "VAR=b" ...   (tools/transport_single.py ARGS, two rounds)
set -o pipefail
TAG=${1:?tag}; ARGS=${2:?args}; shift 2
O=gpurun_out/$TAG
mkdir -p "$O"
for r in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 120 python tools/transport_single.py $ARGS > "$O/x.txt" 2>&1 || exit 1
    echo "$v: $(cat "$O/x.txt")"
  done
done
