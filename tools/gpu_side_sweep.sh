#!/bin/bash
# side-work placement sweep (DWHMC_CR_SIDE_W / _M) at C3, C2, C5 with tools/ab_bench.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
V="CR_SIDE_W=2 CR_SIDE_W=1 CR_SIDE_W=3 CR_SIDE_M=2 CR_SIDE_M=8 CR_SIDE=0"
timeout -k 10 300 python -u tools/ab_bench.py --L 32 --beta 16 --Nt 7 --sweeps 3 --rounds 5 --variants $V \
  > "$O/side_C3.txt" 2>&1 || { tail -20 "$O/side_C3.txt"; exit 1; }
cat "$O/side_C3.txt"
timeout -k 10 300 python -u tools/ab_bench.py --L 48 --beta 32 --chains 4 --Nt 7 --sweeps 2 --rounds 3 --variants $V \
  > "$O/side_C5.txt" 2>&1 || { tail -20 "$O/side_C5.txt"; exit 1; }
cat "$O/side_C5.txt"
