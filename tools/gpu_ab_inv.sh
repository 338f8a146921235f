#!/bin/bash
# A/B of an inversion variant: bash tools/gpu_ab_inv.sh TAG VAR.so BASE.so — parity suite on VAR, then
# the in-process A/B (tools/ab_bench.py) at C3, C2, C5
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}; VAR=${2:?variant .so}; BASE=${3:?base .so}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
DWHMC_LIB=$R/$VAR timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "parity or physics or assembly or simulation" > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 300 python -u tools/ab_bench.py --L 32 --beta 16 --Nt 7 --sweeps 3 --rounds 5 \
  --variants "LIB=$R/$BASE" "LIB=$R/$VAR" > "$O/ab_C3.txt" 2>&1 || { tail -20 "$O/ab_C3.txt"; exit 1; }
cat "$O/ab_C3.txt"
timeout -k 10 300 python -u tools/ab_bench.py --L 16 --beta 8 --Nt 7 --sweeps 3 --rounds 5 \
  --variants "LIB=$R/$BASE" "LIB=$R/$VAR" > "$O/ab_C2.txt" 2>&1 || { tail -20 "$O/ab_C2.txt"; exit 1; }
cat "$O/ab_C2.txt"
timeout -k 10 300 python -u tools/ab_bench.py --L 48 --beta 32 --chains 4 --Nt 7 --sweeps 2 --rounds 3 \
  --variants "LIB=$R/$BASE" "LIB=$R/$VAR" > "$O/ab_C5.txt" 2>&1 || { tail -20 "$O/ab_C5.txt"; exit 1; }
cat "$O/ab_C5.txt"
