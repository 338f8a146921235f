#!/bin/bash
# round 3: GPU suite + the T-scan investigation (rows 7..22, 4 chains, extra η multipliers)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03_scan}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "${2:-}" != "skip-tests" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
fi
timeout -k 10 900 python -u tools/ref_tscan.py --rows 22 21 20 19 18 17 16 15 14 13 12 11 10 9 8 7 --chains 4 \
  --extra-eta-mults 1.1 1.2 1.3 --out "$O/tscan" > "$O/tscan.log" 2>&1 || { tail -30 "$O/tscan.log"; exit 1; }
cat "$O/tscan.log"
