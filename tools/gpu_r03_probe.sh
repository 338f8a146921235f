#!/bin/bash
# round-3 probe: new guard-recovery tests, T-scan timing, driver bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_probe
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "guard or reselect or throughput or split_trajectory" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
timeout -k 10 300 python -u tools/ref_tscan.py --rows 22 15 --chains 2 --out "$O/tscan" > "$O/tscan.log" 2>&1 || { tail -30 "$O/tscan.log"; exit 1; }
cat "$O/tscan.log"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
