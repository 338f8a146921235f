#!/bin/bash
# Eigensolver kernel profile at the batched workload (16 Δ snapshots of one
# L = 32 chain): kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes.
# bash tools/gpu_eig_prof.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- \
  python3 "$R/tests/bench_transport.py" --steps 1 --snapshots 16 --chains 1 > "$O/stats_bench.json" 2> "$O/stats.err" \
  || { tail -5 "$O/stats.err"; exit 1; }
rm -f "$O/stats/run_kernel_trace.csv"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- \
  python3 "$R/tests/bench_transport.py" --steps 1 --snapshots 16 --chains 1 > "$O/fetch.log" 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- \
  python3 "$R/tests/bench_transport.py" --steps 1 --snapshots 16 --chains 1 > "$O/write.log" 2>&1 || exit 1
ls -R "$O" | head -30
