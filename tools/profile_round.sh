#!/bin/bash
# Kernel-trace + PMC traffic profile of bench.py at the headline workload, for
# profiles/.  Usage (on the GPU box, via gpurun):  bash tools/profile_round.sh TAG [ROUND]
# Writes gpurun_out/prof_TAG/{stats,fetch,write}/..., gpurun_out/TAG_traffic.json,
# gpurun_out/TAG_bench_under_rocprof.json and gpurun_out/TAG_bench.json
# (ROUND, default r02, names the committed traffic summary profiles/ROUND_pmc_traffic.json).
set -eo pipefail
TAG=${1:?tag}
ROUND=${2:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 --no-c1 > "$R/gpurun_out/${TAG}_bench_under_rocprof.json" 2> "$O/stats.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 10 --therm 10 --no-c1 --no-cpu-baseline > "$O/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 10 --therm 10 --no-c1 --no-cpu-baseline > "$O/write.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$O/fetch" "$O/write" --L 32 --beta 16 --chains 1 \
  -o "$R/gpurun_out/${TAG}_traffic.json" > "$O/traffic.txt"
cp "$R/gpurun_out/${TAG}_traffic.json" "$R/gpurun_out/${ROUND}_pmc_traffic.json"
