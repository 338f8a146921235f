#!/bin/bash
# Own-eigensolver pass (via gpurun): bash tools/gpu_eig.sh TAG [quick]
# eigensolver tests, the transport + eig-path parity tests, transport timing
# with the own solver, and a kernel-trace profile of the L=32 measurement.
# (Round 6: the rocSOLVER A/B knob is gone; rocSOLVER runs only above n = 5120.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_transport.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "own_eigensolver or eigensystem" > "$O/eig_tests.log" 2>&1 || { tail -60 "$O/eig_tests.log"; exit 1; }
tail -3 "$O/eig_tests.log"
[ "${2:-}" = quick ] && exit 0
timeout -k 10 600 python -u -m pytest tests/test_transport.py tests/test_gpu_parity.py tests/test_simulation.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "transport or eig or simulation" > "$O/tests.log" 2>&1 \
  || { tail -60 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
timeout -k 10 300 python -u tests/bench_transport.py --steps 3 --snapshots 4,8,16 > "$O/transport_own.json" \
  2> "$O/transport_own.err" || { tail -20 "$O/transport_own.err"; exit 1; }
cat "$O/transport_own.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 "$R/tests/bench_transport.py" --steps 2 --snapshots "" --chains 1 > "$O/prof_bench.json" 2> "$O/prof.err" \
  || { tail -5 "$O/prof.err"; exit 1; }
rm -f "$O/prof/run_kernel_trace.csv"
head -25 "$O/prof/run_kernel_stats.csv" | cut -c1-160
