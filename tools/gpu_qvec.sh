# Quaternion eigensystem: correctness (tools/qeig_vec_check.py), one / 16-snapshot
# transport timings with and without it (DWHMC_EIG_QUAT=0), kernel stats.
# Usage: bash tools/gpu_qvec.sh TAG [Ls]
set -o pipefail
O=gpurun_out/${1:?tag}; mkdir -p $O
timeout -k 10 300 python3 tools/qeig_vec_check.py ${2:-4 6 8 12 16 32} > $O/v.txt 2>&1 || exit 1
timeout -k 10 120 python3 tools/transport_single.py 32 5 > $O/t_quat.txt 2>&1 || exit 1
DWHMC_EIG_QUAT=0 timeout -k 10 120 python3 tools/transport_single.py 32 5 > $O/t_one.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/transport_single.py 32 2 16 > $O/s_quat.txt 2>&1 || exit 1
DWHMC_EIG_QUAT=0 timeout -k 10 200 python3 tools/transport_single.py 32 2 16 > $O/s_one.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/transport_single.py 32 3 > /dev/null 2>&1
rm -f $GRAFT_REPO_ROOT/$O/prof/run_kernel_trace.csv
