# k_q_orth (cluster / crowd Cholesky QR) on clean lattices: accuracy, eigensystem time,
# kernel time under rocprofv3, and the clean-lattice GPU tests
set -o pipefail
O=gpurun_out/qorth
mkdir -p $O
timeout -k 10 200 python -u tools/qeig_cluster_check.py 10 32 > $O/cl.log 2>&1 || exit 1
QCL_MU=0 timeout -k 10 200 python -u tools/qeig_cluster_check.py 8 32 >> $O/cl.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/qeig_cluster_check.py 32 > $O/prof.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transport.py -m gpu -k "clean or cluster or particle_hole or degenerate or full_size" > $O/tests.log 2>&1 || exit 1
