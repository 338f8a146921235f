# A/B of the inverse iteration: 16-lane rows per eigenvalue (default) against
# one thread per eigenvalue (DWHMC_QINVIT_THREAD=1): eigensystem accuracy and
# time (tools/qeig_vec_check.py, tools/qeig_cluster_check.py), the transport
# bench, and the GPU transport / eigensolver tests on the default.
set -o pipefail
O=gpurun_out/qiab
mkdir -p $O
timeout -k 10 200 python -u tools/qeig_vec_check.py 8 16 32 > $O/vec_new.log 2>&1 || exit 1
DWHMC_QINVIT_THREAD=1 timeout -k 10 200 python -u tools/qeig_vec_check.py 8 16 32 > $O/vec_old.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/qeig_cluster_check.py 10 32 > $O/cl_new.log 2>&1 || exit 1
QCL_MU=0 timeout -k 10 200 python -u tools/qeig_cluster_check.py 8 32 >> $O/cl_new.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u tests/bench_transport.py --steps 3 --snapshots 16 > $O/t_new_$r.json 2> $O/t_new_$r.err || exit 1
  DWHMC_QINVIT_THREAD=1 timeout -k 10 200 python -u tests/bench_transport.py --steps 3 --snapshots 16 > $O/t_old_$r.json 2> $O/t_old_$r.err || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transport.py tests/test_qeig_gpu.py -m gpu > $O/tests.log 2>&1 || exit 1
