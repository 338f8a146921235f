# the per-batch-size choice of the inverse iteration (launch_q_invit): the
# transport bench at 1, 4, 8, 16 snapshots, default against forced variants
set -o pipefail
O=gpurun_out/qiab2
mkdir -p $O
for r in 1 2; do
  for v in def 0 1; do
    if [ $v = def ]; then unset DWHMC_QINVIT_THREAD; else export DWHMC_QINVIT_THREAD=$v; fi
    timeout -k 10 200 python -u tests/bench_transport.py --steps 3 --snapshots 4,8,16 > $O/t_${v}_$r.json 2> $O/t_${v}_$r.err || exit 1
  done
done
unset DWHMC_QINVIT_THREAD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transport.py tests/test_qeig_gpu.py tests/test_simulation.py -m gpu > $O/tests.log 2>&1 || exit 1
