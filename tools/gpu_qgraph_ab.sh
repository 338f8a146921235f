set -o pipefail
mkdir -p gpurun_out/gab
for r in 1 2; do
  for g in 0 1; do
    DWHMC_Q_GRAPH=$g timeout -k 10 200 python -u tests/bench_transport.py --steps 3 --snapshots 16 > gpurun_out/gab/t_${g}_$r.json 2> gpurun_out/gab/t_${g}_$r.err || exit 1
  done
done
DWHMC_Q_GRAPH=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transport.py tests/test_qeig_gpu.py -m gpu > gpurun_out/gab/tests.log 2>&1 || exit 1
