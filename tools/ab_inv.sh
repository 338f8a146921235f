#!/bin/bash
# parity subset + C3 bench of the current build (inversion A/B)
set -e
O=gpurun_out/${1:-abinv}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "factorize or sweep or full_size or block_product" > $O/test.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 > $O/bench_$i.json 2>$O/bench_$i.err
  python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'], d['ms_per_step'], d.get('cr_inv'))" >> $O/summary.txt
done
