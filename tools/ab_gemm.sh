#!/bin/bash
# parity subset + in-process A/B of block-product variants (via gpurun)
# Usage: bash tools/ab_gemm.sh TAG "VARIANT" ...   (tools/ab_bench.py syntax)
set -eo pipefail
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  > $O/test.log 2>&1
timeout -k 10 300 python -u tools/ab_bench.py --L 32 --beta 16 --rounds 4 --variants "$@" > $O/ab.txt 2>&1
