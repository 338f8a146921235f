set -o pipefail
mkdir -p gpurun_out/r03_inv0b
timeout -k 10 120 ./tools/micro/cr_inv0_stamps 12 16 > gpurun_out/r03_inv0b/inv0_stamps.txt 2>&1 && cat gpurun_out/r03_inv0b/inv0_stamps.txt | head -14 && \
DWHMC_LIB=$PWD/build/var/inv0b.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or physics or assembly" > gpurun_out/r03_inv0b/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03_inv0b/tests.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python -u tools/ab_bench.py --L 32 --beta 16 --Nt 7 --sweeps 3 --rounds 7 --variants "LIB=$PWD/build/var/pair0.so" "LIB=$PWD/build/var/inv0b.so" > gpurun_out/r03_inv0b/ab_C3.txt 2>&1 && cat gpurun_out/r03_inv0b/ab_C3.txt
