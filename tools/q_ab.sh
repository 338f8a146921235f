# A/B of quaternion-reduction build variants (build/var/<name>.so): the
# reduction's device time per variant, via tools/qeig_check.py
set -o pipefail
out=${QAB_OUT:-gpurun_out/qab}
mkdir -p $out
for v in "$@"; do
  echo "== $v" >> $out/q.txt
  DWHMC_LIB=$PWD/build/var/$v.so timeout -k 10 120 python3 tools/qeig_check.py ${QAB_L:-32} >> $out/q.txt 2>&1 || exit 1
done
