# A/B of eigensolver build variants (build/var/<name>.so, "-" = the in-tree
# library): eigensystem accuracy / time at L=32 and 16, one-measurement and
# 16-snapshot transport times.  Usage: bash tools/gpu_qab.sh TAG name ...
set -o pipefail
O=gpurun_out/${1:?tag}; shift; mkdir -p $O
for v in "$@"; do
  if [ "$v" = "-" ]; then unset DWHMC_LIB; else export DWHMC_LIB=$PWD/build/var/$v.so; fi
  echo "== $v" >> $O/ab.txt
  timeout -k 10 200 python3 tools/qeig_vec_check.py 16 32 >> $O/ab.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/transport_single.py 32 5 >> $O/ab.txt 2>&1 || exit 1
  timeout -k 10 200 python3 tools/transport_single.py 32 2 16 >> $O/ab.txt 2>&1 || exit 1
done
if [ -n "${QAB_PROF:-}" ]; then
  unset DWHMC_LIB
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/transport_single.py 32 3 > /dev/null 2>&1
  rm -f $GRAFT_REPO_ROOT/$O/prof/run_kernel_trace.csv
fi
