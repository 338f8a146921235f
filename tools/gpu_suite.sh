#!/bin/bash
# GPU test suite pass (via gpurun): bash tools/gpu_suite.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest "$R/tests" -m gpu -x -v --timeout 300 --timeout-method thread \
  ${2:+-k "$2"} > "$O/tests.log" 2>&1
rc=$?
tail -5 "$O/tests.log"
exit $rc
