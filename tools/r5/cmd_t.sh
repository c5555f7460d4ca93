# round 5: run the given pytest node ids on the GPU (quick checks)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest "$@" -x -v -m gpu --timeout 400 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" $O/tests.log | cut -c1-600 | tail -30
exit $rc
