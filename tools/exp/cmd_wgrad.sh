# parameter-gradient stream: its GPU tests, then the A/B bench (CTN_WGRAD_STREAM=0 as "prev")
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-wgrad}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_stream.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/wgrad_tests.log 2>&1
rc=$?
tail -15 gpurun_out/$T/wgrad_tests.log
[ $rc -le 1 ] || exit $rc        # test failures go on to the A/B; crashes, aborts, timeouts stop here
AB_PREV_ENV=CTN_WGRAD_STREAM=0 AB_PROF=1 bash tools/exp/cmd_ab.sh $T
