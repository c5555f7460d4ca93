# round 4: wave-specialised column GEMM (dW1): its test, the GPU suite, bench + kernel
# stats, A/B against the tiled column kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4n}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_cols_ws.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/cols.log 2>&1 || { tail -30 $O/cols.log; exit 1; }
tail -1 $O/cols.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh ${T}_ab base CTN_COLS_WS=0 || exit 1
