# round 4: dw_bwd window operand precompute + COLS CJC=4: the GPU suite, A/B (tiled column
# kernel), streaming latency
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4p}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh ${T}_ab base CTN_COLS_WS=0 || exit 1
timeout -k 10 300 python tools/bench_streaming.py > $O/streaming.log 2>&1 || { tail $O/streaming.log; exit 1; }
grep -v amdgpu.ids $O/streaming.log | tail -30
