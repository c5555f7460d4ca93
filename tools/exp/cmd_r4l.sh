# round 4: deferral tests, env A/B (packed-FP32 library, round-3 dual, per-block
# reductions), host issue time per phase, c4 fixture training
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4l}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_defer_reduce.py tests/test_gpu_wgrad_stream.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh ${T}_ab base CTN_HIP_LIB=$GRAFT_REPO_ROOT/build/var/libpk.so CTN_DUAL_WS=0 CTN_DEFER_REDUCE=0 || exit 1
timeout -k 10 300 python tools/exp/host_phases.py > $O/host_phases.log 2>&1 || { tail $O/host_phases.log; exit 1; }
tail -15 $O/host_phases.log
timeout -k 10 600 python -u tools/train_paper_fixture.py --config c4 --steps 3000 --out $O/train_c4 > $O/train_c4.log 2>&1 || { tail $O/train_c4.log; exit 1; }
tail -3 $O/train_c4.log
