# round 5: optimizer fast paths, capturable Adam, whole-step HIP graph (tests, bench A/B, host phases)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5graph}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_optim.py tests/test_gpu_graph.py -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_eager.log 2>&1 || { tail $O/bench_eager.log; exit 1; }
tail -1 $O/bench_eager.log | cut -c1-160
timeout -k 10 300 python bench.py --no-cpu-baseline --graph > $O/bench_graph.log 2>&1 || { tail -30 $O/bench_graph.log; exit 1; }
tail -1 $O/bench_graph.log | cut -c1-160
timeout -k 10 300 python tools/exp/host_phases.py --sync --cprofile > $O/host_sync.log 2>&1 || exit 1
grep -A8 "host issue" $O/host_sync.log; grep "fast paths" $O/host_sync.log
