# streaming kernels: tests (reference causal fixture + whole forward), then latency/throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-stream}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_streaming.py tests/test_gpu_benchshape.py -x -v --timeout 300 --timeout-method thread -k "stream or c4_shape" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/bench_streaming.py --out $O/streaming.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cat $O/bench.log
