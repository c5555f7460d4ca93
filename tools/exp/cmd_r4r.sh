# round 4: narrow streaming chunks (SC_W=8 for small calls): streaming tests, latency table,
# and the 1-stream 1-frame latency with the wide chunks for A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4r}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_streaming.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/bench_streaming.py --out $O/streaming.json > $O/streaming.log 2>&1 || { tail $O/streaming.log; exit 1; }
grep -v amdgpu.ids $O/streaming.log
CTN_SC_W=32 timeout -k 10 120 python tools/bench_streaming.py --streams 1,16 --frames 1,4 > $O/streaming_w32.log 2>&1 || exit 1
grep -v amdgpu.ids $O/streaming_w32.log
