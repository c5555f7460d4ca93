# the calibration copy's test, then two default bench lines (copy_peak, live timer stride 9)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-copy}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_copy.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  CTN_COPY_VERBOSE=1 timeout -k 10 400 python bench.py > $O/bench_$r.log 2> $O/bench_$r.err || { tail $O/bench_$r.err; exit 1; }
  tail -1 $O/bench_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['copy_peak'], r['copy_peak_by'], r['frac_of_copy_peak'], r['mean_ms'], r['launches'])"
  grep ctn_copy_bytes $O/bench_$r.err || true
done
