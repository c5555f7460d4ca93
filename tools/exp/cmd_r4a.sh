# round 4: hazard probe wait states, WS dual (no packed FP32), tests, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 200 build/pk_hazard > $O/pk.log 2>&1 || { cat $O/pk.log; exit 1; }
cat $O/pk.log
for sh in "32 3199 g 8" "64 7999 c 3" "3 1000 c 8"; do
  echo "== $sh" >> $O/mb.log
  timeout -k 10 120 build/dual_ws_bench_0 $sh >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
grep -v "^   run" $O/mb.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_tblock.py tests/test_gpu_benchshape.py tests/test_gpu_model.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
CTN_DUAL_WS=0 timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_old.log 2>&1 || { tail $O/bench_old.log; exit 1; }
tail -1 $O/bench_old.log | cut -c1-400
