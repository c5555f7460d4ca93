# round 4: dual v2 raw-d-in-B layout (RAWB) parity + ring depth; block/determinism/streaming tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4e}; mkdir -p $O
for sh in "3 1000 g 6" "2 700 g 6" "32 3199 g 4" "3 1000 c 6" "64 7999 c 2"; do
  echo "== $sh" >> $O/mb.log
  timeout -k 10 120 build/dual_ws_bench_0 $sh >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
echo "== dbg16" >> $O/mb.log
timeout -k 10 120 build/dual_ws_dbg_16 32 3199 g 1 >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
for b in dual_ws_var_0_4_0 dual_ws_var_1_4_0 dual_ws_var_1_5_0 dual_ws_var_1_6_0 dual_ws_var_0_4_1 dual_ws_var_1_4_1 dual_ws_var_1_6_1 dual_ws_bench_2 dual_ws_bench_4; do
  echo "== $b" >> $O/mb.log
  timeout -k 10 120 build/$b 32 3199 g 1 >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
grep -v "^   run" $O/mb.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_tblock.py tests/test_gpu_determinism.py tests/test_gpu_streaming.py tests/test_gpu_wgrad_stream.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_streaming.py > $O/streaming.log 2>&1 || { tail $O/streaming.log; exit 1; }
tail -25 $O/streaming.log
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-250
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 14 | tee $O/kernel_summary.txt
