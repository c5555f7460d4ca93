# round 4: dual WS column split (CJ) x layout (RAWB) + store / compute bounds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4f}; mkdir -p $O
for sh in "3 1000 g 4" "32 3199 g 2" "3 1000 c 4" "64 7999 c 1"; do
  echo "== $sh" >> $O/mb.log
  timeout -k 10 120 build/dual_ws_bench_0 $sh >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
for v in 0_4_4_0 0_4_2_0 0_4_1_0 1_6_4_0 1_6_2_0 1_6_1_0 0_4_2_2 1_6_2_2 0_4_2_8 1_6_2_8 0_4_2_18 1_6_2_18 0_4_2_10 1_6_2_10; do
  for sh in "32 3199 g 1" "64 7999 c 1"; do
    echo "== $v $sh" >> $O/mb.log
    timeout -k 10 120 build/dual_ws_var_$v $sh >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
  done
done
grep -v "^   run\|reproducib" $O/mb.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_streaming.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_streaming.py > $O/streaming.log 2>&1 || { tail $O/streaming.log; exit 1; }
grep -v amdgpu.ids $O/streaming.log
