# round 4: dual microbench at the bench / c4 shapes, then the round measurement (cmd_final.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4g}
O=gpurun_out/$T; mkdir -p $O
for sh in "32 3199 g 3" "64 7999 c 2"; do
  echo "== $sh" >> $O/mb.log
  timeout -k 10 120 build/dual_ws_bench_0 $sh >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
for b in dual_ws_bench_1 dual_ws_bench_2 dual_ws_bench_4 dual_ws_bench_6 dual_ws_var_1_6_2_8 dual_ws_var_1_6_2_10 dual_ws_var_1_6_2_18 dual_ws_var_1_6_4_0 dual_ws_var_1_6_1_0 dual_ws_var_0_4_2_0; do
  echo "== $b" >> $O/mb.log
  timeout -k 10 120 build/$b 32 3199 g 1 >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
grep -v "^   run\|reproducib" $O/mb.log
bash tools/exp/cmd_final.sh $T || exit 1
bash tools/gpu_ab.sh ${T}_ab base CTN_HIP_LIB=$GRAFT_REPO_ROOT/build/var/libpk.so CTN_DUAL_WS=0 CTN_DEFER_REDUCE=0 || exit 1
timeout -k 10 600 python -u tools/train_paper_fixture.py --config c4 --steps 3000 --out $O/train_c4 > $O/train_c4.log 2>&1 || { tail $O/train_c4.log; exit 1; }
tail -3 $O/train_c4.log
python tools/trace_gaps.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/trace_gaps.txt
python tools/step_sequence.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/step_sequence.txt
