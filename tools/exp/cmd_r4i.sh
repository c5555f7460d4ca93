# round 4: dual v3 microbench variants (slot layout x column split), then the round
# measurement (cmd_final.sh), trace gaps and one step's kernel sequence
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4i}
O=gpurun_out/$T; mkdir -p $O
for b in dual_ws_bench_0 dual_ws_var_0_4_1_0 dual_ws_var_0_4_4_0 dual_ws_var_1_6_2_0 dual_ws_var_1_6_1_0 dual_ws_bench_1 dual_ws_bench_2; do
  echo "== $b" >> $O/mb.log
  timeout -k 10 120 build/$b 32 3199 g 2 >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
echo "== c4 shape" >> $O/mb.log
timeout -k 10 120 build/dual_ws_bench_0 64 7999 c 2 >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
grep -v "^   run" $O/mb.log
bash tools/exp/cmd_final.sh $T || exit 1
python tools/trace_gaps.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/trace_gaps.txt
python tools/step_sequence.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/step_sequence.txt
head -5 $O/trace_gaps.txt
