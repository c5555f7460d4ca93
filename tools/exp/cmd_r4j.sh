# round 4: dual v3 (RAWB=1, CJ=1) microbench + bound variants, the c4 gradient test,
# then the round measurement (cmd_final.sh), trace gaps and one step's kernel sequence
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4j}
O=gpurun_out/$T; mkdir -p $O
for b in dual_ws_bench_0; do
  echo "== $b" >> $O/mb.log
  timeout -k 10 120 build/$b 32 3199 g 2 >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
echo "== c4 shape" >> $O/mb.log
timeout -k 10 120 build/dual_ws_bench_0 64 7999 c 2 >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
grep -v "^   run\|reproducib" $O/mb.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_benchshape.py -k "c4_shape_bf16_gradients" -x -q -s -m gpu --timeout 500 --timeout-method thread > $O/c4grad.log 2>&1; grep "largest\|passed\|failed" $O/c4grad.log
bash tools/exp/cmd_final.sh $T || exit 1
python tools/trace_gaps.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/trace_gaps.txt
python tools/step_sequence.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/step_sequence.txt
head -5 $O/trace_gaps.txt
