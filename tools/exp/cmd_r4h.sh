# round 4: the round measurement (cmd_final.sh), env A/B (packed-FP32 library, round-3 dual,
# per-block reductions), c4 fixture training, trace gaps and one step's kernel sequence
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4h}
O=gpurun_out/$T; mkdir -p $O
bash tools/exp/cmd_final.sh $T || exit 1
bash tools/gpu_ab.sh ${T}_ab base CTN_HIP_LIB=$GRAFT_REPO_ROOT/build/var/libpk.so CTN_DUAL_WS=0 CTN_DEFER_REDUCE=0 || exit 1
timeout -k 10 600 python -u tools/train_paper_fixture.py --config c4 --steps 3000 --out $O/train_c4 > $O/train_c4.log 2>&1 || { tail $O/train_c4.log; exit 1; }
tail -3 $O/train_c4.log
python tools/trace_gaps.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/trace_gaps.txt
python tools/step_sequence.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/step_sequence.txt
