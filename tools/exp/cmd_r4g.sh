# round 4: dual microbench at the bench / c4 shapes, then the round measurement (cmd_final.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4g}
O=gpurun_out/$T; mkdir -p $O
for sh in "32 3199 g 3" "64 7999 c 2"; do
  echo "== $sh" >> $O/mb.log
  timeout -k 10 120 build/dual_ws_bench_0 $sh >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
grep -v "^   run" $O/mb.log
bash tools/exp/cmd_final.sh $T
timeout -k 10 600 python -u tools/train_paper_fixture.py --config c4 --steps 3000 --out $O/train_c4 > $O/train_c4.log 2>&1 || { tail $O/train_c4.log; exit 1; }
tail -3 $O/train_c4.log
