# cLN statistics batch in the WS GEMMs: microbenchmark (library build before/after),
# the GPU suite and the c4 A/B against build/ab/lib_prev.so with kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-clnb}
O=gpurun_out/$T
mkdir -p $O
for b in ws_old ws_new ws_old ws_new; do
  echo "$b" >> $O/mb.log
  WSB_NOSTREAM=1 WSB_FRAG=1 timeout -k 10 60 build/mb/$b | grep "fwd2" >> $O/mb.log || exit 1
done
cat $O/mb.log
AB_BENCH="--config c4 --steps 8 --warmup 2" bash tools/exp/cmd_ab.sh $T || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/profc4 -o run --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 > $O/profc4.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/profc4/*kernel_stats.csv | head -1) 4 8
