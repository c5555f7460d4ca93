# fragment-order resident weights: microbenchmarks (row-major vs fragment-order loads),
# then the A/B bench against build/ab/lib_prev.so (tools/exp/cmd_ab.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-frag}
O=gpurun_out/$T
mkdir -p $O
export CTN_GEMM_DUAL=3 WSB_NOSTREAM=1
for f in 0 1; do
  if [ $f = 1 ]; then export WSB_FRAG=1 DB_FRAG=1; fi
  echo "frag=$f" >> $O/mb.log
  timeout -k 10 60 build/mb/ws_bench | grep EXP >> $O/mb.log || exit 1
  timeout -k 10 60 build/mb/dual_bench | grep EXP >> $O/mb.log || exit 1
done
echo "no D partial stores" >> $O/mb.log
timeout -k 10 60 build/mb/dual_nod | grep EXP >> $O/mb.log || exit 1
DB_M=2 timeout -k 10 60 build/mb/dual_nod | grep EXP >> $O/mb.log || exit 1
DB_M=2 timeout -k 10 60 build/mb/dual_bench | grep EXP >> $O/mb.log || exit 1
cat $O/mb.log
unset CTN_GEMM_DUAL WSB_NOSTREAM WSB_FRAG DB_FRAG
AB_PROF=1 bash tools/exp/cmd_ab.sh $T
