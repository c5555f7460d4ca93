# WS GEMM register prefetch depth 2 for the 8-wave configurations vs the library (1)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pf2}
mkdir -p $O
export WSB_NOSTREAM=1 WSB_FRAG=1
for r in 1 2; do for b in ws_base ws_pf2; do
  echo "$b" >> $O/ws.log
  timeout -k 10 60 build/mb/$b | grep EXP >> $O/ws.log || exit 1
done; done
cat $O/ws.log
