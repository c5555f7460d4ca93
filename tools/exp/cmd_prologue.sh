# resident-weight prologue order: WS / dual GEMM microbenchmarks at M = 2 (one tile per
# workgroup: the fixed cost) and M = 32 (the bench shape), three builds each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-prologue}
mkdir -p $O
export CTN_GEMM_DUAL=3 WSB_NOSTREAM=1
for rep in 1 2; do
for m in 2 32; do
  for b in ws_late ws_early ws_now; do
    echo "$b" >> $O/ws.log
    WSB_M=$m timeout -k 10 60 build/mb/$b | grep EXP >> $O/ws.log || exit 1
  done
  for b in du_late du_early du_now; do
    echo "$b" >> $O/dual.log
    DB_M=$m timeout -k 10 60 build/mb/$b | grep EXP >> $O/dual.log || exit 1
  done
done
done
cat $O/ws.log $O/dual.log
