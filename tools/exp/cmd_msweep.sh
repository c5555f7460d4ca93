# fixed per-launch cost of the WS and dual GEMMs: time over the utterance count M
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-msweep}
mkdir -p $O
export CTN_GEMM_DUAL=3 WSB_NOSTREAM=1
for m in 2 4 8 16 32 64; do
  WSB_M=$m timeout -k 10 60 build/mb/ws_bench | grep EXP >> $O/ws.log || exit 1
  DB_M=$m timeout -k 10 60 build/mb/dual_bench >> $O/dual.log || exit 1
done
cat $O/ws.log $O/dual.log
