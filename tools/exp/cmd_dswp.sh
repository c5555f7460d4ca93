# software-pipelined LDS-DMA WS GEMM (CTN_WS_DSWP) vs the library order, microbenchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dswp}
mkdir -p $O
export WSB_NOSTREAM=1 WSB_FRAG=1
for r in 1 2; do for b in ws_base ws_dswp; do
  echo "$b" >> $O/ws.log
  timeout -k 10 60 build/mb/$b | grep EXP | head -1 >> $O/ws.log || exit 1
done; done
cat $O/ws.log
