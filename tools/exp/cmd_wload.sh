# resident-weight load pattern: WS GEMM microbenchmark at M = 2 and 32 for the
# library build and timing-only builds (no loads / contiguous 1-KiB / rotated order)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-wload}
mkdir -p $O
export WSB_NOSTREAM=1
for m in 2 32; do
  for b in ws_late ws_now ws_contig ws_rot ws_crot ws_late; do
    echo "$b" >> $O/ws.log
    WSB_M=$m timeout -k 10 60 build/mb/$b | grep EXP >> $O/ws.log || exit 1
  done
done
cat $O/ws.log
