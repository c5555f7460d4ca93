# diagnostic builds of the wave-specialised dual GEMM (build/dual_ws_dbg_<bits>): shape list
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
for b in "$@"; do
  for sh in "32 3199 g 6" "64 7999 c 3"; do
    echo "== dbg $b shape $sh" >> $O/dbg.log
    timeout -k 10 90 build/dual_ws_dbg_$b $sh >> $O/dbg.log 2>&1 || { echo "EXIT $?" >> $O/dbg.log; cat $O/dbg.log; exit 1; }
  done
done
cat $O/dbg.log
