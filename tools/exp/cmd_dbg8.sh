cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dbg4
for b in dual_ws_dbg_8_nopk dual_ws_dbg_8; do echo "== $b" >> gpurun_out/dbg4/out.log; timeout -k 10 120 build/$b 32 3199 g 4 >> gpurun_out/dbg4/out.log 2>&1 || exit 1; done
for sh in "32 3199 g 6" "64 7999 c 3" "3 1000 c 6"; do echo "== nopk $sh" >> gpurun_out/dbg4/out.log; timeout -k 10 120 build/dual_ws_bench_0_nopk $sh >> gpurun_out/dbg4/out.log 2>&1 || exit 1; done
cat gpurun_out/dbg4/out.log
