# round 5: dual GEMM bound-finding (build/dual_ws_bench_<bits>, CTN_DV_EXP: DESIGN.md §15)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5dvexp}
mkdir -p $O
for e in ${EXPS:-0 1 2 64 32 34 96 4 8}; do
  timeout -k 10 90 ./build/dual_ws_bench_$e 32 3199 g 1 > $O/exp_$e.log 2>&1 || { echo "exp $e failed"; tail $O/exp_$e.log; exit 1; }
  grep -E "^EXP|^COLS" $O/exp_$e.log
done
