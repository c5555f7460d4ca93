# round 5: N-image dual variants (build/dual_ws_nv_<nimg>_<nc>_<cjn>_<exp>)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5dvnv}
mkdir -p $O
for v in ${VARS:-0_8_4_0 1_8_4_0 1_8_2_0 1_4_4_0 1_4_2_0}; do
  for rep in 1 2; do
    timeout -k 10 90 ./build/dual_ws_nv_$v ${SHAPE:-32 3199 g} 2 > $O/nv_${v}_$rep.log 2>&1 || { echo "var $v failed"; tail $O/nv_${v}_$rep.log; exit 1; }
    echo "$v: $(grep -E '^M=|^reprod|^EXP .* ws ' $O/nv_${v}_$rep.log | tr '\n' ' ')"
  done
done
