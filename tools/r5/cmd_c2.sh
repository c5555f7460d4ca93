# round 5: column waves one vs two tiles per iteration (build/dual_ws_c2_<0|1>), c2 and c4 shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5c2}
mkdir -p $O
for shape in "32 3199 g" "64 7999 c"; do
  for rep in 1 2; do
    for v in 0 1; do
      timeout -k 10 90 ./build/dual_ws_c2_$v $shape 2 > $O/c2_${v}_${rep}_${shape// /_}.log 2>&1 || { echo "c2 $v failed"; tail $O/c2_${v}_${rep}_${shape// /_}.log; exit 1; }
      echo "C2=$v $shape: $(grep -E '^M=|^reprod|^EXP .* ws ' $O/c2_${v}_${rep}_${shape// /_}.log | tr '\n' ' ' | cut -c1-300)"
    done
  done
done
