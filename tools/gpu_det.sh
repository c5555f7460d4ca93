# Dual-GEMM run-to-run reproducibility (tools/microbench/dual_det.hip) per diagnostic
# build under build/det/: <name>[:c] runs the cLN form.  Bound-finding / race hunt only.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1}; shift
mkdir -p $O
export CTN_GEMM_DUAL=3
IFS=';' read -ra SH <<< "${SHAPES:-32 3199;3 1000}"   # "M K;M K;..."
for spec in "$@"; do
  b=${spec%%:*}; nk=g; [ "$spec" != "$b" ] && nk=c
  for shape in "${SH[@]}"; do
    echo "== $b $nk $shape" >> $O/det.log
    timeout -k 10 150 build/det/$b $shape ${NRUN:-30} $nk >> $O/det.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "EXIT $rc" >> $O/det.log; cat $O/det.log; exit 1; }
  done
done
grep "==\|runs differ" $O/det.log
