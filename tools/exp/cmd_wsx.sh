# WS GEMM scheduling experiments (tools/microbench/ws_bench.hip builds under build/wsx/)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-wsx}; shift
mkdir -p $O
export CTN_GEMM_DUAL=3
for r in 1 2; do for b in "$@"; do echo "== $b run $r"; timeout -k 10 90 build/wsx/$b | grep "EXP\|us" || exit 1; done; done > $O/wsx.log 2>&1
cat $O/wsx.log
