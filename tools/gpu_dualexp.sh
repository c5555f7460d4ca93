set -eo pipefail
cd $GRAFT_REPO_ROOT
for e in 0 1 12 13 14 28 76 92 94 222; do CTN_GEMM_DUAL=3 timeout -k 10 60 ./build/dual_bench_$e 2>&1 | grep -v "^stream" | sed "s/^/EXP=$e /"; done
