# run the named microbenchmark binaries under build/ (bound-finding only)
set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1}; shift
mkdir -p $O
export CTN_GEMM_DUAL=3
for b in "$@"; do echo "== $b" >> $O/mb.log; timeout -k 10 90 build/$b >> $O/mb.log 2>&1; done
cat $O/mb.log
