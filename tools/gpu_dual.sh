# dual-GEMM iteration: parity tests for the dual path, then microbench variants
set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dual}; shift
mkdir -p $O
CTN_GEMM_DUAL=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_tblock.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for e in "$@"; do CTN_GEMM_DUAL=3 timeout -k 5 60 ./build/dual_bench_$e; done
