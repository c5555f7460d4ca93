set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_tblock.py tests/test_gpu_model.py -q -m gpu -x > gpurun_out/t8.log 2>&1; echo "TESTS EXIT $?"; tail -1 gpurun_out/t8.log
CTN_GEMM_BM=128 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/b6_128.log 2>&1; echo "BENCH128 EXIT $?"; tail -1 gpurun_out/b6_128.log | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/b6_64.log 2>&1; echo "BENCH64 EXIT $?"; tail -1 gpurun_out/b6_64.log | cut -c1-200
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof6 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/p6.log 2>&1; echo "PROF EXIT $?"
