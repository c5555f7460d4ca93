set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_tblock.py tests/test_gpu_model.py -q -m gpu -x > gpurun_out/t7.log 2>&1; echo "TESTS EXIT $?"; tail -2 gpurun_out/t4.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/b5.log 2>&1; echo "BENCH EXIT $?"
tail -1 gpurun_out/b5.log | cut -c1-300
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/p5.log 2>&1; echo "PROF EXIT $?"
