set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_model.py -q -m gpu > gpurun_out/t3.log 2>&1; echo "TESTS EXIT $?"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/b1.log 2>&1; echo "BENCH EXIT $?"
tail -2 gpurun_out/b1.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/p1.log 2>&1; echo "PROF EXIT $?"
