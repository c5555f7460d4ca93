# quick iteration: tblock/model GPU tests, a short bench, kernel stats
set -eo pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-q}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tblock.py tests/test_gpu_model.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 16
