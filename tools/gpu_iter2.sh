# One optimisation iteration on the GPU box: GPU tests, a short bench, kernel stats.
# Each GPU step has its own limit; the chain stops at the first failure.
set -eo pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -q -m gpu -x > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err
cut -c1-220 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1
python tools/prof_summary.py $O/prof/run_kernel_stats.csv 7 16
