# consumer-side statistics fold: WS GEMM microbench, GPU suite, bench line and kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-fold}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 90 build/wsx/fold2 | grep EXP > $O/ws.log || exit 1
cat $O/ws.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-160
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 10
