set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-c4a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 > $O/c4.json 2> $O/c4.err
tail -1 $O/c4.json | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 > $O/prof_c4.log 2>&1
python tools/prof_summary.py $(ls $O/prof_c4/*kernel_stats.csv | head -1) 4 12
