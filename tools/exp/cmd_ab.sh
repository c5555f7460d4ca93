# A/B of the bench line between the in-tree library and build/ab/lib_prev.so on one box
# (alternating runs), optional microbench binaries first: cmd_ab.sh TAG [bin ...].
# AB_PREV_ENV="VAR=value ..." makes "prev" the in-tree library under that environment;
# AB_BENCH="..." replaces the bench arguments (default: c2, 20 steps).
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-ab}; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for b in "$@"; do
  timeout -k 10 90 $b | grep EXP > $O/$(basename $b).log || exit 1
  echo "== $b"; cat $O/$(basename $b).log
done
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  env ${AB_PREV_ENV:-CTN_HIP_LIB=$PWD/build/ab/lib_prev.so} timeout -k 10 200 python bench.py ${AB_BENCH:---no-cpu-baseline --steps 20 --warmup 5} > $O/bench_prev$i.log 2>&1 || exit 1
  echo "prev$i $(tail -1 $O/bench_prev$i.log | cut -c1-120)"
  timeout -k 10 200 python bench.py ${AB_BENCH:---no-cpu-baseline --steps 20 --warmup 5} > $O/bench_new$i.log 2>&1 || exit 1
  echo "new$i  $(tail -1 $O/bench_new$i.log | cut -c1-120)"
done
if [ -n "$AB_PROF" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
  python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 10
fi
