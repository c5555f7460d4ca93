# Wave-specialised pair-A dual GEMM on the box: microbenchmark (parity vs gemm_dual_kernel,
# reproducibility, time; bound-finding builds), then optional test files and bench.
# usage: gpu_dualws.sh <tag> [pytest files...]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
for e in ${DV_EXPS:-0 1 2 4 6}; do
  for sh in "32 3199 g 8" "3 1000 g 8" "64 7999 c 4" "3 1000 c 8"; do
    [ $e != 0 ] && [ "$sh" != "32 3199 g 8" ] && continue
    echo "== exp $e shape $sh" >> $O/mb.log
    timeout -k 10 90 build/dual_ws_bench_$e $sh >> $O/mb.log 2>&1 || { echo "EXIT $?" >> $O/mb.log; cat $O/mb.log; exit 1; }
  done
done
cat $O/mb.log
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-300
  CTN_DUAL_WS=0 timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_old.log 2>&1 || { tail $O/bench_old.log; exit 1; }
  tail -1 $O/bench_old.log | cut -c1-300
fi
