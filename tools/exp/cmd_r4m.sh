# round 4: WS GEMM flag-ring variants (microbench), the GPU suite (c4 trained fixture,
# deferral, determinism), the bench line and kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4m}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for b in ws_fl0_dr4 ws_fl1_dr4 ws_fl1_dr6 ws_fl1_dr8; do
  echo "== $b" >> $O/mb.log
  WSB_FRAG=1 WSB_NOSTREAM=1 timeout -k 10 120 build/wsv/$b >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
grep -v "^   " $O/mb.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 12 | tee $O/kernel_summary.txt
