# round measurement: GPU suite, smoke, the default bench line (with the CPU baseline),
# kernel stats, whole-step HBM traffic (FETCH_SIZE / WRITE_SIZE passes), c4 line + stats
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O/pmc
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-250
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 12 | tee $O/kernel_summary.txt
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc/p$i.log 2>&1 || exit 1
done
python tools/pmc_traffic.py $O/pmc $O/pmc_traffic.json
python tools/pmc_step.py $O/pmc $(ls $O/prof/*kernel_trace.csv | head -1) 52.95 $O/pmc_step.json
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 > $O/c4.log 2>&1 || exit 1
tail -1 $O/c4.log | cut -c1-200
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/profc4 -o run --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 > $O/profc4.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/profc4/*kernel_stats.csv | head -1) 4 12 | tee $O/c4_kernel_summary.txt
timeout -k 10 300 python bench.py --config c5 --steps 6 --warmup 2 > $O/c5.log 2>&1 || exit 1
tail -1 $O/c5.log | cut -c1-200
