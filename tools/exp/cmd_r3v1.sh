# round 3: dual GEMM with late DMA issue + permlane row sums (+ DMA'd cLN statistics):
# reproducibility screen, the whole GPU suite, c2 and c4 bench lines with kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r3v1}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
SHAPES="32 3199;3 1000;64 7999" NRUN=40 bash tools/gpu_det.sh $T base base:c > /dev/null || exit 1
grep "runs differ" $O/det.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-150
timeout -k 10 200 python bench.py --config c4 --steps 10 --warmup 3 > $O/c4.log 2>&1 || exit 1
tail -1 $O/c4.log | cut -c1-150
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 12
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/profc4 -o run --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 > $O/profc4.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/profc4/*kernel_stats.csv | head -1) 3 12
