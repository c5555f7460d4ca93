# round 4: flat exchange over a persistent gradient buffer the deferred blocks write into; A/B against the plain step + trace
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4sync5}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ddp.py tests/test_gpu_defer_reduce.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/plain$i.json 2> $O/plain$i.err || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --ddp > $O/flat$i.json 2> $O/flat$i.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --ddp --steps 5 --warmup 3 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 60 25 > $O/kernels.txt
for f in $O/*.json; do echo $f; tail -1 $f | cut -c1-200; done
