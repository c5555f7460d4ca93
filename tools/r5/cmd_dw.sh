# round 5: wave-item depthwise kernels — parity against the lane-group kernels, the
# spin-timeout reporting, determinism at the bench shapes, then bench A/B (CTN_DW_WAVE)
# and kernel stats of the default tree
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r5dw}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dw_wave.py tests/test_gpu_spin_timeout.py tests/test_gpu_determinism.py -x -v -m gpu --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for v in 1 0 1 0; do
  CTN_DW_WAVE=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_w$v.log 2>&1 || { tail $O/bench_w$v.log; exit 1; }
  echo "CTN_DW_WAVE=$v $(tail -1 $O/bench_w$v.log | cut -c1-130)"
  tail -1 $O/bench_w$v.log >> $O/bench_w$v.jsonl
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 0 > $O/prof.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 14 | tee $O/kernel_summary.txt
