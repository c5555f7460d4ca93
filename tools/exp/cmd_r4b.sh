# round 4: WS dual v2 (4 row + 8 column + 4 LDS-DMA memory waves): parity vs gemm_dual_kernel,
# reproducibility, timing (+ bound-finding builds), tests, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4b}; mkdir -p $O
for sh in "32 3199 g 8" "64 7999 c 3" "3 1000 c 8" "3 1000 g 8"; do
  echo "== $sh" >> $O/mb.log
  timeout -k 10 120 build/dual_ws_bench_0 $sh >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
for e in 1 2 4; do
  echo "== exp $e" >> $O/mb.log
  timeout -k 10 120 build/dual_ws_bench_$e 32 3199 g 1 >> $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
done
grep -v "^   run" $O/mb.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_tblock.py tests/test_gpu_benchshape.py tests/test_gpu_model.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0 1 0; do
  CTN_DUAL_WS=$v timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_$v.log 2>&1 || { tail $O/bench_$v.log; exit 1; }
  tail -1 $O/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('CTN_DUAL_WS=$v', d['value'], d['ms_per_step'], r['mean_ms'], r['frac'])"
done
