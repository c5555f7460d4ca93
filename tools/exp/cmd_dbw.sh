# decoder MFMA tests, a bench line and the decoder kernels' times (one box)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dbw1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python tools/exp/enc_check.py > $O/enc_check.log 2>&1 && cat $O/enc_check.log || { tail -20 $O/enc_check.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder_mfma.py tests/test_gpu_model.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-150
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 40 | grep -E "dec_|enc_|total"
