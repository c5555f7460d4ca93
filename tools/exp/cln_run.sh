set -eo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cln
timeout -k 10 600 python -u -m pytest tests/test_gpu_tblock.py tests/test_gpu_model.py tests/test_gpu_streaming.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/cln/tests.log 2>&1 || { tail -30 gpurun_out/cln/tests.log; exit 1; }
tail -2 gpurun_out/cln/tests.log
bash tools/gpu_cfgprof.sh cfgp3 > gpurun_out/cln/cfg.log 2>&1; head -14 gpurun_out/cln/cfg.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/cln/c2.log 2>&1
tail -1 gpurun_out/cln/c2.log | cut -c1-150
