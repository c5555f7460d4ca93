# WS GEMM LDS-DMA rings: block/model tests on the default build, then kernel times
# against builds without the output/gx-GEMM rings (build/var/libnog.so) and without
# any ring (build/var/libreg.so), one box
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-wsn}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tblock.py tests/test_gpu_benchshape.py tests/test_gpu_model.py tests/test_gpu_layers.py tests/test_gpu_streaming.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
PAT='gemm_ws_kernel<' bash tools/gpu_variants.sh ${T}_var 0 nog reg 0
grep -o '"final_loss": [-0-9.]*' gpurun_out/${T}_var/b*.json
