# LDS-DMA column GEMM and WS ring: block/model tests, bench A/B (CTN_COLS_DMA) and the
# register-staged WS variant build (build/var/libwsreg.so), one box
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-cols1}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tblock.py tests/test_gpu_benchshape.py tests/test_gpu_model.py tests/test_gpu_layers.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh ${T}_ab base CTN_COLS_DMA=0 || exit 1
PAT='gemm_ws_kernel<0|gemm_cols' bash tools/gpu_variants.sh ${T}_var 0 wsreg
