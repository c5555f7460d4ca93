set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dv1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder_mfma.py tests/test_gpu_model.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh ${1:-dv1}ab base CTN_DU_COLS=0 2>&1 | grep -E "frame_outer|gemm_cols|enc_|frames|base|CTN"
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > $O/c5.json 2> $O/c5.err
tail -1 $O/c5.json | cut -c1-120
