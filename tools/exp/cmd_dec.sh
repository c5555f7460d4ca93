set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dec1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decoder_mfma.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
PAT="dec_|frame_outer|ola|enc_" bash tools/gpu_ab.sh ${1:-dec1}ab base CTN_DEC_MFMA=0 2>&1 | grep -E "dec_|ola|base|CTN|frame_outer|enc_"
