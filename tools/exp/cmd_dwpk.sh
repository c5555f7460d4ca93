# packed-fp32 depthwise kernels: the bench-shape bf16 model test on the default and the
# scalar build (build/var/libold.so), the block tests, then kernel times, one box
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-dwpk}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for L in 0 old; do
  if [ $L = 0 ]; then LIB=$GRAFT_REPO_ROOT/conv-tasnet_amd/libctn_hip.so; else LIB=$GRAFT_REPO_ROOT/build/var/lib$L.so; fi
  CTN_HIP_LIB=$LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_benchshape.py -k "bench_step_bf16" -x -q -s --timeout 200 --timeout-method thread > $O/bs_$L.log 2>&1
  echo "$L rc=$? $(grep -h 'SI-SNR diff' $O/bs_$L.log | cut -c1-160)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_tblock.py tests/test_gpu_layers.py tests/test_gpu_streaming.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PAT='dw_' bash tools/gpu_variants.sh ${T}_var 0 old 0 old
grep -o '"final_loss": [-0-9.]*' gpurun_out/${T}_var/b*.json
