set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nf
timeout -k 10 120 python tools/exp/causal_prefix.py > gpurun_out/nf/prefix.log 2>&1; echo "prefix rc=$?"
cat gpurun_out/nf/prefix.log | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest tests/test_gpu_layers.py -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/nf/layers.log 2>&1; echo "layers rc=$?"
tail -40 gpurun_out/nf/layers.log
