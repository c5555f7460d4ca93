# WS GEMM LDS-DMA ring: the whole GPU suite and smoke() on the default build, then the
# ring-depth variants (build/var/libdr<D>.so, -DCTN_WS_DR=D) by kernel time, one box
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-wsdr}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
PAT='gemm_ws_kernel<0' bash tools/gpu_variants.sh ${T}_var 0 dr3 dr6 dr8
