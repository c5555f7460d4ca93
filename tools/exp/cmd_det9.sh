# dual GEMM: late-DMA and drained-epilogue variants (reproducibility, then timing)
set -o pipefail
NRUN=25 bash tools/gpu_det.sh det9 pl_late:c bp_late:c g_late pl_d1:c || exit 1
export CTN_GEMM_DUAL=3
for b in g g_d1 g_late c c_pl_d1 c_pl_late; do echo "== $b"; timeout -k 10 60 build/tb/$b || exit 1; done > gpurun_out/det9/timing.log 2>&1
cat gpurun_out/det9/timing.log
