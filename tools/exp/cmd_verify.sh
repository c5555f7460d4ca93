# dual-GEMM reproducibility screen of the library build, then the GPU suite and the A/B
# bench against build/ab/lib_prev.so with a kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-verify}
SHAPES="3 1000;32 3199" NRUN=30 bash tools/gpu_det.sh $T lib:c lib || exit 1
AB_PROF=1 bash tools/exp/cmd_ab.sh $T
