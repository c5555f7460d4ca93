set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_ab.sh r4fold base CTN_WS_FOLD=0 CTN_WS_FOLD=1 CTN_WS_FOLD=2 || exit 1
