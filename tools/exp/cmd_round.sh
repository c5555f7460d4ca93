# round measurement in one call: cmd_final.sh (GPU suite, smoke, bench line with the CPU
# baseline, kernel stats, FETCH/WRITE passes, c4 / c5 lines) and the MFMA-utilisation passes
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-round}
bash tools/exp/cmd_final.sh $T || exit 1
bash tools/gpu_pmc_mfma.sh ${T}_mfma || exit 1
