# WS GEMM bound-finding with fragment-ordered weights: library build and builds without
# stores (1), A loads (2), MFMAs (4), epilogue math (8), loads+stores (3), MFMA+math (12)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-wsbound}
mkdir -p $O
export WSB_NOSTREAM=1 WSB_FRAG=1
for e in 0 1 2 4 8 3 12; do
  timeout -k 10 60 build/mb/ws_e$e | grep EXP >> $O/ws.log || exit 1
done
cat $O/ws.log
