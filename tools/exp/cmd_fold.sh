# round 4: consumer-side gLN statistics fold in the WS GEMMs: microbenchmark (batched
# fold loads), GPU suite, step A/B against finalize launches (CTN_WS_FOLD)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4fold; mkdir -p $O
WSB_FRAG=1 WSB_NOSTREAM=1 timeout -k 10 120 build/wsv/ws_foldfix > $O/mb.log 2>&1 || { cat $O/mb.log; exit 1; }
grep -v "^   " $O/mb.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r4fold_ab base CTN_WS_FOLD=0 CTN_WS_FOLD=2 || exit 1
