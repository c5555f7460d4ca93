# End-of-round check on one box: the whole GPU suite, smoke(), then the round
# deliverables (tools/gpu_round2.sh: bench line, kernel stats, PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_round2.sh ${T}_r2
