# BN path + full GPU suite, then a short bench (regression check)
set -eo pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-bn}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -v -m gpu -k "bn" --timeout 120 --timeout-method thread > $O/bn.log 2>&1 || { tail -40 $O/bn.log; exit 1; }
tail -5 $O/bn.log
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-200
