set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-f2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/exp/host_phases.py > $O/hostph.log 2>&1; head -8 $O/hostph.log; tail -3 $O/hostph.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 > $O/c4.json 2> $O/c4.err
tail -1 $O/c4.json | cut -c1-160
