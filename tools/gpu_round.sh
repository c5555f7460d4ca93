# Round deliverables on one MI355X: GPU tests, smoke, the default bench line
# (with cpu_baseline), rocprofv3 --stats of the same bench command, and
# FETCH_SIZE / WRITE_SIZE passes for roofline.traffic.  Every GPU step has its
# own time limit and the chain stops at the first failure.
set -eo pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -q -m gpu -x > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc/p1 -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc1.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc/p2 -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc2.log 2>&1
# the JSON lands in profiles/ on the box only: copy $O/traffic.log to profiles/pmc_traffic.json here
python tools/pmc_traffic.py $O/pmc profiles/pmc_traffic.json > $O/traffic.log
echo PMC done
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py > $O/prof_bench.json 2>&1
echo PROF done
