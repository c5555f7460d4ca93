# one iteration: GPU tests, bench, kernel stats, and two PMC passes (fetch bytes, LDS conflicts)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_tblock.py tests/test_gpu_model.py -q -m gpu -x > $O/tests.log 2>&1; echo "TESTS EXIT $?"; tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.log 2>&1; echo "BENCH EXIT $?"; tail -1 $O/bench.log | cut -c1-160
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1; echo "PROF EXIT $?"
i=0
for grp in "FETCH_SIZE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc$i.log 2>&1
  echo "PMC $i EXIT $?"
done
