# round 4: post-backward flat gradient all-reduce vs DDP hooks (world size 1, RCCL),
# and the DDP / flat-exchange GPU tests (two gloo ranks on the one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4sync}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ddp.py tests/test_gpu_defer_reduce.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/plain$i.json 2> $O/plain$i.err || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --ddp > $O/flat$i.json 2> $O/flat$i.err || exit 1
  CTN_GRAD_SYNC=ddp timeout -k 10 300 python bench.py --no-cpu-baseline --ddp > $O/ddp$i.json 2> $O/ddp$i.err || exit 1
done
python - <<'PY' $O
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), d["value"], d["ms_per_step"], d["config"]["parallelism"], d["config"]["deferred_grad_reduce_blocks"])
PY
