# Round-2 parity additions on one MI355X: bench-shape / c5 / trained-model / step
# tests, DDP over the HIP modules, and a DDP (RCCL) bench at world size 1.
set -eo pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-nt}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_benchshape.py tests/test_gpu_ddp.py -v -s -m gpu --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_plain.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --ddp --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_ddp.log 2>&1
echo "plain: $(tail -1 $O/bench_plain.log | cut -c1-190)"
echo "ddp:   $(tail -1 $O/bench_ddp.log | cut -c1-190)"
