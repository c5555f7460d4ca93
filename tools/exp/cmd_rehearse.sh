# round 4: the bench's N-rank path (spawn_ranks, flat exchange, timing all-gather) as two
# gloo ranks on the one GPU; not a measurement
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-rehearse}
O=gpurun_out/$T; mkdir -p $O
CTN_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/n2_flat.json 2> $O/n2_flat.err || { tail -20 $O/n2_flat.err; exit 1; }
tail -1 $O/n2_flat.json | cut -c1-400
CTN_GRAD_SYNC=ddp CTN_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/n2_ddp.json 2> $O/n2_ddp.err || { tail -20 $O/n2_ddp.err; exit 1; }
tail -1 $O/n2_ddp.json | cut -c1-400
