# round 5: the N=2 bench job rehearsed on one GPU over gloo (code path only, not a
# measurement): chunked flat exchange (default) and one-message exchange
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5rehearse}
mkdir -p $O
export CTN_BENCH_REHEARSAL=1
for ch in 4 1; do
  CTN_FLAT_CHUNKS=$ch timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + ch)) bench.py --gpus 2 --steps 5 --warmup 2 --profile-steps 0 --no-cpu-baseline > $O/n2_chunks$ch.log 2>&1 || { tail -20 $O/n2_chunks$ch.log; exit 1; }
  tail -1 $O/n2_chunks$ch.log | cut -c1-220
done
