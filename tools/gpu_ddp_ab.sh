# DDP (RCCL, world size 1) step time against the plain step, per DDP option set
set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ddpab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/plain.log 2>&1
echo "plain: $(tail -1 $O/plain.log | cut -c90-140)"
i=0
for v in "CTN_DDP_VIEW=0 CTN_DDP_STATIC=0" "CTN_DDP_VIEW=1 CTN_DDP_STATIC=0" "CTN_DDP_VIEW=1 CTN_DDP_STATIC=1" "CTN_DDP_VIEW=1 CTN_DDP_STATIC=1 CTN_DDP_BUCKET_MB=100"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29600+i)) bench.py --ddp --no-cpu-baseline --steps 20 --warmup 5 > $O/ddp$i.log 2>&1
  echo "$v: $(tail -1 $O/ddp$i.log | cut -c90-140)"
done
