"""DDP over the HIP modules (VERDICT r01 "What's missing" 3).

Two processes (world_size 2, gloo — the only backend two ranks can share on the
one-GPU box) each put the HIP ``ConvTasNet`` on cuda:0 inside
``DistributedDataParallel``, run forward / PIT loss / backward on their half of
the batch (DDP's bucket hooks all-reduce the C-ABI-produced gradients while the
remaining blocks' backward runs), then ``ctn_optim.clip_grad_norm_`` + ``Adam``
on the reduced gradients (train.py / bench.py's step, replacing
src/train.py:120-122's DataParallel).  Checked against the single-process
full-batch HIP step: averaged gradients equal the full-batch gradients (loss =
batch mean, equal shards), and both ranks end with identical parameters.
fp32 (tight) and bf16 with packed weights (the throughput mode).  The same with the
bench's default exchange, ctn_dist.FlatGradAllReduce (the TemporalBlock gradient
reductions deferred and run in groups during the backward pass, each group's slice of
the persistent buffer all-reduced while the backward goes on, the rest after it).
GPU only.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(N=64, L=20, B=64, H=128, P=3, X=2, R=2, C=2)
M, T = 4, 8000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _batch():
    import synthetic
    return synthetic.speech_like(M, CFG["C"], T, 21)


def _step(model, mix, src, bf16, sync=None):
    """forward -> cal_loss -> zero_grad -> backward [-> flat gradient all-reduce] ->
    clip(5) -> Adam (solver.py:178-186)."""
    import ctn_optim
    import pit_criterion as pc
    opt = ctn_optim.Adam(model.parameters(), lr=1e-3)
    lens = torch.full((mix.shape[0],), T, dtype=torch.int64, device=mix.device)
    inner = model.module if hasattr(model, "module") else model
    inner.act_dtype = torch.bfloat16 if bf16 else torch.float32
    est = model(mix)
    loss = pc.cal_loss(src, est, lens)[0]
    opt.zero_grad()
    loss.backward()
    if sync is not None:
        sync.sync()
    grads = [p.grad.detach().cpu().clone() for p in model.parameters()]
    ctn_optim.clip_grad_norm_(model.parameters(), 5.0)
    opt.step()
    torch.cuda.synchronize()
    return float(loss), grads, [p.detach().cpu().clone() for p in model.parameters()]


def _worker(rank, world, port, bf16, view, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import conv_tasnet as ct
        import ctn_dist
        import ctn_ops
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        model = ct.ConvTasNet(**CFG).to(dev)
        sync = None
        if view == "flat":
            # the bench's default: one flat all-reduce after backward, deferred reductions on
            sync = ctn_dist.FlatGradAllReduce(model.parameters())
            net = model
        else:
            # view: the bench / train.py options (gradients as bucket views, static graph)
            net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], bucket_cap_mb=0.1,
                                                            gradient_as_bucket_view=view, static_graph=view)
        mix, src = _batch()
        shard = slice(rank * (M // world), (rank + 1) * (M // world))
        if sync is not None:
            # one exchange before the measured step: the step's deferred blocks then write
            # into a persistent gradient buffer that already holds gradients
            import pit_criterion as pc
            model.act_dtype = torch.bfloat16 if bf16 else torch.float32
            lens = torch.full((M // world,), T, dtype=torch.int64, device=dev)
            pc.cal_loss(src[shard].to(dev), net(mix[shard].to(dev)), lens)[0].backward()
            sync.sync()
            model.zero_grad(set_to_none=True)
        n0 = ctn_ops.DEFERRED_BLOCKS
        loss, grads, params = _step(net, mix[shard].to(dev), src[shard].to(dev), bf16, sync)
        # deferral under torch.distributed only for the post-backward exchange
        assert (ctn_ops.DEFERRED_BLOCKS > n0) == (view == "flat"), ctn_ops.DEFERRED_BLOCKS - n0
        if sync is not None:   # chunked exchange: the early chunks went out during backward
            assert sync.early_chunks >= 2, sync.early_chunks
        q.put((rank, loss, [g.numpy() for g in grads], [p.numpy() for p in params]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("bf16,view", [(False, False), (True, False), (False, True), (False, "flat"),
                                       (True, "flat")])
def test_ddp_two_ranks_hip_model_matches_full_batch(bf16, view):
    import conv_tasnet as ct
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, bf16, view, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=300) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    # single-process full batch on the same GPU, same init
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = ct.ConvTasNet(**CFG).to(dev)
    mix, src = _batch()
    loss, grads, params = _step(model, mix.to(dev), src.to(dev), bf16)
    assert abs(0.5 * (res[0][1] + res[1][1]) - loss) < (1e-4 if not bf16 else 2e-2)
    tol = 1e-4 if not bf16 else 3e-2
    for (_, _, g_rank, p_rank) in res:
        for i, (a, b) in enumerate(zip(g_rank, grads)):
            b = b.numpy()
            if b.size == 1:   # PReLU alpha: cancellation-heavy scalar sum
                assert abs(float(a) - float(b)) < (1e-3 if not bf16 else 5e-2) * (1 + abs(float(b))), i
                continue
            e = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
            assert e < tol, (i, e)
    # the all-reduce leaves identical gradients, hence identical parameters, on both ranks
    for a, b in zip(res[0][2], res[1][2]):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(res[0][3], res[1][3]):
        np.testing.assert_array_equal(a, b)
