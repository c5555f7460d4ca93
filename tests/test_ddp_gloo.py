"""Multi-process data parallelism on CPU (gloo, world_size 2): the DDP gradient
all-reduce over equal per-rank shards reproduces the single-process full-batch
gradient of the reference loss (loss = -mean over the batch,
DDP averages rank gradients), the bench's flat post-backward exchange
(ctn_dist.FlatGradAllReduce) gives DDP's gradients to the bit, and the bench's
max-over-ranks timing reduction.
The model here is the CPU oracle wrapped in an nn.Module — the HIP path runs the
same DDP wrapper on RCCL on the GPU box."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ctn_oracle as O

CFG = O.Cfg(N=16, L=8, B=8, H=16, P=3, X=2, R=1, C=2)


class OracleModel(torch.nn.Module):
    def __init__(self, params):
        super().__init__()
        self.names = [n for n, _ in O.param_shapes(CFG)]
        self.p = torch.nn.ParameterList([torch.nn.Parameter(params[n].clone()) for n in self.names])

    def forward(self, mix):
        return O.model_forward(CFG, mix, {n: p for n, p in zip(self.names, self.p)})


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import train
    torch.manual_seed(0)
    params = O.init_params(CFG, 7)
    mix, src = O.synth_batch(4, CFG.C, 400, 3)
    lens = torch.tensor([400, 400, 400, 400])
    shard = slice(rank * 2, rank * 2 + 2)
    model = torch.nn.parallel.DistributedDataParallel(OracleModel(params))
    est = model(mix[shard])
    loss = O.cal_loss(src[shard], est, lens[shard])[0]
    loss.backward()
    grads = [p.grad.clone() for p in model.module.p]
    # the bench's / train.py's exchange: one flat all-reduce after backward.  Rank 1 starts
    # from perturbed weights, which the constructor's broadcast from rank 0 replaces.
    plain = OracleModel(params)
    if rank == 1:
        with torch.no_grad():
            for p in plain.p:
                p.add_(1.0)
    net = train.FlatDP(plain)                # train.py's wrapper for world size > 1
    O.cal_loss(src[shard], net(mix[shard]), lens[shard])[0].backward()
    net.grad_sync.sync()                     # what solver.py runs after backward
    flat = [p.grad.clone() for p in plain.p]
    t = torch.tensor([0.1 * (rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)                  # bench.py timing reduction
    q.put((rank, [g.numpy() for g in grads], float(t), [g.numpy() for g in flat]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_ddp_two_ranks_match_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # full-batch reference in this process
    params = O.init_params(CFG, 7)
    mix, src = O.synth_batch(4, CFG.C, 400, 3)
    _, _, _, grads = O.fwd_bwd(CFG, params, mix, src, torch.tensor([400] * 4))
    for (_, g_rank, tmax, g_flat) in res:
        assert abs(tmax - 0.2) < 1e-12
        for n, gr in zip([n for n, _ in O.param_shapes(CFG)], g_rank):
            torch.testing.assert_close(torch.from_numpy(gr), grads[n], rtol=1e-4, atol=1e-6)
        for a, b in zip(g_rank, g_flat):     # the flat exchange averages exactly as DDP does
            assert (a == b).all()
    # both ranks hold identical gradients after the all-reduce
    for a, b in zip(res[0][1], res[1][1]):
        assert (a == b).all()


def test_grad_buffer_registry():
    """ctn_ops hands a deferred block backward the exchange's view of a parameter's
    gradient while the exchange (its owner) lives, fresh memory after."""
    import ctn_ops
    p = torch.nn.Parameter(torch.zeros(3, 4))
    q = torch.nn.Parameter(torch.zeros(5))
    buf = torch.empty(12)
    v = buf.view(3, 4)
    assert not ctn_ops._synced_after_backward(p)
    ctn_ops.register_synced_after_backward([p], [v])
    assert ctn_ops._synced_after_backward(p) and not ctn_ops._synced_after_backward(q)
    assert ctn_ops._grad_buffer(p) is v
    assert ctn_ops._grad_buffer(q).shape == (5,)
    del v, buf
    g = ctn_ops._grad_buffer(p)
    assert g.shape == (3, 4) and ctn_ops._synced_after_backward(p)


def _flat_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ctn_dist
    a = torch.nn.Parameter(torch.full((4,), float(rank)))     # broadcast: rank 0's zeros win
    b = torch.nn.Parameter(torch.zeros(2, 3))
    sync = ctn_dist.FlatGradAllReduce([a, b])
    for step in range(2):                                      # the buffer is reused
        a.grad = torch.full((4,), float(rank + 1 + step))
        b.grad = None if rank == 1 else torch.full((2, 3), 3.0 * rank)   # unused on rank 1
        sync.sync()
        # numpy, not tensors: a tensor travels as a shared-memory handle that vanishes if
        # this process exits before the parent unpickles it
        q.put((rank, step, a.detach().numpy().copy(), a.grad.numpy().copy(), b.grad.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_flat_exchange_mean_unused_and_reuse():
    """World size 3: the exchange averages (a non-power-of-two world), an unused parameter
    contributes zeros, the persistent buffer is reused across steps, and the constructor
    broadcasts rank 0's weights."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flat_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(6)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, step, a, ga, gb in res:
        a, ga, gb = torch.from_numpy(a), torch.from_numpy(ga), torch.from_numpy(gb)
        assert torch.equal(a, torch.zeros(4))
        torch.testing.assert_close(ga, torch.full((4,), (1 + 2 + 3) / 3 + step))
        torch.testing.assert_close(gb, torch.full((2, 3), (0.0 + 0.0 + 6.0) / 3))
