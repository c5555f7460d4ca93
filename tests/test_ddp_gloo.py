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


def _chunk_worker(rank, world, port, mode, q):
    """The chunked exchange driven the way ctn_ops drives it during backward (pass start,
    deferred block writes into the views, on_reduced per group), on CPU tensors."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctn_dist
        import ctn_ops
        ps = [torch.nn.Parameter(torch.zeros(n)) for n in (4, 6, 3, 5, 2)]   # a b c d + e (never deferred)
        fa = ctn_dist.FlatGradAllReduce(ps, chunks=3)
        blocks = [[ps[0]], [ps[1]], [ps[2]], [ps[3]]]
        pos = {id(p): k for k, p in enumerate(ps)}

        def vals(step, k):   # this rank's local gradient of parameter k at a step
            return [torch.arange(p.numel(), dtype=torch.float32) * (k + 1) + 10.0 * rank + step for p in ps][k]

        def deferred_pass(step, order):
            for p in ps:
                p.grad = None                     # zero_grad(set_to_none=True)
            fa.on_pass_start()
            for grp in order:
                for p in grp:
                    v = ctn_ops._grad_buffer(p)   # the deferred block writes into its view
                    v.copy_(vals(step, pos[id(p)]))
                    p.grad = v
                fa.on_reduced(grp)
            ps[4].grad = vals(step, 4)            # an immediate gradient (encoder, decoder, ...)

        # step 0 learns the layout (rank 1 reports its blocks in another order in "mismatch")
        order0 = blocks if not (mode == "mismatch" and rank == 1) else [blocks[1], blocks[0]] + blocks[2:]
        deferred_pass(0, order0)
        try:
            fa.sync()
        except RuntimeError as e:
            q.put((rank, "raised", str(e)))
            return
        out = {"step0": [p.grad.clone().numpy() for p in ps]}
        deferred_pass(1, blocks)                  # learnt: two chunks go out during the pass
        early = fa.early_chunks
        fa.sync()
        out["step1"] = [p.grad.clone().numpy() for p in ps]
        out["early1"] = early
        # gradient accumulation: a second pass before sync() (AccumulateGrad adds in place)
        deferred_pass(2, blocks)
        fa.on_pass_start()
        for k, p in enumerate(ps):
            p.grad.add_(vals(3, k))
        fa.sync()
        out["step23"] = [p.grad.clone().numpy() for p in ps]
        out["early23"] = fa.early_chunks - early
        q.put((rank, "ok", out))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _run_chunks(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chunk_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(300)
def test_flat_exchange_chunks_overlap_and_accumulation():
    """Chunked exchange: chunks launched during the pass give the mean; two
    backward passes before one sync() give the mean of the summed local gradients (the
    early chunks of the first pass are dropped, their views still hold local values)."""
    res = _run_chunks("ok")
    mean = lambda step, k: sum(torch.arange([4, 6, 3, 5, 2][k], dtype=torch.float32) * (k + 1) + 10.0 * r + step
                               for r in range(2)) / 2
    for rank, status, out in res:
        assert status == "ok"
        assert out["early1"] == 2 and out["early23"] == 2   # pass A launched them, pass B dropped them
        for k in range(5):
            torch.testing.assert_close(torch.from_numpy(out["step0"][k]), mean(0, k))
            torch.testing.assert_close(torch.from_numpy(out["step1"][k]), mean(1, k))
            torch.testing.assert_close(torch.from_numpy(out["step23"][k]), mean(2, k) + mean(3, k))


@pytest.mark.timeout(300)
def test_flat_exchange_layout_mismatch_raises():
    """VERDICT r05 Next 7: ranks that learnt different chunk layouts raise on every rank
    (instead of issuing different all-reduce sequences and deadlocking)."""
    res = _run_chunks("mismatch")
    assert [r[1] for r in res] == ["raised", "raised"]
    assert all("different gradient-chunk layouts" in r[2] for r in res)
