"""Parameter update (ctn_optim): clip_grad_norm_ + Adam on the HIP path against
torch.nn.utils.clip_grad_norm_ / torch.optim.Adam in plain PyTorch fp32 — the
calls the reference solver makes (src/solver.py:184-186, src/train.py:129-133).

CPU tests cover the chunk planner (host code) and argument validation; the GPU
tests compare numerics.  Tolerances: clipping and Adam are a few fp32
operations per element; the HIP path evaluates the same formulas with fused
multiply-adds and an fp64 norm reduction, so results agree to ~1e-6 relative
(the Adam update is compared after several steps)."""
import copy
import ctypes

import pytest
import torch


@pytest.fixture(scope="module")
def lib():
    import ctn_lib as L
    return L.load()


def _plan(lib, sizes, aligned=True):
    import ctn_lib as L
    base = 4096 if aligned else 4100
    segs = (L.OptSegment * len(sizes))(*[L.OptSegment(base, base, base, base, n) for n in sizes])
    n = lib.ctn_opt_plan(segs, len(sizes), None, 0)
    chunks = (L.OptChunk * max(n, 1))()
    assert lib.ctn_opt_plan(segs, len(sizes), chunks, n) == n
    return n, chunks


def test_plan_covers_every_element_once(lib):
    sizes = [1, 3, 8192, 8193, 20000, 0, 5]
    n, chunks = _plan(lib, sizes)
    cover = {i: 0 for i in range(len(sizes))}
    for c in chunks[:n]:
        ln = c.len & 0x7FFFFFFF
        assert not (c.len & 0x80000000)
        assert c.off % 8192 == 0 and 0 < ln <= 8192
        assert c.off + ln <= sizes[c.seg]
        cover[c.seg] += ln
    assert cover == {i: s for i, s in enumerate(sizes)}
    assert n == sum((s + 8191) // 8192 for s in sizes)


def test_plan_flags_unaligned_segments(lib):
    n, chunks = _plan(lib, [100], aligned=False)
    assert n == 1 and chunks[0].len & 0x80000000


def test_plan_rejects_bad_tables(lib):
    import ctn_lib as L
    segs = (L.OptSegment * 1)(L.OptSegment(None, None, None, None, 10))
    assert lib.ctn_opt_plan(segs, 1, None, 0) < 0
    assert "no grad" in lib.ctn_last_error().decode()
    hp = L.AdamHParams(1e-3, 0.9, 0.999, 1e-8, 0.0, 0)
    assert lib.ctn_adam_step(None, None, 0, ctypes.byref(hp), None) != 0


def test_cpu_tensors_raise():
    import ctn_lib as L
    import ctn_optim
    p = torch.nn.Parameter(torch.randn(4))
    p.grad = torch.randn(4)
    with pytest.raises(L.CtnLibraryError):
        ctn_optim.clip_grad_norm_([p], 1.0)
    with pytest.raises(L.CtnLibraryError):
        ctn_optim.Adam([p]).step()


def _params(dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(256, 512, 1), (512,), (1,), (3, 7), (512, 1, 3), (100003,), (8192,), (8193,)]
    return [torch.randn(s, generator=g).to(dev) for s in shapes]


def _grads(ps, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(p.shape, generator=g).to(p.device) * 0.3 for p in ps]


@pytest.mark.gpu
@pytest.mark.parametrize("max_norm", [5.0, 1e6])
def test_clip_matches_torch(max_norm):
    import ctn_optim
    dev = torch.device("cuda")
    ps = [torch.nn.Parameter(t) for t in _params(dev)]
    qs = [torch.nn.Parameter(t.clone()) for t in _params(dev)]
    for a, b, g in zip(ps, qs, _grads(ps, 1)):
        a.grad, b.grad = g.clone(), g.clone()
    n_ref = torch.nn.utils.clip_grad_norm_(qs, max_norm)
    n_hip = ctn_optim.clip_grad_norm_(ps, max_norm)
    torch.testing.assert_close(n_hip, n_ref, rtol=1e-6, atol=0)
    for a, b in zip(ps, qs):
        torch.testing.assert_close(a.grad, b.grad, rtol=2e-6, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("wd", [0.0, 1e-2])
def test_adam_matches_torch(wd):
    import ctn_optim
    dev = torch.device("cuda")
    ps = [torch.nn.Parameter(t) for t in _params(dev)]
    qs = [torch.nn.Parameter(t.clone()) for t in _params(dev)]
    o_hip = ctn_optim.Adam(ps, lr=1e-3, weight_decay=wd)
    o_ref = torch.optim.Adam(qs, lr=1e-3, weight_decay=wd, foreach=False)
    for step in range(5):
        for a, b, g in zip(ps, qs, _grads(ps, 10 + step)):
            a.grad, b.grad = g.clone(), g.clone()
        o_hip.step()
        o_ref.step()
    for a, b in zip(ps, qs):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    for a, b in zip(ps, qs):
        for k in ("exp_avg", "exp_avg_sq"):
            torch.testing.assert_close(o_hip.state[a][k], o_ref.state[b][k], rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
def test_adam_state_dict_round_trip_with_torch():
    """A torch Adam checkpoint (solver.py:116 optim_dict) continues identically here, and back."""
    import ctn_optim
    dev = torch.device("cuda")
    ps = [torch.nn.Parameter(t) for t in _params(dev)]
    qs = [torch.nn.Parameter(t.clone()) for t in _params(dev)]
    o_ref = torch.optim.Adam(qs, lr=2e-3, foreach=False)
    for step in range(2):
        for b, g in zip(qs, _grads(qs, 20 + step)):
            b.grad = g
        o_ref.step()
    with torch.no_grad():
        for a, b in zip(ps, qs):
            a.copy_(b)
    o_hip = ctn_optim.Adam(ps, lr=2e-3)
    o_hip.load_state_dict(copy.deepcopy(o_ref.state_dict()))   # as torch.save/torch.load would
    for step in range(3):
        for a, b, g in zip(ps, qs, _grads(ps, 30 + step)):
            a.grad, b.grad = g.clone(), g.clone()
        o_hip.step()
        o_ref.step()
    for a, b in zip(ps, qs):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    sd = o_hip.state_dict()
    assert float(sd["state"][0]["step"]) == 5.0
    o_back = torch.optim.Adam([torch.nn.Parameter(a.detach().clone()) for a in ps], lr=2e-3)
    o_back.load_state_dict(sd)
    assert float(o_back.state_dict()["state"][0]["step"]) == 5.0


@pytest.mark.gpu
def test_adam_plan_reused_across_steps():
    """Re-planning costs a synchronous upload: steady-state steps must hit the cache."""
    import ctn_optim
    dev = torch.device("cuda")
    ps = [torch.nn.Parameter(t) for t in _params(dev)]
    o = ctn_optim.Adam(ps)
    for step in range(4):
        o.zero_grad(set_to_none=False)
        for a, g in zip(ps, _grads(ps, step)):
            a.grad.copy_(g) if a.grad is not None else setattr(a, "grad", g)
        o.step()
    assert len(o._plans) == 1


@pytest.mark.gpu
def test_fast_paths_match_torch():
    """The host fast paths (same parameters, gradient pointers and sizes as the previous
    fully checked call: ctn_optim._clip_fast, Adam._fast_step) against torch's clip + Adam
    over steps with in-place gradients, then a step where one parameter has no gradient
    (full path again), then the state_dict step counts."""
    import ctn_optim
    dev = torch.device("cuda")
    ps = [torch.nn.Parameter(t) for t in _params(dev)]
    qs = [torch.nn.Parameter(t.clone()) for t in _params(dev)]
    o_hip = ctn_optim.Adam(ps, lr=1e-3)
    o_ref = torch.optim.Adam(qs, lr=1e-3, foreach=False)
    for a, b in zip(ps, qs):
        a.grad, b.grad = torch.zeros_like(a), torch.zeros_like(b)
    fast_steps = 0
    for step in range(6):
        for a, b, g in zip(ps, qs, _grads(ps, 40 + step)):
            a.grad.copy_(g)
            b.grad.copy_(g)
        n_hip = ctn_optim.clip_grad_norm_(ps, 1.0)
        n_ref = torch.nn.utils.clip_grad_norm_(qs, 1.0)
        torch.testing.assert_close(n_hip, n_ref, rtol=1e-6, atol=0)
        o_hip.step()
        o_ref.step()
        fast_steps += bool(o_hip._fast.get(0) and o_hip._fast[0][4])
    assert fast_steps >= 4
    ps[1].grad, qs[1].grad = None, None
    for a, b, g in zip(ps, qs, _grads(ps, 60)):
        if a.grad is not None:
            a.grad.copy_(g)
            b.grad.copy_(g)
    o_hip.step()
    o_ref.step()
    for a, b in zip(ps, qs):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    sd = o_hip.state_dict()
    assert [float(sd["state"][i]["step"]) for i in range(3)] == [7.0, 6.0, 7.0]


@pytest.mark.gpu
def test_fast_paths_with_fresh_gradients_each_step():
    """zero_grad(set_to_none=True) training: every step's gradients are new tensors at
    other addresses (a spacer allocation shifts them); the fast paths still apply (same
    sizes and alignments) with the pointer table rebuilt, and the updates equal torch's."""
    import ctn_optim
    dev = torch.device("cuda")
    ps = [torch.nn.Parameter(t) for t in _params(dev)]
    qs = [torch.nn.Parameter(t.clone()) for t in _params(dev)]
    o_hip = ctn_optim.Adam(ps, lr=1e-3)
    o_ref = torch.optim.Adam(qs, lr=1e-3, foreach=False)
    hits0 = dict(ctn_optim.FAST_STATS)
    keep = []
    for step in range(6):
        keep.append(torch.empty(1000 * (step + 1), device=dev))     # moves the next allocations
        for a, b, g in zip(ps, qs, _grads(ps, 80 + step)):
            a.grad, b.grad = g.clone(), g.clone()
        torch.testing.assert_close(ctn_optim.clip_grad_norm_(ps, 1.0), torch.nn.utils.clip_grad_norm_(qs, 1.0),
                                   rtol=1e-6, atol=0)
        o_hip.step()
        o_ref.step()
        for a, b in zip(ps, qs):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    assert ctn_optim.FAST_STATS["clip_hit"] - hits0["clip_hit"] >= 4
    assert ctn_optim.FAST_STATS["adam_hit"] - hits0["adam_hit"] >= 4
