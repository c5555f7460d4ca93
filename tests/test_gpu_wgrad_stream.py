"""Parameter-gradient tails on a second stream (ConvTasNet.wgrad_stream,
ctn_tblock_backward_split): the same kernels on the same inputs, so every gradient is
bit-identical to the one-stream backward; and the cases where the split would be
observable (autograd.grad, accumulation into existing gradients, hooks) take the
one-stream path.  GPU only."""
import os
import sys

import pytest
import torch

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "conv-tasnet_amd"))

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(norm="gLN", causal=False):
    import conv_tasnet as ct
    torch.manual_seed(0)
    m = ct.ConvTasNet(64, 16, 64, 128, 3, 3, 2, 2, norm_type=norm, causal=causal).to(DEV)
    m.act_dtype = torch.bfloat16
    return m


def _grads(m, mix, src, split):
    import pit_criterion as pc
    m.wgrad_stream = split
    m.zero_grad(set_to_none=True)
    est = m(mix)
    loss = pc.cal_loss(src, est, torch.full((mix.shape[0],), mix.shape[1], device=DEV))[0]
    loss.backward()
    return [p.grad.detach().clone() for p in m.parameters()]


@pytest.mark.parametrize("norm,causal", [("gLN", False), ("cLN", True)])
def test_split_backward_bit_identical(norm, causal):
    m = _model(norm, causal)
    torch.manual_seed(1)
    mix = torch.randn(3, 4000, device=DEV)
    src = torch.randn(3, 2, 4000, device=DEV)
    ref = _grads(m, mix, src, False)
    for _ in range(3):   # repeated: the side stream's buffers are reused safely
        got = _grads(m, mix, src, True)
        for a, b in zip(ref, got):
            assert torch.equal(a, b)


def test_split_not_used_when_observable():
    """autograd.grad w.r.t. the parameters, accumulation into existing gradients and
    gradient hooks all see the same values as without the split."""
    import pit_criterion as pc
    m = _model()
    torch.manual_seed(2)
    mix = torch.randn(2, 4000, device=DEV)
    src = torch.randn(2, 2, 4000, device=DEV)
    lens = torch.full((2,), 4000, device=DEV)
    params = list(m.parameters())
    ref = _grads(m, mix, src, False)

    m.wgrad_stream = True
    m.zero_grad(set_to_none=True)
    loss = pc.cal_loss(src, m(mix), lens)[0]
    gs = torch.autograd.grad(loss, params)
    assert all(p.grad is None for p in params)
    for a, b in zip(ref, gs):
        assert torch.equal(a, b)

    # accumulation: a second backward adds to the first
    m.zero_grad(set_to_none=True)
    pc.cal_loss(src, m(mix), lens)[0].backward()
    pc.cal_loss(src, m(mix), lens)[0].backward()
    for a, p in zip(ref, params):
        assert torch.allclose(p.grad, 2 * a, rtol=1e-6, atol=1e-7)

    # a hook on one block weight sees the finished gradient
    m.zero_grad(set_to_none=True)
    w = next(m.separator.blocks()).net[0].weight
    seen = []
    h = w.register_hook(lambda g: seen.append(g.detach().clone()))
    pc.cal_loss(src, m(mix), lens)[0].backward()
    h.remove()
    idx = [i for i, p in enumerate(params) if p is w][0]
    assert len(seen) == 1 and torch.equal(seen[0], ref[idx])


def test_split_join_survives_a_failed_backward(monkeypatch):
    """A backward that raises after split blocks queued their end-of-backward join
    drops the callback; the next split backward must still queue (and run) its own
    join, so .grad is never read while the side stream may still write it."""
    import ctn_ops as ops
    import pit_criterion as pc
    m = _model()
    torch.manual_seed(3)
    mix = torch.randn(2, 4000, device=DEV)
    src = torch.randn(2, 2, 4000, device=DEV)
    lens = torch.full((2,), 4000, device=DEV)
    ref = _grads(m, mix, src, False)

    joins = []
    real_join = ops._join_wgrad
    monkeypatch.setattr(ops, "_join_wgrad", lambda *a: (joins.append(a), real_join(*a)))

    def boom(_):
        raise RuntimeError("injected failure after the blocks' backward")

    m.wgrad_stream = True
    m.zero_grad(set_to_none=True)
    # the hook on the first block's input fires after every block's backward has run
    blk0 = next(m.separator.blocks())
    fwd = blk0._forward_rows

    def hooked(x, *a):
        x.register_hook(boom)
        return fwd(x, *a)

    monkeypatch.setattr(blk0, "_forward_rows", hooked)
    with pytest.raises(RuntimeError, match="injected failure"):
        pc.cal_loss(src, m(mix), lens)[0].backward()
    monkeypatch.setattr(blk0, "_forward_rows", fwd)
    torch.cuda.synchronize()
    n0 = len(joins)                         # the engine drops a failed pass's callbacks

    got = _grads(m, mix, src, True)
    assert len(joins) == n0 + 1             # the next pass joins anyway
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
