"""Bit-for-bit reproducibility at the shapes the bench and c4 run (VERDICT r03 Next 1c).

A TemporalBlock forward + backward (every kernel of the block: weight-stationary GEMMs,
the wave-specialised dual GEMM, depthwise forward / backward, the slab reductions) is run
twice on identical inputs at the c2 bench dispatch (gLN, M=32, K=3199) and at c4's
(causal cLN, M=64, K=7999), bf16 with packed weights, and every output, data gradient
and parameter gradient must agree bitwise.  Every statistic and gradient partial is
combined in a fixed order, so any difference is a race or a hardware
hazard (the packed-FP32 op_sel hazard made the dual GEMM's norm-2
statistics differ run to run).  The same is checked for the dual GEMM alone against the
previous kernel (CTN_DUAL_WS=0) through the public block: C and dW2 are bit-identical by
construction, the norm-2 sums agree to summation order.  GPU only.
"""
import numpy as np
import pytest
import torch

from test_gpu_benchshape import _block_params, _hip_block

pytestmark = pytest.mark.gpu


def _run(M, K, d, causal, norm, seed):
    torch.manual_seed(seed)
    params = _block_params(31 + d, 256, 512)
    x = torch.randn(M, 256, K)
    G = torch.randn(M, 256, K)
    return _hip_block(x, G, params, d, causal, norm, torch.bfloat16, packed=True)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("M,K,d,causal,norm", [(32, 3199, 2, 0, "gLN"), (64, 7999, 16, 1, "cLN")])
def test_block_bitwise_reproducible_at_bench_shapes(M, K, d, causal, norm):
    a = _run(M, K, d, causal, norm, 5)
    b = _run(M, K, d, causal, norm, 5)
    assert torch.equal(a[0], b[0]), "block output"
    assert torch.equal(a[1], b[1]), "data gradient"
    for i, (ga, gb) in enumerate(zip(a[2], b[2])):
        assert torch.equal(ga, gb), ("parameter gradient", i, float((ga - gb).abs().max()))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("norm,causal", [("gLN", 0), ("cLN", 1)])
def test_wave_specialised_dual_matches_previous_kernel(norm, causal, monkeypatch):
    """The block backward with the wave-specialised pair-A dual GEMM (default) against
    the round-3 gemm_dual_kernel (CTN_DUAL_WS=0) at the bench dispatch: the same MFMA
    sequences and operand transforms, so the data gradient and dW2 agree to the rounding
    of the norm-2 sums' summation order (both deterministic)."""
    outs = []
    for v in ("1", "0"):
        monkeypatch.setenv("CTN_DUAL_WS", v)
        outs.append(_run(32, 3199, 4, causal, norm, 9))
    (y1, gx1, gp1), (y0, gx0, gp0) = outs
    assert torch.equal(y1, y0)
    e = float((gx1 - gx0).norm() / gx0.norm())
    assert e < 1e-3, e
    for i, (a, b) in enumerate(zip(gp1, gp0)):
        if b.numel() == 1:
            assert abs(float(a - b)) < 1e-2 * (1 + abs(float(b))), i
            continue
        r = float((a - b).norm() / max(float(b.norm()), 1e-30))
        assert r < 1e-3, (i, r)
