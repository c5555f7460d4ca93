"""Wave-item depthwise kernels (ctn_dw_wave.hip) against the lane-group kernels (ctn_tcn.hip).

With H = 512 and P = 3 (every BASELINE.json configuration) the TemporalBlock's depthwise
forward and backward run the wave-item kernels by default; CTN_DW_WAVE=0 selects the
lane-group kernels, which the oracle tests of rounds 1-4 pinned.  Both walk the same comb
items with the same per-element arithmetic, so the block output, the data gradient and every
parameter gradient but the depthwise weight's are bit-identical; the depthwise weight's
gradient groups the same products by n1 row instead of by gd row, which
moves a few products across work items at segment edges: 1e-5 relative.  The cases cover
the bench dispatch (gLN, M=32, K=3199) at small and large dilations, ragged utterances
whose walks end in edge steps, causal gLN, and c4's causal cLN (statistics batches of 63
steps, parking, edge steps).  GPU only (reference: conv_tasnet.py:176,212-272,289).
"""
import pytest
import torch

from test_gpu_benchshape import _block_params, _hip_block

pytestmark = pytest.mark.gpu

WD = 4   # index of the depthwise weight in _block_params' order


def _diff(a, b):
    """Mismatch summary: NaN counts, max |difference| where both finite, first mismatch."""
    na, nb = int(torch.isnan(a).sum()), int(torch.isnan(b).sum())
    ok = torch.isfinite(a) & torch.isfinite(b)
    d = (a - b).abs()[ok]
    bad = (a != b).nonzero()
    return dict(nan=(na, nb), maxdiff=float(d.max()) if d.numel() else None,
                first=bad[0].tolist() if len(bad) else None, count=len(bad))


def _run(M, K, d, causal, norm, seed, monkeypatch, wave):
    if wave is None:
        monkeypatch.delenv("CTN_DW_WAVE", raising=False)
    else:
        monkeypatch.setenv("CTN_DW_WAVE", "1" if wave else "0")
    torch.manual_seed(seed)
    params = _block_params(41 + d, 256, 512)
    x = torch.randn(M, 256, K)
    G = torch.randn(M, 256, K)
    return _hip_block(x, G, params, d, causal, norm, torch.bfloat16, packed=True)


CASES = [
    (32, 3199, 1, 0, "gLN"),
    (32, 3199, 64, 0, "gLN"),
    (7, 3000, 4, 0, "gLN"),
    (5, 1000, 128, 0, "gLN"),
    (7, 3000, 2, 1, "gLN"),
    (3, 3199, 16, 1, "cLN"),
    (64, 7999, 1, 1, "cLN"),
    (4, 2000, 8, 0, "cLN"),
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("M,K,d,causal,norm", CASES)
def test_wave_item_depthwise_matches_lane_group(M, K, d, causal, norm, monkeypatch):
    y1, gx1, gp1 = _run(M, K, d, causal, norm, 3, monkeypatch, True)
    y0, gx0, gp0 = _run(M, K, d, causal, norm, 3, monkeypatch, False)
    assert torch.equal(y1, y0), _diff(y1, y0)
    assert torch.equal(gx1, gx0), _diff(gx1, gx0)
    for i, (a, b) in enumerate(zip(gp1, gp0)):
        if i == WD:
            r = float((a - b).norm() / b.norm())
            assert r < 1e-5, ("depthwise weight gradient", r)
        else:
            assert torch.equal(a, b), ("parameter gradient", i, _diff(a, b))


def test_wave_item_kernels_are_the_default(monkeypatch):
    """The default run (no CTN_DW_WAVE) launches the wave-item kernels: their results differ
    from the lane-group kernels' in the depthwise weight gradient's last bits only."""
    _, _, gp_def = _run(2, 1000, 4, 0, "gLN", 1, monkeypatch, None)
    _, _, gp1 = _run(2, 1000, 4, 0, "gLN", 1, monkeypatch, True)
    _, _, gp0 = _run(2, 1000, 4, 0, "gLN", 1, monkeypatch, False)
    assert torch.equal(gp_def[WD], gp1[WD])
    assert not torch.equal(gp1[WD], gp0[WD])
