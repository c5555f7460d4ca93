"""TemporalBlock HIP path (ctn_tblock_forward/backward) vs the reference's
golden vectors and vs the CPU oracle.  GPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ctn_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _names(causal):
    off = 1 if causal else 0
    return ["net.0.weight", "net.1.weight", "net.2.gamma", "net.2.beta", "net.3.net.0.weight",
            f"net.3.net.{1 + off}.weight", f"net.3.net.{2 + off}.gamma", f"net.3.net.{2 + off}.beta",
            f"net.3.net.{3 + off}.weight"]


def run_block(x_ncw, params, P, dil, causal, norm, G_ncw, dtype=torch.float32):
    import ctn_ops as ops
    import ctn_lib as L
    M, B, K = x_ncw.shape
    H = params[0].shape[0]
    fr = ops.Frames.of(M, K)
    x = ops.ncw_to_rows(x_ncw.to(DEV), fr, dtype).requires_grad_(True)
    ps = [p.to(DEV).float().clone().requires_grad_(True) for p in params]
    cfg = (B, H, P, dil, causal, L.NORM_GLN if norm == "gLN" else L.NORM_CLN)
    y = ops.TBlockFn.apply(x, fr, cfg, None, None, *ps)
    y_ncw = ops.rows_to_ncw(y, fr, torch.float32)
    (y_ncw * G_ncw.to(DEV)).sum().backward()
    gx = ops.rows_to_ncw(x.grad, fr, torch.float32)
    return y_ncw.detach().cpu(), gx.detach().cpu(), [p.grad.detach().cpu() for p in ps], y, x


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


TB = [(n, c, d) for n in ("gLN", "cLN") for c in (0, 1) for d in (1, 2, 4, 8, 16, 32, 64, 128)]


@pytest.mark.parametrize("norm,causal,d", TB)
def test_tblock_golden_f32(norm, causal, d):
    g = np.load(os.path.join(GOLDEN, "tblock.npz"))
    tag = f"tb.{norm}.{causal}.{d}"
    names = _names(causal)
    params = [torch.from_numpy(g[tag + ".p:" + n]) for n in names]
    y, gx, gp, yrows, _ = run_block(torch.from_numpy(g[tag + ".x"]), params, 3, d, causal, norm,
                                    torch.from_numpy(g[tag + ".G"]))
    # tolerance: fp32 everywhere, different summation order than the reference
    np.testing.assert_allclose(y.numpy(), g[tag + ".out"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(gx.numpy(), g[tag + ".gx"], rtol=1e-4, atol=2e-4)
    for n, gg in zip(names, gp):
        ref = g[tag + ".g:" + n]
        scale = np.abs(ref).max() + 1e-6
        np.testing.assert_allclose(gg.numpy().reshape(ref.shape), ref, rtol=1e-3, atol=1e-4 * scale + 1e-5,
                                   err_msg=n)
    # padded rows stay zero
    fr_rows = yrows.view(1, -1, yrows.shape[1])
    assert torch.count_nonzero(fr_rows[:, 301:]) == 0


def _paper_block(seed, B=256, H=512, causal=False, norm="gLN"):
    rng = np.random.default_rng(seed)
    P = 3
    shapes = [(H, B, 1), (1,), (1, H, 1), (1, H, 1), (H, 1, P), (1,), (1, H, 1), (1, H, 1), (B, H, 1)]
    out = []
    for s in shapes:
        if s == (1,):
            out.append(torch.tensor([0.25 + 0.1 * rng.standard_normal()], dtype=torch.float32))
        else:
            out.append(torch.from_numpy((rng.standard_normal(s) * O.xavier_normal_std(s)).astype(np.float32)))
    return out


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 3e-2)])
@pytest.mark.parametrize("d,causal,norm", [(1, 0, "gLN"), (128, 0, "gLN"), (16, 1, "cLN")])
def test_tblock_paper_dims_vs_oracle(dtype, tol, d, causal, norm):
    """Paper dims (B=256, H=512), 2 utterances of K=3199 frames: multi-tile GEMMs,
    chunked weight-gradient GEMMs, all vs the fp32 CPU oracle."""
    torch.manual_seed(0)
    params = _paper_block(1, causal=bool(causal), norm=norm)
    M, B, K = 2, 256, 3199
    x = torch.randn(M, B, K)
    G = torch.randn(M, B, K)
    y, gx, gp, _, _ = run_block(x, params, 3, d, causal, norm, G, dtype)
    cfg = O.Cfg(4, 4, B, 512, 3, int(np.log2(d)) + 1, 1, 2, norm, bool(causal))
    xi = int(np.log2(d))
    names = [O.block_prefix(0, xi) + n for n in _names(causal)]
    pd = {n: p.clone().requires_grad_(True) for n, p in zip(names, params)}
    xr = x.clone().requires_grad_(True)
    yr = O.temporal_block(cfg, xr, pd, 0, xi)
    (yr * G).sum().backward()
    assert rel(y, yr.detach()) < tol
    assert rel(gx, xr.grad) < tol
    for n, gg in zip(names, gp):
        if dtype == torch.bfloat16 and pd[n].numel() == 1:
            # dL/d alpha = sum over M*K*H terms of dL/da * min(x, 0); the per-frame norm
            # backward makes it a heavily cancelling sum, so bf16-stored operands leave
            # O(1) relative noise in it.  Its fp32 parity is checked above (dtype=f32).
            continue
        assert rel(gg.reshape(pd[n].shape), pd[n].grad) < tol * 5, n


def test_weight_packs_match_per_call_conversion():
    """bf16 weight copies packed once per step (ctn_pack_weights) give bit-identical
    results to the per-call conversion, and refresh when the fp32 weight changes."""
    import ctn_lib as L
    import ctn_ops as ops
    torch.manual_seed(0)
    params = _paper_block(3)
    M, B, K = 2, 256, 700
    fr = ops.Frames.of(M, K)
    x = ops.ncw_to_rows(torch.randn(M, B, K, device=DEV), fr, torch.bfloat16)
    cfg = (B, 512, 3, 4, False, L.NORM_GLN)
    ps = [p.to(DEV).clone().requires_grad_(True) for p in params]
    packs = ops.WeightPacks()

    def run(pack):
        for p in ps:
            p.grad = None
        xx = x.clone().requires_grad_(True)
        y = ops.TBlockFn.apply(xx, fr, cfg, pack, None, *ps)
        y.float().square().sum().backward()
        return y.detach(), xx.grad.detach(), [p.grad.detach().clone() for p in ps]

    for step in range(2):
        ref = run(None)
        got = run(packs.get([(ps[0], ps[8])], x.device)[0])
        assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])
        for a, b in zip(ref[2], got[2]):
            assert torch.equal(a, b)
        with torch.no_grad():   # in-place update: the packed copy must refresh
            ps[0].mul_(0.5)
            ps[8].add_(0.01)


def _frag_order(w: np.ndarray) -> np.ndarray:
    """include/ctn.h ctn_weight_pack fragment order of W [O][I], restated with numpy:
    flat index ((g*2 + nb)*(I/32) + kb)*512 + lane*8 + e holds
    W[g*32 + ((lane&15)>>2)*8 + nb*4 + (lane&3)][kb*32 + (lane>>4)*8 + e]."""
    O, I = w.shape
    g, nb, kb, lane, e = np.meshgrid(np.arange(O // 32), np.arange(2), np.arange(I // 32), np.arange(64),
                                     np.arange(8), indexing="ij")
    n = g * 32 + ((lane & 15) >> 2) * 8 + nb * 4 + (lane & 3)
    k = kb * 32 + (lane >> 4) * 8 + e
    return w[n, k].reshape(-1)


@pytest.mark.parametrize("O,I", [(512, 256), (256, 512), (96, 160)])
def test_pack_weights_fragment_order(O, I):
    """ctn_pack_weights' fragment-order copies (and their transposes) hold exactly the
    permutation include/ctn.h documents, element for element, besides the row-major
    bf16 copy and transpose."""
    import ctn_lib as L
    torch.manual_seed(0)
    w = torch.randn(O, I, device=DEV)
    outs = [torch.full((O * I,), float("nan"), dtype=torch.bfloat16, device=DEV) for _ in range(4)]
    pk = (L.WeightPack * 1)(L.WeightPack(w.data_ptr(), O, I, *[t.data_ptr() for t in outs]))
    L.check(L.load().ctn_pack_weights(pk, 1, L.stream_handle(w.device)), "ctn_pack_weights")
    torch.cuda.synchronize()
    wb = w.to(torch.bfloat16).cpu()
    dst, dst_t, frag, frag_t = [t.cpu() for t in outs]
    assert torch.equal(dst.view(O, I), wb)
    assert torch.equal(dst_t.view(I, O), wb.t())
    wn = wb.float().numpy()
    assert np.array_equal(frag.float().numpy(), _frag_order(wn))
    assert np.array_equal(frag_t.float().numpy(), _frag_order(np.ascontiguousarray(wn.T)))


@pytest.mark.parametrize("d,causal,norm", [(2, 0, "gLN"), (32, 1, "gLN"), (2, 0, "cLN"), (32, 1, "cLN")])
def test_dual_gemm_matches_four_kernel_path(d, causal, norm, monkeypatch):
    """The dual GEMMs (row GEMM + weight gradient in one pass, ctn_gemm_dual.hip) give
    the same results as the separate row/column GEMM kernels on identical bf16
    operands: data gradients bit-identical up to the fp32 summation order of the
    statistics, weight gradients up to the row-chunk summation order."""
    torch.manual_seed(0)
    params = _paper_block(5, causal=bool(causal), norm=norm)
    M, B, K = 3, 256, 1000
    x = torch.randn(M, B, K)
    G = torch.randn(M, B, K)
    outs = []
    for flag in ("0", "3"):   # four-kernel path vs both dual pairs
        monkeypatch.setenv("CTN_GEMM_DUAL", flag)
        outs.append(run_block(x, params, 3, d, causal, norm, G, torch.bfloat16)[:3])
    (y0, gx0, gp0), (y1, gx1, gp1) = outs
    errs = {n: rel(a, b) for n, a, b in zip(_names(causal), gp1, gp0)}
    print(norm, causal, d, "gx", rel(gx1, gx0), errs)
    assert torch.equal(y0, y1)
    assert rel(gx1, gx0) < 2e-3
    for (n, e), a, b in zip(errs.items(), gp1, gp0):
        assert e < 5e-3 or (a.numel() == 1 and abs(float(a - b)) < 1e-2 * (1 + abs(float(b)))), (n, errs)


@pytest.mark.parametrize("d,causal,norm", [(2, 0, "gLN"), (32, 1, "gLN"), (1, 0, "gLN"), (4, 1, "cLN"),
                                           (64, 1, "cLN"), (2, 0, "cLN")])
def test_fused_norm1_backward_matches_separate_kernel(d, causal, norm, monkeypatch):
    """bf16 gLN / cLN: the norm-1/PReLU-1 backward applied inside the gx GEMM's
    operand stage (OP_NORM1_BWD, ctn_gemm_ws.hip; cLN with per-row statistics and
    means) gives the results of the separate norm1_bwd kernel: the same per-element
    arithmetic on the same bf16 inputs, so gx and dW1 agree up to fp32 rounding, and
    the PReLU-1 alpha gradient up to its summation order."""
    torch.manual_seed(1)
    params = _paper_block(5, causal=bool(causal), norm=norm)
    M, B, K = 3, 256, 1000
    x = torch.randn(M, B, K)
    G = torch.randn(M, B, K)
    monkeypatch.setenv("CTN_GEMM_DUAL", "1")
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("CTN_FUSE_N1", flag)
        outs.append(run_block(x, params, 3, d, causal, norm, G, torch.bfloat16)[:3])
    (y0, gx0, gp0), (y1, gx1, gp1) = outs
    errs = {n: rel(a, b) for n, a, b in zip(_names(causal), gp1, gp0)}
    print(norm, causal, d, "gx", rel(gx1, gx0), errs)
    assert torch.equal(y0, y1)
    assert rel(gx1, gx0) < 2e-3
    for (n, e), a, b in zip(errs.items(), gp1, gp0):
        assert e < 5e-3 or (a.numel() == 1 and abs(float(a - b)) < 1e-2 * (1 + abs(float(b)))), (n, errs)


@pytest.mark.parametrize("dual", ["0", "3"])
@pytest.mark.parametrize("d,causal,norm", [(2, 0, "gLN"), (32, 1, "cLN"), (2, 0, "cLN")])
def test_backward_bitwise_deterministic(d, causal, norm, dual, monkeypatch):
    """Every statistic and gradient partial is combined in a fixed order:
    repeated runs on identical inputs give bit-identical outputs and gradients."""
    monkeypatch.setenv("CTN_GEMM_DUAL", dual)
    torch.manual_seed(0)
    params = _paper_block(5, causal=bool(causal), norm=norm)
    M, B, K = 3, 256, 1000
    x = torch.randn(M, B, K)
    G = torch.randn(M, B, K)
    runs = [run_block(x, params, 3, d, causal, norm, G, torch.bfloat16)[:3] for _ in range(3)]
    ref = run_block(x, params, 3, d, causal, norm, G, torch.float32)[:3]
    y0, gx0, gp0 = runs[0]
    print("vs fp32:", "gx", rel(gx0, ref[1]), {n: rel(a, b) for n, a, b in zip(_names(causal), gp0, ref[2])})
    for y, gx, gp in runs[1:]:
        assert torch.equal(y0, y)
        assert torch.equal(gx0, gx), rel(gx, gx0)
        for n, a, b in zip(_names(causal), gp, gp0):
            assert torch.equal(a, b), (n, rel(a, b))
