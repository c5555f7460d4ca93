"""Stand-alone module forwards on the HIP path (ctn_layers.hip, include/ctn.h ABI v4):
GlobalLayerNorm / ChannelwiseLayerNorm against the reference's own golden vectors
(tests/golden/ops.npz, captured from src/conv_tasnet.py:307-355), and
DepthwiseSeparableConv / TemporalConvNet against the fp32 CPU oracle (oracle/, test
infrastructure), forward and backward.  Tolerances: fp32 outputs 1e-5 relative L2,
gradients 1e-4 (1e-3 for the cancelling PReLU alpha sums); bf16 5e-2.  GPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ctn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("nm", ["gln", "cln"])
def test_layer_norm_modules_vs_reference_golden(nm):
    import conv_tasnet as ct
    z = np.load(os.path.join(GOLDEN, "ops.npz"))
    mod = (ct.GlobalLayerNorm if nm == "gln" else ct.ChannelwiseLayerNorm)(24).to(DEV)
    with torch.no_grad():
        mod.gamma.copy_(torch.from_numpy(z[f"{nm}.gamma"]))
        mod.beta.copy_(torch.from_numpy(z[f"{nm}.beta"]))
    y = torch.from_numpy(z[f"{nm}.y"]).to(DEV).requires_grad_(True)
    out = mod(y)
    (out * torch.from_numpy(z[f"{nm}.G"]).to(DEV)).sum().backward()
    assert rel(out.detach(), z[f"{nm}.out"]) < 1e-5
    assert rel(y.grad, z[f"{nm}.gy"]) < 1e-4
    assert rel(mod.gamma.grad, z[f"{nm}.ggamma"]) < 1e-4
    assert rel(mod.beta.grad, z[f"{nm}.gbeta"]) < 1e-4


def _randomize(mod, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in mod.parameters():
            p.copy_(0.3 * torch.randn(p.shape, generator=g) + (1.0 if p.dim() == 3 and p.shape[0] == 1 else 0.0))
    return mod


@pytest.mark.parametrize("norm,causal,dil", [("gLN", False, 1), ("gLN", False, 4), ("cLN", True, 2),
                                             ("cLN", False, 8), ("BN", True, 1)])
def test_depthwise_separable_conv_vs_oracle(norm, causal, dil):
    import conv_tasnet as ct
    C_in, C_out, P, M, K = 32, 16, 3, 2, 300
    pad = (P - 1) * dil if causal else (P - 1) * dil // 2
    mod = _randomize(ct.DepthwiseSeparableConv(C_in, C_out, P, 1, pad, dil, norm, causal), 5).to(DEV)
    x = torch.randn(M, C_in, K) * 1.5
    G = torch.randn(M, C_out, K)
    xg = x.to(DEV).requires_grad_(True)
    y = mod(xg)
    (y * G.to(DEV)).sum().backward()
    # oracle: the reference's layer sequence in fp32 on the CPU
    ps = {n: p.detach().cpu().clone().requires_grad_(True) for n, p in mod.named_parameters()}
    xc = x.clone().requires_grad_(True)
    net = [n for n in ps]
    dw_w = ps["net.0.weight"]
    off = 1 if causal else 0
    h = O.depthwise(xc, dw_w, dil, causal)
    h = O.prelu(h, ps[f"net.{1 + off}.weight"])
    if norm == "BN":
        h = O.bn(h, ps[f"net.{2 + off}.weight"], ps[f"net.{2 + off}.bias"])
    elif norm == "gLN":
        h = O.gln(h, ps[f"net.{2 + off}.gamma"], ps[f"net.{2 + off}.beta"])
    else:
        h = O.cln(h, ps[f"net.{2 + off}.gamma"], ps[f"net.{2 + off}.beta"])
    yr = torch.nn.functional.conv1d(h, ps[f"net.{3 + off}.weight"])
    (yr * G).sum().backward()
    assert rel(y.detach(), yr.detach()) < 1e-5
    assert rel(xg.grad, xc.grad) < 1e-4
    for n, p in mod.named_parameters():
        tol = 1e-3 if p.numel() == 1 else 1e-4
        assert rel(p.grad, ps[n].grad) < tol, n
    assert net


@pytest.mark.parametrize("norm,causal,mask", [("gLN", False, "relu"), ("cLN", True, "softmax")])
def test_temporal_conv_net_vs_oracle(norm, causal, mask):
    import conv_tasnet as ct
    N, B, H, P, X, R, C, M, K = 32, 16, 32, 3, 3, 2, 2, 2, 250
    tcn = _randomize(ct.TemporalConvNet(N, B, H, P, X, R, C, norm, causal, mask), 9).to(DEV)
    gen = torch.Generator().manual_seed(17)   # fixed inputs (the global RNG depends on test order)
    w = torch.rand(M, N, K, generator=gen) * 2
    G = torch.randn(M, C, N, K, generator=gen)
    wg = w.to(DEV).requires_grad_(True)
    est = tcn(wg)
    assert est.shape == (M, C, N, K)
    (est * G.to(DEV)).sum().backward()
    cfg = O.Cfg(N, 16, B, H, P, X, R, C, norm, causal, mask_nonlinear=mask)
    params = {"separator." + n: p.detach().cpu().clone().requires_grad_(True) for n, p in tcn.named_parameters()}
    wc = w.clone().requires_grad_(True)
    er = O.separator(cfg, wc, params)
    (er * G).sum().backward()
    assert rel(est.detach(), er.detach()) < 1e-4
    assert rel(wg.grad, wc.grad) < 2e-3
    errs = {n: rel(p.grad, params["separator." + n].grad) for n, p in tcn.named_parameters() if p.numel() > 1}
    bad = {n: e for n, e in errs.items() if e >= 2e-3}
    assert not bad, (bad, max(errs.values()))


def test_layers_bf16_close_to_fp32():
    import conv_tasnet as ct
    mod = _randomize(ct.DepthwiseSeparableConv(64, 32, 3, 1, 2, 2, "gLN", False), 3).to(DEV)
    x = torch.randn(3, 64, 500, device=DEV)
    y32 = mod(x)
    y16 = mod(x.to(torch.bfloat16))
    assert y16.dtype == torch.bfloat16
    assert rel(y16.float().detach(), y32.detach()) < 5e-2


def test_layer_padded_rows_stay_zero():
    import ctn_lib as L
    import ctn_ops as ops
    fr = ops.Frames.of(2, 100)
    x = ops.ncw_to_rows(torch.randn(2, 16, 100, device=DEV), fr, torch.float32)
    g = torch.rand(1, 16, 1, device=DEV) + 0.5
    b = torch.randn(1, 16, 1, device=DEV)
    for code in (L.NORM_GLN, L.NORM_CLN):
        y = ops.LayerNormFn.apply(x, fr, code, g, b)
        assert torch.count_nonzero(y.view(2, fr.Kp, 16)[:, 100:]) == 0
    y = ops.DepthwiseFn.apply(x, fr, (3, 4, True), torch.randn(16, 1, 3, device=DEV))
    assert torch.count_nonzero(y.view(2, fr.Kp, 16)[:, 100:]) == 0
