"""The wave-specialised column GEMM (ctn_dual_ws.hip, COLS mode: memory + column waves
only, plain bf16 operands, transposed partials; opt-in, CTN_COLS_WS=1) that can compute
the first 1x1 conv's weight gradient dW1 = gh1^T . x in the block backward, checked through the public 1x1
conv layer (ctn_conv1x1_backward: dW = gy^T . x, the same GemmCols shape C=256 -> 512):
against an fp32 matmul of the same bf16 operands, against the tiled column kernel
(CTN_COLS_WS=0), and run to run bitwise.  Padded frame rows contribute nothing.  GPU
only."""
import os
import sys

import pytest
import torch

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "conv-tasnet_amd"))

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _dw(x, gy, fr, cout):
    import ctn_ops as ops
    w = torch.nn.Parameter(torch.randn(cout, x.shape[1], 1, device=DEV) * 0.05)
    xr = x.clone().requires_grad_(True)
    y = ops.Conv1x1Fn.apply(xr, fr, w)
    y.backward(gy)
    torch.cuda.synchronize()
    return w.grad.detach().reshape(cout, -1).clone()


@pytest.mark.parametrize("M,K", [(4, 3199), (32, 3199), (3, 1000)])
def test_cols_ws_matches_fp32_and_tiled_kernel(M, K, monkeypatch):
    import ctn_ops as ops
    fr = ops.Frames.of(M, K)
    g = torch.Generator(device=DEV).manual_seed(M * 7 + K)
    x = torch.randn(fr.rows, 256, device=DEV, generator=g).to(torch.bfloat16)
    gy = torch.randn(fr.rows, 512, device=DEV, generator=g).to(torch.bfloat16)
    pad = torch.arange(fr.rows, device=DEV) % fr.Kp >= K      # padded frames are zero rows
    x[pad] = 0
    gy[pad] = 0
    ref = gy.float().t() @ x.float()                           # [512][256]
    monkeypatch.setenv("CTN_COLS_WS", "1")
    a = _dw(x, gy, fr, 512)
    b = _dw(x, gy, fr, 512)
    assert torch.equal(a, b), "run-to-run"
    e = float((a - ref).norm() / ref.norm())
    assert e < 1e-5, e
    monkeypatch.setenv("CTN_COLS_WS", "0")
    c = _dw(x, gy, fr, 512)
    e2 = float((a - c).norm() / c.norm())
    assert e2 < 1e-5, e2
