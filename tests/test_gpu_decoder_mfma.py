"""bf16 decoder on the matrix cores (ctn_codec.hip dec_fwd_mfma / dec_bwd_mfma, used for
N in {256, 512}; the MFMA encoder forward; the decoder and encoder basis gradients as
column GEMMs) against the VALU codec kernels and frame_outer (CTN_DEC_MFMA=0,
CTN_ENC_MFMA=0, CTN_DU_COLS=0, the same bf16 inputs) and against fp32 mode, through
the whole model forward and backward so the encoder, mask conv, nonlinearity, basis,
overlap-add and their gradients are all on the path (conv_tasnet.py:106-140,
utils.py:9-46).  The encoder forward runs fp32 matrix-core products on the VALU
kernel's operands (bit-identical output, tools/exp/enc_check.py); the decoder paths
round their operands (masked sources, decoder basis) to bf16 where the VALU path
multiplies in fp32, so the
tolerance is the bf16 one: estimate within 1e-2 relative L2 of the VALU path; estimate
and gradients no further from fp32 than the VALU path's (x1.5) or within 1e-2 / 3e-2
(PReLU alpha: 3e-2 absolute, a cancelling sum); padded samples
exactly zero.  GPU only."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _run(model, mix, G, mfma, monkeypatch):
    # the matrix-core paths together: the MFMA decoder (with dV as a column GEMM) and the
    # encoder's dU as a column GEMM; off = the VALU decoder and frame_outer for both
    monkeypatch.setenv("CTN_DEC_MFMA", "1" if mfma else "0")
    monkeypatch.setenv("CTN_DU_COLS", "1" if mfma else "0")
    monkeypatch.setenv("CTN_ENC_MFMA", "1" if mfma else "0")
    model.zero_grad(set_to_none=True)
    est = model(mix)
    (est * G).sum().backward()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    return est.detach().clone(), grads


@pytest.mark.parametrize("N,C,mask,L_", [(256, 2, "relu", 20), (256, 3, "softmax", 16), (512, 3, "softmax", 20),
                                         (512, 2, "relu", 16)])
def test_decoder_mfma_matches_valu_path(N, C, mask, L_, monkeypatch):
    import conv_tasnet as ct
    torch.manual_seed(0)
    model = ct.ConvTasNet(N, L_, 64, 128, 3, 2, 1, C, norm_type="gLN", causal=False, mask_nonlinear=mask).to(DEV)
    model.act_dtype = torch.bfloat16
    M, T = 3, 5003
    mix = torch.randn(M, T, device=DEV)
    G = torch.randn(M, C, T, device=DEV)
    e1, g1 = _run(model, mix, G, True, monkeypatch)
    e0, g0 = _run(model, mix, G, False, monkeypatch)
    model.act_dtype = torch.float32
    e32, g32 = _run(model, mix, G, True, monkeypatch)   # fp32 runs the VALU codec kernels either way
    assert e1.shape == (M, C, T)
    assert torch.isfinite(e1).all()
    assert rel(e1, e0) < 1e-2
    assert rel(e1, e32) < max(1.5 * rel(e0, e32), 1e-2)
    for n in g0:
        assert torch.isfinite(g1[n]).all(), n
        if g0[n].numel() == 1:   # PReLU alpha: a cancelling sum, bf16 noise is O(1e-2) absolute
            d_mf, d_va = abs(float(g1[n] - g32[n])), abs(float(g0[n] - g32[n]))
            assert d_mf < max(1.5 * d_va, 3e-2 * (1 + abs(float(g32[n])))), (n, d_mf, d_va)
        else:
            # both bf16 paths against fp32: the matrix-core path no further off than
            # the VALU path (x1.5) or within 3e-2 (the encoder basis gradient, a sum of
            # cancelling terms through the ReLU mask, moves by a few % between any two
            # bf16 roundings of the forward)
            e_mf, e_va = rel(g1[n], g32[n]), rel(g0[n], g32[n])
            assert e_mf < max(1.5 * e_va, 3e-2), (n, e_mf, e_va)


def test_decoder_mfma_padding_and_tail(monkeypatch):
    """Frames past K and samples past (K-1)S + L stay zero (the reference's F.pad)."""
    import conv_tasnet as ct
    torch.manual_seed(1)
    model = ct.ConvTasNet(256, 20, 64, 128, 3, 1, 1, 2, norm_type="gLN", causal=False).to(DEV)
    model.act_dtype = torch.bfloat16
    T = 4007   # (K-1)*10 + 20 = 4000 < T: the last 7 samples are padding
    mix = torch.randn(2, T, device=DEV)
    monkeypatch.setenv("CTN_DEC_MFMA", "1")
    with torch.no_grad():
        est = model(mix)
    K = (T - 20) // 10 + 1
    assert torch.count_nonzero(est[:, :, (K - 1) * 10 + 20:]) == 0
    assert torch.count_nonzero(est[:, :, :(K - 1) * 10 + 20]) > 0
