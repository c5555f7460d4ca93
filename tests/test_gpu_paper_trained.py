"""Separating paper-config parity at the north-star tolerance (BASELINE.json): the
bench workload's shape (32 utterances x 4 s @ 8 kHz, paper config N=256 L=20 B=256
H=512 P=3 X=8 R=4 gLN) through the HIP path with weights trained until the model
separates (tests/golden/make_golden_paper_trained.py; reference SI-SNRi per utterance
from jwr1995/Conv-TasNet's own cal_SISNRi).  bf16 activations: every utterance's
SI-SNRi within 0.1 dB of the reference's; fp32 mode within 0.01 dB.

The c4 fixture (model_c4_trained.npz) does the same for the causal cLN variant (L=16)
at c4's per-GPU dispatch: 64 utterances of 4 s @ 16 kHz (K=7999 frames, M=64)."""
import numpy as np
import pytest
import torch

import paper_fixture as PF
from oracle import ctn_oracle as O

pytestmark = [pytest.mark.gpu]
need_c2 = pytest.mark.skipif(not PF.available(), reason="model_paper_trained.npz not generated")
need_c4 = pytest.mark.skipif(not PF.available(PF.PATH_C4), reason="model_c4_trained.npz not generated")


def _sisnri(dtype, path=PF.PATH, c=PF.CFG):
    import conv_tasnet as ct
    import pit_criterion as pc
    params, mix, src, g = PF.load(path, c)
    model = ct.ConvTasNet(c.N, c.L, c.B, c.H, c.P, c.X, c.R, c.C, norm_type=c.norm_type, causal=c.causal).cuda()
    model.load_state_dict(params)
    model.act_dtype = dtype
    lens = torch.full((mix.shape[0],), mix.shape[1], dtype=torch.int64, device="cuda")
    with torch.no_grad():
        est = model(mix.cuda())
        loss, max_snr, est_m, reord = pc.cal_loss(src.cuda(), est, lens)
    reord = reord.cpu().numpy()
    got = np.array([O.cal_sisnri(src[b].numpy(), reord[b], mix[b].numpy()) for b in range(mix.shape[0])])
    return got, g, float(loss)


@need_c2
def test_paper_trained_bf16_sisnri_within_0p1db():
    got, g, loss = _sisnri(torch.bfloat16)
    ref = g["sisnri"]
    assert ref.mean() > 3.0, "fixture model should separate"
    d = np.abs(got - ref)
    assert d.max() < 0.1, (d.max(), int(d.argmax()), got[d.argmax()], ref[d.argmax()])
    assert abs(loss - float(g["loss"])) < 0.1


@need_c2
def test_paper_trained_fp32_sisnri_within_0p01db():
    got, g, loss = _sisnri(torch.float32)
    d = np.abs(got - g["sisnri"])
    assert d.max() < 0.01, d.max()
    assert abs(loss - float(g["loss"])) < 1e-3


@need_c4
def test_c4_trained_bf16_sisnri_within_0p1db():
    got, g, loss = _sisnri(torch.bfloat16, PF.PATH_C4, PF.CFG_C4)
    ref = g["sisnri"]
    assert ref.mean() > 3.0, "fixture model should separate"
    d = np.abs(got - ref)
    assert d.max() < 0.1, (d.max(), int(d.argmax()), got[d.argmax()], ref[d.argmax()])
    assert abs(loss - float(g["loss"])) < 0.1


@need_c4
def test_c4_trained_fp32_sisnri_within_0p01db():
    got, g, loss = _sisnri(torch.float32, PF.PATH_C4, PF.CFG_C4)
    d = np.abs(got - g["sisnri"])
    assert d.max() < 0.01, d.max()
    assert abs(loss - float(g["loss"])) < 1e-3


@need_c2
@pytest.mark.timeout(900)
def test_paper_trained_bf16_backward_at_bench_dispatch():
    """Backward with SEPARATING weights at the c2 dispatch: the PIT
    loss of three utterances {0, 16, 31} of the fixture's 32-utterance batch, run through
    the whole M=32 bf16 forward/backward (gLN, the 1x1 convs and the depthwise conv act
    per utterance, so the weight gradients are those three utterances' alone).
      (1) dispatch: against the same three utterances run alone (M=3) through the same
          bf16 path, every gradient tensor within 0.15 relative L2 (gLN statistics group
          their partial sums by the grid, see below);
      (2) values: against the fp32 oracle's gradients of the three utterances, per tensor
          (the bounds of test_gpu_benchshape.py::_check_grads_bf16).  Measured on MI355X
          (round 6; the HIP path is bitwise reproducible): loss -3.23927 against the
          oracle's -3.23924; worst weight 0.0865 relative L2 (deep-block W1 / W2 of a
          converged model, whose gradients are small against their per-frame terms),
          gamma/beta 0.069, alphas 0.072 x the mean |alpha gradient|."""
    import conv_tasnet as ct
    import pit_criterion as pc
    from test_gpu_benchshape import _check_grads_bf16, rel
    c = PF.CFG
    params, mix, src, g = PF.load()
    sel = [0, mix.shape[0] // 2, mix.shape[0] - 1]

    def hip_grads(mx, sr, pick):
        model = ct.ConvTasNet(c.N, c.L, c.B, c.H, c.P, c.X, c.R, c.C).cuda()
        model.load_state_dict(params)
        model.act_dtype = torch.bfloat16
        est = model(mx.cuda())[pick]
        lens = torch.full((len(sel),), mx.shape[1], dtype=torch.int64, device="cuda")
        loss = pc.cal_loss(sr.cuda(), est, lens)[0]
        model.zero_grad()
        loss.backward()
        return dict(model.named_parameters()), float(loss)

    p32, l32 = hip_grads(mix, src[sel], sel)
    p3, l3 = hip_grads(mix[sel], src[sel], list(range(len(sel))))
    shapes = dict(O.param_shapes(c))
    alphas = [n for n, shape in shapes.items() if shape == (1,)]
    g32 = {n: p32[n].grad.detach().cpu().double() for n in p32}
    g3 = {n: p3[n].grad.detach().cpu().double() for n in p3}
    # PReLU alphas: one sum over every position of a block's [M, H, K] tensor whose terms
    # cancel, so the summation order alone (the M=32 and M=3 grids partition the rows into
    # different workgroup partials) moves a small alpha gradient by a large fraction of
    # itself: bounded against the mean |alpha gradient| like the value check below
    a_scale = float(np.mean([abs(float(g32[n].reshape(-1)[0])) for n in alphas]))
    disp = {n: (abs(float(g32[n].reshape(-1)[0] - g3[n].reshape(-1)[0])) / a_scale if n in alphas
                else rel(g32[n], g3[n])) for n in g32}
    worst_w = sorted(((n, e) for n, e in disp.items() if n not in alphas), key=lambda kv: -kv[1])[:4]
    worst_a = sorted(((n, e) for n, e in disp.items() if n in alphas), key=lambda kv: -kv[1])[:4]
    print("M=32 vs M=3 (same bf16 path): weights/norms", worst_w, "alphas (x mean |g|)", worst_a,
          "losses", l32, l3)
    _, loss_r, _, grads_r = O.fwd_bwd(c, params, mix[sel], src[sel], torch.full((len(sel),), mix.shape[1]))
    print("loss bf16", l32, "oracle", loss_r)
    assert abs(l32 - loss_r) < 0.1
    _check_grads_bf16(c, p32, grads_r, w_lim=0.1, n_lim=0.25, a_lim=0.3)
    # gLN's utterance statistics are fp64 sums of per-workgroup partials whose grouping
    # follows the grid, so the two dispatches round a few float statistics differently;
    # bf16 storage through 32 trained blocks turns that into up to ~5% relative L2 in some
    # deep-block gradients (measured 0.050; alphas 0.068 x mean |g|, round 6) — the bound
    # catches a misplaced row range (O(1)), the value check above pins the numbers
    assert worst_w[0][1] < 0.15, worst_w
    assert worst_a[0][1] < 0.3, worst_a
