"""Full-model, encoder/decoder and PIT-loss HIP paths vs the reference's golden
vectors (tests/golden, captured from jwr1995/Conv-TasNet) and the CPU oracle.
GPU only.  Tolerances: fp32 mode — 1e-4 relative on outputs, 2e-3 on
gradients (fp32 MFMA, different reduction order); bf16 mode — SI-SNRi within
0.1 dB of the reference (BASELINE.json north_star) and 5e-2 relative L2 on
the estimate."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ctn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def T(a, dev=DEV):
    return torch.from_numpy(np.array(a)).to(dev)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def cfg_of(g):
    N, L, B, H, P, X, R, C = [int(v) for v in g["cfg"]]
    return O.Cfg(N, L, B, H, P, X, R, C, str(g["cfg_norm"]), bool(int(g["cfg_causal"])), str(g["cfg_mask"]))


def build(cfg, g):
    import conv_tasnet as ct
    m = ct.ConvTasNet(cfg.N, cfg.L, cfg.B, cfg.H, cfg.P, cfg.X, cfg.R, cfg.C, norm_type=cfg.norm_type,
                      causal=cfg.causal, mask_nonlinear=cfg.mask_nonlinear)
    if "p:encoder.conv1d_U.weight" in g.files:
        sd = {n: torch.from_numpy(g["p:" + n]) for n, _ in O.param_shapes(cfg)}
    else:
        sd = O.init_params(cfg, int(g["seed"]))
    m.load_state_dict(sd, strict=False)
    return m.to(DEV)


def run(model, g, bf16=False):
    import pit_criterion as pc
    mix, src, lens = T(g["mix"]), T(g["src"]), T(g["len"])
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
        est = model(mix)
    loss, max_snr, est_m, reord = pc.cal_loss(src, est, lens)
    model.zero_grad()
    loss.backward()
    return est_m, loss, max_snr, reord


MODELS = ["model_c1.npz", "model_paper_short.npz", "model_causal_cln.npz", "model_3spk.npz",
          "model_softmax_pad.npz", "model_bn.npz", "model_5spk.npz", "model_9spk.npz"]


@pytest.mark.parametrize("name", MODELS)
def test_model_fp32_vs_reference(name):
    g = load(name)
    cfg = cfg_of(g)
    model = build(cfg, g)
    est, loss, max_snr, reord = run(model, g)
    scale = float(np.abs(g["est"]).max())
    np.testing.assert_allclose(est.detach().cpu().numpy(), g["est"], rtol=1e-3, atol=2e-4 * scale)
    assert rel(est.detach().cpu().numpy(), g["est"]) < 1e-4
    np.testing.assert_allclose(float(loss), float(g["loss"]), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(max_snr.detach().cpu().numpy(), g["max_snr"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(reord.cpu().numpy(), g["reord"], rtol=1e-3, atol=2e-4 * scale)
    params = dict(model.named_parameters())
    for n, shape in O.param_shapes(cfg):
        gr = params[n].grad.detach().cpu().reshape(-1).numpy()
        gn = float(g["gnorm:" + n])
        if shape == (1,):
            # PReLU alpha: one sum over M*K*H terms with heavy cancellation; the fp32
            # reduction order alone moves it by ~1e-4 absolute
            np.testing.assert_allclose(gr, g["ghead:" + n], rtol=2e-3, atol=1e-3, err_msg=n)
            continue
        np.testing.assert_allclose(np.linalg.norm(gr), gn, rtol=2e-3, atol=1e-6, err_msg=n)
        np.testing.assert_allclose(gr[:64], g["ghead:" + n], rtol=2e-3, atol=2e-3 * gn + 1e-7, err_msg=n)
        if "g:" + n in g.files:
            assert rel(gr, g["g:" + n].reshape(-1)) < 2e-3, n
    if cfg.C == 2:
        for b in range(est.shape[0]):
            l = int(g["len"][b])
            v = O.cal_sisnri(g["src"][b, :, :l], reord[b, :, :l].cpu().numpy(), g["mix"][b, :l])
            assert abs(v - g["sisnri"][b]) < 1e-3


@pytest.mark.parametrize("name", ["model_paper_short.npz", "model_c1.npz", "model_causal_cln.npz"])
def test_model_bf16_sisnri_within_0p1db(name):
    g = load(name)
    cfg = cfg_of(g)
    model = build(cfg, g)
    est, loss, max_snr, reord = run(model, g, bf16=True)
    assert rel(est.detach().cpu().numpy(), g["est"]) < 5e-2
    assert abs(float(loss) - float(g["loss"])) < 0.1
    for b in range(est.shape[0]):
        l = int(g["len"][b])
        v = O.cal_sisnri(g["src"][b, :, :l], reord[b, :, :l].cpu().numpy(), g["mix"][b, :l])
        assert abs(v - g["sisnri"][b]) < 0.1, (v, g["sisnri"][b])
    # bf16-mode weight gradients: measured 2-5 % relative L2 error vs fp32 on the paper
    # dims (bf16 activations through 32 residual blocks); checked as norm agreement, and
    # as full-tensor relative error where the fixture holds the full gradient
    params = dict(model.named_parameters())
    for n, shape in O.param_shapes(cfg):
        if len(shape) < 2:
            continue
        gr = params[n].grad.detach().cpu().reshape(-1).numpy()
        assert abs(np.linalg.norm(gr) / float(g["gnorm:" + n]) - 1) < 0.1, n
        if "g:" + n in g.files:
            assert rel(gr, g["g:" + n].reshape(-1)) < 0.1, n


def _bn_modules(model):
    """(oracle norm prefix, nn.BatchNorm1d) of every TemporalBlock norm."""
    out = []
    for r, rep in enumerate(model.separator.network[2]):
        for xi, blk in enumerate(rep):
            n1, n2 = blk._norms()
            off = 1 if blk._geo[4] else 0
            p = O.block_prefix(r, xi)
            out += [(p + "net.2.", n1), (p + f"net.3.net.{2 + off}.", n2)]
    return out


def test_bn_running_statistics_and_eval_mode():
    """BatchNorm1d blocks (norm_type "BN", conv_tasnet.py:302-303): a training-mode
    forward updates running_mean / running_var (momentum 0.1, unbiased variance) and
    num_batches_tracked as torch does; an eval-mode forward normalizes with them.
    Checked against the fp32 oracle run with nn.BatchNorm1d buffer semantics."""
    g = load("model_bn.npz")
    cfg = cfg_of(g)
    model = build(cfg, g)
    mix = T(g["mix"])
    with torch.no_grad():
        model(mix)                                    # training mode
    mods = _bn_modules(model)
    params = {n: torch.from_numpy(g["p:" + n]) for n, _ in O.param_shapes(cfg)}
    running = {p: (torch.zeros(m.num_features), torch.ones(m.num_features)) for p, m in mods}
    try:
        O.BN_RUNNING, O.BN_TRAINING = running, True
        O.model_forward(cfg, torch.from_numpy(g["mix"]), params)
        for p, m in mods:
            assert int(m.num_batches_tracked) == 1
            np.testing.assert_allclose(m.running_mean.cpu().numpy(), running[p][0].numpy(), rtol=1e-4, atol=1e-5,
                                       err_msg=p)
            np.testing.assert_allclose(m.running_var.cpu().numpy(), running[p][1].numpy(), rtol=1e-4, atol=1e-5,
                                       err_msg=p)
        model.eval()
        with torch.no_grad():
            est = model(mix)
        O.BN_TRAINING = False
        ref = O.model_forward(cfg, torch.from_numpy(g["mix"]), params)
    finally:
        O.BN_RUNNING, O.BN_TRAINING = None, True
    assert rel(est.cpu().numpy(), ref.numpy()) < 1e-4
    for p, m in mods:                                 # eval mode leaves the buffers alone
        assert int(m.num_batches_tracked) == 1


def test_bn_bf16_training_step():
    """bf16 activations through the BN path against the REFERENCE's gradients
    (model_bn.npz, BatchNorm1d in training mode): the estimate within 5e-2 relative L2,
    and every parameter gradient tensor on its own (a permuted or misplaced gradient of
    equal norm must fail).  Training-mode BatchNorm subtracts the batch mean of its
    gradient, so some tensors are small differences of large terms and bf16 storage moves
    them by the noise of their terms, not of their value (measured on MI355X):
      * weight matrices: relative L2 < 0.15 (measured up to 0.107);
      * gamma / beta vectors: relative L2 < 0.5 (measured up to 0.35; the BN gammas after
        PReLU have gradients ~100x smaller than their neighbours': 0.012-0.026);
      * PReLU alphas (one sum over every position): |error| < 0.3 x the mean |gradient| of
        all alphas, 1.56 (measured up to 0.219 x, first block; 0.054 x on an alpha whose
        gradient is 0.087).
    Plus the whole gradient vector's cosine against the reference > 0.99.  The fp32 run of
    the same model (test_model_fp32_vs_reference) pins every tensor at 2e-3: the bounds
    here are bf16 storage, not the BN arithmetic."""
    g = load("model_bn.npz")
    cfg = cfg_of(g)
    model = build(cfg, g)
    est, loss, max_snr, reord = run(model, g, bf16=True)
    assert rel(est.detach().cpu().numpy(), g["est"]) < 5e-2
    params = dict(model.named_parameters())
    names = [(n, shape) for n, shape in O.param_shapes(cfg)]
    got = {n: params[n].grad.detach().cpu().reshape(-1).numpy().astype(np.float64) for n, _ in names}
    ref = {n: g["g:" + n].reshape(-1).astype(np.float64) for n, _ in names}
    alphas = [n for n, shape in names if int(np.prod(shape)) == 1]
    alpha_scale = float(np.mean([abs(ref[n][0]) for n in alphas])) if alphas else 1.0
    errs, bad = {}, []
    for n, shape in names:
        assert np.isfinite(got[n]).all(), n
        if n in alphas:
            e = abs(got[n][0] - ref[n][0]) / alpha_scale
            lim = 0.3
        else:
            e = rel(got[n], ref[n])
            lim = 0.5 if sum(d > 1 for d in shape) <= 1 else 0.15
        errs[n] = e
        if e >= lim:
            bad.append((n, e, lim))
    print("worst per-tensor gradient errors", sorted(errs.items(), key=lambda kv: -kv[1])[:8])
    assert not bad, bad
    a = np.concatenate([got[n] for n, _ in names])
    b = np.concatenate([ref[n] for n, _ in names])
    assert float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b))) > 0.99


@pytest.mark.parametrize("L_", [20, 16])
def test_encoder_standalone(L_):
    import conv_tasnet as ct
    g = load("ops.npz")
    enc = ct.Encoder(L_, 32).to(DEV)
    enc.conv1d_U.weight.data.copy_(T(g[f"enc{L_}.U"]))
    out = enc(T(g[f"enc{L_}.x"]))
    (out * T(g[f"enc{L_}.G"])).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), g[f"enc{L_}.out"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(enc.conv1d_U.weight.grad.cpu().numpy(), g[f"enc{L_}.gU"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("L_", [20, 16])
def test_decoder_standalone(L_):
    import conv_tasnet as ct
    g = load("ops.npz")
    dec = ct.Decoder(32, L_).to(DEV)
    dec.basis_signals.weight.data.copy_(T(g[f"dec{L_}.V"]))
    w = T(g[f"dec{L_}.w"]).requires_grad_(True)
    m = T(g[f"dec{L_}.m"]).requires_grad_(True)
    out = dec(w, m)
    (out * T(g[f"dec{L_}.G"])).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), g[f"dec{L_}.out"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(w.grad.cpu().numpy(), g[f"dec{L_}.gw"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(m.grad.cpu().numpy(), g[f"dec{L_}.gm"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(dec.basis_signals.weight.grad.cpu().numpy(), g[f"dec{L_}.gV"], rtol=1e-4,
                               atol=1e-3)


@pytest.mark.parametrize("C", [2, 3, 5, 6, 8])
@pytest.mark.parametrize("tag", ["eq", "neq"])
def test_pit_loss(C, tag):
    """C <= 3: pit.npz; C = 5, 6, 8 (C! up to 40,320 permutations, the device-decoded
    wide path): pit_wide.npz (tests/golden/make_golden_wide.py)."""
    import pit_criterion as pc
    g = load("pit.npz" if C <= 3 else "pit_wide.npz")
    k = f"pit.C{C}.{tag}"
    est0 = T(g[k + ".est"]).requires_grad_(True)
    est = est0 * 1.0
    loss, max_snr, est_m, reord = pc.cal_loss(T(g[k + ".src"]), est, T(g[k + ".len"]))
    assert est_m is est                                    # masked in place, same object (pit_criterion.py:24)
    loss.backward()
    np.testing.assert_allclose(float(loss), float(g[k + ".loss"]), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(max_snr.detach().cpu().numpy(), g[k + ".max_snr"], rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(est_m.detach().cpu().numpy(), g[k + ".est_m"])
    np.testing.assert_array_equal(reord.cpu().numpy(), g[k + ".reord"])
    np.testing.assert_allclose(est0.grad.cpu().numpy(), g[k + ".gest"], rtol=1e-3, atol=1e-7)
