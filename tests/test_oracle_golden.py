"""Pin the CPU oracle (oracle/ctn_oracle.py) against vectors captured from the
real reference (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ctn_oracle as O


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def T(a):
    return torch.from_numpy(np.array(a))


def close(a, b, rtol=1e-5, atol=1e-5):
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def fwd_bwd(fn, inputs, G):
    ins = [x.clone().requires_grad_(True) for x in inputs]
    out = fn(*ins)
    (out * G).sum().backward()
    return out.detach(), [x.grad for x in ins]


@pytest.mark.parametrize("nm", ["gln", "cln"])
def test_norms(nm):
    g = load("ops.npz")
    fn = O.gln if nm == "gln" else O.cln
    out, (gy, gg, gb) = fwd_bwd(fn, [T(g[f"{nm}.y"]), T(g[f"{nm}.gamma"]), T(g[f"{nm}.beta"])],
                               T(g[f"{nm}.G"]))
    close(out, g[f"{nm}.out"])
    close(gy, g[f"{nm}.gy"], 1e-4, 1e-4)
    close(gg, g[f"{nm}.ggamma"], 1e-4, 1e-4)
    close(gb, g[f"{nm}.gbeta"], 1e-4, 1e-4)


@pytest.mark.parametrize("L", [20, 16])
def test_encoder(L):
    g = load("ops.npz")
    out, (_, gU) = fwd_bwd(O.encoder, [T(g[f"enc{L}.x"]), T(g[f"enc{L}.U"])], T(g[f"enc{L}.G"]))
    close(out, g[f"enc{L}.out"])
    close(gU, g[f"enc{L}.gU"], 1e-4, 1e-4)


def test_ola_known_answer():
    g = load("ops.npz")
    close(O.overlap_and_add(T(g["ola.kat.sig"]), 2), g["ola.kat.out"], 0, 0)
    for L, S in ((20, 10), (16, 8), (15, 7), (6, 3)):
        close(O.overlap_and_add(T(g[f"ola{L}_{S}.sig"]), S), g[f"ola{L}_{S}.out"])


@pytest.mark.parametrize("L", [20, 16])
def test_decoder(L):
    g = load("ops.npz")
    out, (gw, gm, gV) = fwd_bwd(lambda w, m, V: O.decoder(w, m, V, L),
                                [T(g[f"dec{L}.w"]), T(g[f"dec{L}.m"]), T(g[f"dec{L}.V"])],
                                T(g[f"dec{L}.G"]))
    close(out, g[f"dec{L}.out"], 1e-5, 1e-4)
    close(gw, g[f"dec{L}.gw"], 1e-4, 1e-4)
    close(gm, g[f"dec{L}.gm"], 1e-4, 1e-4)
    close(gV, g[f"dec{L}.gV"], 1e-4, 1e-3)


TB = [(n, c, d) for n in ("gLN", "cLN") for c in (0, 1) for d in (1, 2, 4, 8, 16, 32, 64, 128)]


@pytest.mark.parametrize("norm,causal,d", TB)
def test_temporal_block(norm, causal, d):
    g = load("tblock.npz")
    tag = f"tb.{norm}.{causal}.{d}"
    names = sorted(k[len(tag) + 3:] for k in g.files if k.startswith(tag + ".p:"))
    cfg = O.Cfg(4, 4, 8, 16, 3, 1, 1, 2, norm, bool(causal))
    # tblock_fixtures used a bare TemporalBlock; map its names onto block (0, xi)
    xi = int(np.log2(d))
    cfg = O.Cfg(4, 4, 8, 16, 3, xi + 1, 1, 2, norm, bool(causal))
    pre = O.block_prefix(0, xi)
    params = {pre + n: T(g[tag + ".p:" + n]).clone().requires_grad_(True) for n in names}
    x = T(g[tag + ".x"]).clone().requires_grad_(True)
    out = O.temporal_block(cfg, x, params, 0, xi)
    (out * T(g[tag + ".G"])).sum().backward()
    close(out, g[tag + ".out"], 1e-5, 1e-4)
    close(x.grad, g[tag + ".gx"], 1e-4, 1e-4)
    for n in names:
        close(params[pre + n].grad, g[tag + ".g:" + n], 1e-4, 2e-4)


@pytest.mark.parametrize("C", [2, 3, 5, 6, 8])
@pytest.mark.parametrize("tag", ["eq", "neq"])
def test_pit(C, tag):
    g = load("pit.npz" if C <= 3 else "pit_wide.npz")   # pit_wide: make_golden_wide.py
    k = f"pit.C{C}.{tag}"
    est = T(g[k + ".est"]).clone().requires_grad_(True)
    loss, max_snr, est_m, reord = O.cal_loss(T(g[k + ".src"]), est, T(g[k + ".len"]))
    loss.backward()
    close(loss, g[k + ".loss"], 1e-5, 1e-5)
    close(max_snr, g[k + ".max_snr"], 1e-5, 1e-5)
    close(est_m, g[k + ".est_m"], 0, 0)
    close(reord, g[k + ".reord"], 0, 0)
    close(est.grad, g[k + ".gest"], 1e-4, 1e-7)


@pytest.mark.parametrize("C", [9, 10])
@pytest.mark.parametrize("tag", ["eq", "neq"])
def test_pit_assign_vs_reference_c9_c10(C, tag):
    """The oracle's assignment form of the PIT maximum (si_snr_pit_assign, used to check
    C > 10 where the reference cannot enumerate C!) against the reference captured at
    C = 9, 10 (pit_c9_10.npz, make_golden_wide.py --c9): same maximum, same permutation
    rank, same reordered estimate."""
    g = load("pit_c9_10.npz")
    k = f"pit.C{C}.{tag}"
    max_snr, perm, rank, est_m = O.si_snr_pit_assign(T(g[k + ".src"]), T(g[k + ".est"]), T(g[k + ".len"]))
    close(max_snr, g[k + ".max_snr"], 1e-5, 1e-5)
    assert rank.tolist() == g[k + ".idx"].tolist()
    reord = torch.stack([est_m[b, perm[b]] for b in range(est_m.shape[0])])
    close(reord, g[k + ".reord"], 0, 0)


def test_pit_assign_equals_enumeration_small_c():
    """Assignment and the reference's enumeration (O.si_snr_pit) agree at C = 4..7 on random
    inputs: same maximum and the same permutation rank."""
    rng = np.random.default_rng(5)
    for C in range(4, 8):
        src = torch.from_numpy(rng.standard_normal((3, C, 200)).astype(np.float32))
        est = src[:, torch.from_numpy(rng.permutation(C))] * 0.7 + \
            torch.from_numpy(rng.standard_normal((3, C, 200)).astype(np.float32)) * 0.6
        lens = torch.tensor([200, 150, 90])
        m1, _, idx, _ = O.si_snr_pit(src, est, lens)
        m2, _, rank, _ = O.si_snr_pit_assign(src, est, lens)
        close(m2, m1, 1e-6, 1e-6)
        assert rank.tolist() == idx.tolist()


def test_sisnr():
    g = load("sisnr.npz")
    for c in range(2):
        close(O.cal_sisnr(g["ref"][c], g["est"][c]), g["sisnr"][c], 1e-10, 1e-10)
    close(O.cal_sisnri(g["ref"], g["est"], g["mix"]), g["sisnri"], 1e-10, 1e-10)


def cfg_of(g):
    N, L, B, H, P, X, R, C = [int(v) for v in g["cfg"]]
    return O.Cfg(N, L, B, H, P, X, R, C, str(g["cfg_norm"]), bool(int(g["cfg_causal"])),
                 str(g["cfg_mask"]))


def model_params(g, cfg):
    if "p:encoder.conv1d_U.weight" in g.files:
        return {n: T(g["p:" + n]) for n, _ in O.param_shapes(cfg)}
    return O.init_params(cfg, int(g["seed"]))


MODELS = ["model_c1.npz", "model_paper_short.npz", "model_causal_cln.npz", "model_3spk.npz",
          "model_softmax_pad.npz", "model_bn.npz", "model_5spk.npz", "model_9spk.npz"]


@pytest.mark.parametrize("name", MODELS)
def test_model(name):
    g = load(name)
    cfg = cfg_of(g)
    params = model_params(g, cfg)
    est, loss, max_snr, grads = O.fwd_bwd(cfg, params, T(g["mix"]), T(g["src"]), T(g["len"]))
    scale = float(np.abs(g["est"]).max())
    close(est, g["est"], 1e-4, 1e-4 * scale)
    close(loss, g["loss"], 1e-4, 1e-4)
    close(max_snr, g["max_snr"], 1e-4, 1e-4)
    for n, _ in O.param_shapes(cfg):
        gn = float(g["gnorm:" + n])
        close(grads[n].norm(), gn, 2e-3, 1e-6)
        close(grads[n].reshape(-1)[:64], g["ghead:" + n], 2e-3, 2e-3 * gn + 1e-7)
        if "g:" + n in g.files:
            close(grads[n], g["g:" + n], 2e-3, 2e-3 * gn + 1e-7)


def test_model_sisnri_and_reorder():
    g = load("model_c1.npz")
    est, reord = g["est"], g["reord"]
    for b in range(est.shape[0]):
        v = O.cal_sisnri(g["src"][b], reord[b], g["mix"][b])
        close(v, g["sisnri"][b], 1e-6, 1e-6)


def test_train_step():
    g = load("model_c1.npz")
    cfg = cfg_of(g)
    params = model_params(g, cfg)
    _, after = O.train_step(cfg, params, T(g["mix"]), T(g["src"]), T(g["len"]))
    for n, _ in O.param_shapes(cfg):
        # Adam normalises g/sqrt(g^2): a 1e-3 step on near-zero grads is order-sensitive
        close(after[n], g["step:" + n], 1e-5, 2e-5)


def test_reference_init_semantics():
    """c1 was initialised by the reference itself: gamma/beta are xavier-normal
    (conv_tasnet.py:41-43 overwrites :316-317), PReLU alphas 0.25."""
    g = load("model_c1.npz")
    cfg = cfg_of(g)
    for n, shape in O.param_shapes(cfg):
        p = g["p:" + n]
        if len(shape) == 1:
            assert np.all(p == 0.25), n
        elif n.endswith("gamma"):
            assert not np.allclose(p, 1.0), n


def test_trained_model_fixture():
    """The oracle reproduces the reference's output and per-utterance SI-SNRi on the
    weights the reference trained (tests/golden/make_golden_trained.py)."""
    g = load("model_trained_c1.npz")
    N, L_, B, H, P, X, R, C = [int(v) for v in g["cfg"]]
    cfg = O.Cfg(N, L_, B, H, P, X, R, C)
    params = {n: T(g["p:" + n]) for n, _ in O.param_shapes(cfg)}
    with torch.no_grad():
        est = O.model_forward(cfg, T(g["mix"]), params)
        loss, _, est_m, reord = O.cal_loss(T(g["src"]), est, T(g["len"]))
    scale = float(np.abs(g["est"]).max())
    close(est_m, g["est"], 1e-4, 1e-5 * scale)
    close(float(loss), float(g["loss"]), 1e-5, 1e-5)
    for b in range(est.shape[0]):
        l = int(g["len"][b])
        v = O.cal_sisnri(g["src"][b, :, :l], reord[b, :, :l].numpy(), g["mix"][b, :l])
        assert abs(v - g["sisnri"][b]) < 1e-3


def test_paper_trained_fixture_oracle():
    """The oracle on the separating paper-config fixture (two of its utterances, to keep
    the CPU suite short): per-utterance SI-SNRi equal to the reference's."""
    import paper_fixture as PF
    if not PF.available():
        pytest.skip("model_paper_trained.npz not generated")
    params, mix, src, g = PF.load()
    for b in (0, 17):
        est = O.model_forward(PF.CFG, mix[b:b + 1], params)
        lens = torch.tensor([mix.shape[1]])
        _, _, _, reord = O.cal_loss(src[b:b + 1], est, lens)
        v = O.cal_sisnri(src[b].numpy(), reord[0].detach().numpy(), mix[b].numpy())
        assert abs(v - g["sisnri"][b]) < 1e-3, (b, v, g["sisnri"][b])
