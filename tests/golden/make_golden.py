"""Capture golden vectors from the REAL reference (build container only).

Run from the repo root:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports jwr1995/Conv-TasNet from /root/reference/src (read-only) with one
shim — ``torch.Tensor.cuda`` → identity — because ``src/utils.py:40`` calls
``.cuda()`` unconditionally.  ``evaluate.py`` imports librosa/mir_eval, which
are not installed, so they are stubbed in ``sys.modules`` (only ``cal_SISNR``/
``cal_SISNRi`` are called).  Nothing from the reference is written except
numeric inputs/outputs (``.npz``) and one serialized package produced by the
reference's own ``ConvTasNet.serialize`` (``package_tiny.pth``).

Recorded environment: torch version in every npz under key ``__torch__``.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference/src")
torch.Tensor.cuda = lambda self, *a, **k: self          # utils.py:40 shim
for _m in ("librosa", "mir_eval", "mir_eval.separation"):
    sys.modules.setdefault(_m, types.ModuleType(_m))
sys.modules["mir_eval.separation"].bss_eval_sources = None
sys.modules["mir_eval"].separation = sys.modules["mir_eval.separation"]

import conv_tasnet as ref_ct          # noqa: E402
import pit_criterion as ref_pit       # noqa: E402
import utils as ref_utils             # noqa: E402
import evaluate as ref_eval           # noqa: E402

from oracle import ctn_oracle as O    # noqa: E402  (only for init_params / names)

torch.set_num_threads(8)


def save(name, **arrs):
    arrs["__torch__"] = np.array(torch.__version__)
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: (v.detach().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in arrs.items()})
    print("wrote", path, os.path.getsize(path), "bytes")


def grads_of(module, inputs, G):
    """Backward of sum(out * G); returns out, grads of inputs and of named params."""
    for p in module.parameters():
        p.grad = None
    ins = [x.clone().requires_grad_(True) for x in inputs]
    out = module(*ins)
    (out * G).sum().backward()
    pg = {f"g:{n}": p.grad.clone() for n, p in module.named_parameters()}
    return out.detach(), [x.grad.clone() for x in ins], pg


def randomize_params(module, rng):
    with torch.no_grad():
        for n, p in module.named_parameters():
            if p.dim() == 1 and p.numel() == 1:      # PReLU: keep it away from 0.25 symmetric
                p.fill_(float(rng.uniform(0.05, 0.5)))
            else:
                p.copy_(torch.from_numpy(rng.standard_normal(p.shape).astype(np.float32)) * 0.3)


def ops_fixtures():
    rng = np.random.default_rng(100)
    out = {}
    # --- gLN / cLN (conv_tasnet.py:307-355) -------------------------------
    for nm, cls in (("gln", ref_ct.GlobalLayerNorm), ("cln", ref_ct.ChannelwiseLayerNorm)):
        mod = cls(24)
        randomize_params(mod, rng)
        y = torch.from_numpy((rng.standard_normal((2, 24, 37)) * 2 + 0.7).astype(np.float32))
        G = torch.from_numpy(rng.standard_normal((2, 24, 37)).astype(np.float32))
        o, (gy,), pg = grads_of(mod, [y], G)
        out.update({f"{nm}.y": y, f"{nm}.G": G, f"{nm}.out": o, f"{nm}.gy": gy,
                    f"{nm}.gamma": mod.gamma.detach(), f"{nm}.beta": mod.beta.detach(),
                    f"{nm}.ggamma": pg["g:gamma"], f"{nm}.gbeta": pg["g:beta"]})
    # --- Encoder (conv_tasnet.py:97-117) ------------------------------------
    for L in (20, 16):
        enc = ref_ct.Encoder(L, 32)
        randomize_params(enc, rng)
        x = torch.from_numpy(rng.standard_normal((2, 1001)).astype(np.float32))
        G = torch.from_numpy(rng.standard_normal((2, 32, (1001 - L) // (L // 2) + 1)).astype(np.float32))
        o, _, pg = grads_of(enc, [x], G)
        out.update({f"enc{L}.x": x, f"enc{L}.U": enc.conv1d_U.weight.detach(), f"enc{L}.out": o,
                    f"enc{L}.G": G, f"enc{L}.gU": pg["g:conv1d_U.weight"]})
    # --- overlap_and_add (utils.py:9-46) --------------------------------------
    sig = torch.tensor([[[[4., 1., 0., 2.], [3., 3., 1., 0.], [2., 4., 4., 1.]],
                         [[0., 1., 2., 3.], [4., 0., 1., 2.], [3., 4., 0., 1.]]],
                        [[[1., 1., 1., 1.], [2., 2., 2., 2.], [3., 3., 3., 3.]],
                         [[0., 0., 1., 1.], [1., 0., 1., 0.], [2., 2., 0., 0.]]]])
    out["ola.kat.sig"] = sig
    out["ola.kat.out"] = ref_utils.overlap_and_add(sig, 2)
    for L, S in ((20, 10), (16, 8), (15, 7), (6, 3)):
        s = torch.from_numpy(rng.standard_normal((2, 3, 11, L)).astype(np.float32))
        out[f"ola{L}_{S}.sig"] = s
        out[f"ola{L}_{S}.out"] = ref_utils.overlap_and_add(s, S)
    # --- Decoder (conv_tasnet.py:120-142) -------------------------------------
    for L in (20, 16):
        dec = ref_ct.Decoder(32, L)
        randomize_params(dec, rng)
        w = torch.from_numpy(np.abs(rng.standard_normal((2, 32, 50))).astype(np.float32))
        m = torch.from_numpy(np.abs(rng.standard_normal((2, 3, 32, 50))).astype(np.float32))
        G = torch.from_numpy(rng.standard_normal((2, 3, 49 * (L // 2) + L)).astype(np.float32))
        o, (gw, gm), pg = grads_of(dec, [w, m], G)
        out.update({f"dec{L}.w": w, f"dec{L}.m": m, f"dec{L}.V": dec.basis_signals.weight.detach(),
                    f"dec{L}.G": G, f"dec{L}.out": o, f"dec{L}.gw": gw, f"dec{L}.gm": gm,
                    f"dec{L}.gV": pg["g:basis_signals.weight"]})
    save("ops.npz", **out)


def tblock_fixtures():
    """TemporalBlock (conv_tasnet.py:212-238) over dilations, causal, gLN/cLN."""
    rng = np.random.default_rng(200)
    out = {}
    Bc, Hc, P, K = 8, 16, 3, 301
    for norm in ("gLN", "cLN"):
        for causal in (False, True):
            for d in (1, 2, 4, 8, 16, 32, 64, 128):
                pad = (P - 1) * d if causal else (P - 1) * d // 2
                blk = ref_ct.TemporalBlock(Bc, Hc, P, 1, pad, d, norm_type=norm, causal=causal)
                randomize_params(blk, rng)
                x = torch.from_numpy(rng.standard_normal((1, Bc, K)).astype(np.float32))
                G = torch.from_numpy(rng.standard_normal((1, Bc, K)).astype(np.float32))
                o, (gx,), pg = grads_of(blk, [x], G)
                tag = f"tb.{norm}.{int(causal)}.{d}"
                out[tag + ".x"], out[tag + ".G"], out[tag + ".out"], out[tag + ".gx"] = x, G, o, gx
                for n, p in blk.named_parameters():
                    out[tag + ".p:" + n] = p.detach().clone()
                    out[tag + ".g:" + n] = pg["g:" + n]
    save("tblock.npz", **out)


def pit_fixtures():
    """cal_loss (pit_criterion.py:12-113), C=2/3, equal and unequal lengths."""
    rng = np.random.default_rng(300)
    out = {}
    for C in (2, 3):
        for tag, lens in (("eq", [1000, 1000, 1000]), ("neq", [1000, 731, 402])):
            src = rng.standard_normal((3, C, 1000)).astype(np.float32)
            for b, l in enumerate(lens):
                src[b, :, l:] = 0
            mix = src.sum(1)
            # a deliberately permuted, noisy estimate so non-identity perms win
            perm = [list(rng.permutation(C)) for _ in range(3)]
            est = np.stack([src[b, perm[b]] for b in range(3)]) * 0.8 + \
                0.5 * rng.standard_normal((3, C, 1000)).astype(np.float32) + 0.3
            s = torch.from_numpy(src)
            e = torch.from_numpy(est.astype(np.float32)).requires_grad_(True)
            e2 = e * 1.0
            lengths = torch.tensor(lens)
            loss, max_snr, est_m, reord = ref_pit.cal_loss(s, e2, lengths)
            loss.backward()
            k = f"pit.C{C}.{tag}"
            out.update({k + ".src": s, k + ".est": e.detach(), k + ".len": lengths,
                        k + ".loss": loss.detach(), k + ".max_snr": max_snr.detach(),
                        k + ".est_m": est_m.detach(), k + ".reord": reord.detach(),
                        k + ".gest": e.grad, k + ".mix": mix})
    save("pit.npz", **out)


def build_ref_model(cfg, params=None, seed=None):
    m = ref_ct.ConvTasNet(cfg.N, cfg.L, cfg.B, cfg.H, cfg.P, cfg.X, cfg.R, cfg.C,
                          norm_type=cfg.norm_type, causal=cfg.causal,
                          mask_nonlinear=cfg.mask_nonlinear)
    if params is not None:
        missing, unexpected = m.load_state_dict(params, strict=False)
        assert not unexpected and all("running" in k or "num_batches" in k for k in missing), \
            (missing, unexpected)
    names = [n for n, _ in m.named_parameters()]
    assert names == [n for n, _ in O.param_shapes(cfg)], "param order mismatch"
    return m


def model_fixture(name, cfg, M, T, seed, lens=None, full=False, step=False, ref_init_seed=None):
    rng = np.random.default_rng(seed)
    if ref_init_seed is not None:
        torch.manual_seed(ref_init_seed)
        model = build_ref_model(cfg)             # reference init (conv_tasnet.py:41-43)
    else:
        model = build_ref_model(cfg, O.init_params(cfg, seed))
    mix, src = O.synth_batch(M, cfg.C, T, seed + 7)
    lengths = torch.tensor(lens if lens is not None else [T] * M)
    for b in range(M):
        mix[b, lengths[b]:] = 0
        src[b, :, lengths[b]:] = 0
    est = model(mix)
    loss, max_snr, est_m, reord = ref_pit.cal_loss(src, est, lengths)
    loss.backward()
    out = {"mix": mix, "src": src, "len": lengths, "est": est_m.detach(), "loss": loss.detach(),
           "max_snr": max_snr.detach(), "reord": reord.detach(),
           "cfg": np.array([cfg.N, cfg.L, cfg.B, cfg.H, cfg.P, cfg.X, cfg.R, cfg.C]),
           "cfg_norm": np.array(cfg.norm_type), "cfg_causal": np.array(int(cfg.causal)),
           "cfg_mask": np.array(cfg.mask_nonlinear), "seed": np.array(seed)}
    sisnri = [ref_eval.cal_SISNRi(src[b, :, :lengths[b]].numpy(), reord[b, :, :lengths[b]].detach().numpy(),
                                  mix[b, :lengths[b]].numpy()) for b in range(M)] if cfg.C == 2 else []
    out["sisnri"] = np.array(sisnri, dtype=np.float64)
    for n, p in model.named_parameters():
        g = p.grad.detach().reshape(-1)
        if full:
            out["p:" + n] = p.detach().clone()
            out["g:" + n] = p.grad.detach().clone()
        out["gnorm:" + n] = g.norm()
        out["ghead:" + n] = g[:64].clone()
    if step:
        torch.nn.utils.clip_grad_norm_(model.parameters(), 5.0)       # solver.py:184-185
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)           # train.py:130-132
        opt.step()
        for n, p in model.named_parameters():
            out["step:" + n] = p.detach().clone()
    save(name, **out)


def package_fixture():
    cfg = O.Cfg(8, 4, 6, 10, 3, 2, 1, 2)
    torch.manual_seed(5)
    model = build_ref_model(cfg)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    mix, src = O.synth_batch(2, 2, 64, 11)
    loss = ref_pit.cal_loss(src, model(mix), torch.tensor([64, 64]))[0]
    loss.backward()
    opt.step()
    pkg = ref_ct.ConvTasNet.serialize(model, opt, 3, tr_loss=torch.arange(4.), cv_loss=torch.arange(4.) + 1)
    torch.save(pkg, os.path.join(HERE, "package_tiny.pth"))
    y = model(mix)
    save("package_tiny.npz", mix=mix, est=y.detach())


def sisnr_fixtures():
    rng = np.random.default_rng(400)
    ref = rng.standard_normal((2, 900))
    est = ref[::-1] * 0.3 + ref * 0.7 + 0.2 * rng.standard_normal((2, 900))
    mix = ref.sum(0)
    save("sisnr.npz", ref=ref, est=est, mix=mix,
         sisnr=np.array([ref_eval.cal_SISNR(ref[0], est[0]), ref_eval.cal_SISNR(ref[1], est[1])]),
         sisnri=np.array(ref_eval.cal_SISNRi(ref, est, mix)))


if __name__ == "__main__":
    torch.manual_seed(0)
    ops_fixtures()
    tblock_fixtures()
    pit_fixtures()
    sisnr_fixtures()
    package_fixture()
    # c1: reference init (pins init semantics) + full grads + one Adam step
    model_fixture("model_c1.npz", O.Cfg(64, 20, 64, 128, 3, 2, 2, 2), 1, 32000, 0,
                  full=True, step=True, ref_init_seed=0)
    # paper dims, short T, two utterances
    model_fixture("model_paper_short.npz", O.Cfg(256, 20, 256, 512, 3, 8, 4, 2), 2, 4000, 1)
    # causal cLN, L=16 (16 kHz), half a second
    model_fixture("model_causal_cln.npz", O.Cfg(256, 16, 256, 512, 3, 8, 4, 2, "cLN", True), 1, 8000, 2)
    # 3 speakers, N=512
    model_fixture("model_3spk.npz", O.Cfg(512, 20, 256, 512, 3, 8, 4, 3), 1, 4000, 3)
    # softmax mask + padded (unequal) lengths, small dims, full grads
    model_fixture("model_softmax_pad.npz", O.Cfg(64, 20, 64, 128, 3, 2, 2, 2, "gLN", False, "softmax"),
                  2, 8000, 4, lens=[8000, 6500], full=True)
    # BatchNorm variant (train mode), small dims, full grads
    model_fixture("model_bn.npz", O.Cfg(64, 20, 64, 128, 3, 2, 2, 2, "BN"), 2, 4000, 5, full=True)
