"""Trained-model fixture from the REAL reference (build container only).

Run from the repo root:
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_trained.py

Trains jwr1995/Conv-TasNet's own ``ConvTasNet`` (c1 dims: N=64 L=20 B=64
H=128 P=3 X=2 R=2, gLN, relu mask) with its own ``cal_loss`` and the solver's
update (clip_grad_norm_(5) + Adam lr 1e-3, src/solver.py:178-186) on fresh
synthetic speech-like mixtures (oracle.synth_batch) for a few hundred steps,
so that the model actually separates: the bf16 SI-SNRi tolerance test
(±0.1 dB, BASELINE.json north_star) then compares a meaningful SI-SNRi
(1.5-4 dB on the held-out batch after 6000 steps) instead of the ~0 dB or
less of random weights.  Captures the trained
weights, a held-out batch, the reference's output on it and its per-utterance
SI-SNRi (reference ``evaluate.cal_SISNRi``).  Same import shims as
make_golden.py (``torch.Tensor.cuda`` → identity for src/utils.py:40;
librosa/mir_eval stubbed, only cal_SISNRi is called).
"""
import os
import sys
import time
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
import evaluate as ref_eval           # noqa: E402

from oracle import ctn_oracle as O    # noqa: E402  (synthetic data, names)

torch.set_num_threads(8)

STEPS = int(os.environ.get("TRAIN_STEPS", "6000"))
BATCH, T = 4, 8000


def main():
    cfg = O.Cfg(64, 20, 64, 128, 3, 2, 2, 2)
    torch.manual_seed(0)
    model = ref_ct.ConvTasNet(cfg.N, cfg.L, cfg.B, cfg.H, cfg.P, cfg.X, cfg.R, cfg.C)
    assert [n for n, _ in model.named_parameters()] == [n for n, _ in O.param_shapes(cfg)]
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    lens = torch.tensor([T] * BATCH)
    t0 = time.time()
    for step in range(STEPS):
        mix, src = O.synth_batch(BATCH, cfg.C, T, 10_000 + step)
        est = model(mix)
        loss = ref_pit.cal_loss(src, est, lens)[0]
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 5.0)
        opt.step()
        if step % 100 == 0 or step == STEPS - 1:
            print(f"step {step} loss {float(loss):.3f} ({time.time() - t0:.0f} s)", flush=True)
    model.eval()
    # held-out batch: two full-length utterances and one with a padded tail
    M, Te = 3, 16000
    mix, src = O.synth_batch(M, cfg.C, Te, 777)
    lengths = torch.tensor([Te, Te, 12000])
    mix[2, 12000:] = 0
    src[2, :, 12000:] = 0
    with torch.no_grad():
        est = model(mix)
        loss, max_snr, est_m, reord = ref_pit.cal_loss(src, est, lengths)
    sisnri = [ref_eval.cal_SISNRi(src[b, :, :lengths[b]].numpy(), reord[b, :, :lengths[b]].numpy(),
                                  mix[b, :lengths[b]].numpy()) for b in range(M)]
    print("held-out SI-SNRi (dB):", [round(float(v), 2) for v in sisnri])
    out = {"mix": mix, "src": src, "len": lengths, "est": est_m, "loss": loss, "max_snr": max_snr,
           "reord": reord, "sisnri": np.array(sisnri, dtype=np.float64),
           "cfg": np.array([cfg.N, cfg.L, cfg.B, cfg.H, cfg.P, cfg.X, cfg.R, cfg.C]),
           "cfg_norm": np.array(cfg.norm_type), "cfg_causal": np.array(int(cfg.causal)),
           "cfg_mask": np.array(cfg.mask_nonlinear), "seed": np.array(0), "train_steps": np.array(STEPS),
           "__torch__": np.array(torch.__version__)}
    for n, p in model.named_parameters():
        out["p:" + n] = p.detach().clone()
    path = os.path.join(HERE, "model_trained_c1.npz")
    np.savez_compressed(path, **{k: (v.detach().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in out.items()})
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
