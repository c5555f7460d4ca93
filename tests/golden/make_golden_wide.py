"""Golden vectors for more than 4 speakers, captured from the REAL reference (build
container only; the same import shim as make_golden.py, whose helpers this reuses).

Run from the repo root:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_wide.py

pit_wide.npz   : cal_loss (pit_criterion.py:12-113) for C = 5, 6, 8 — C! = 120, 720,
                 40,320 permutations (pit_criterion.py:66) — equal and unequal lengths
pit_c9_10.npz  : the same at C = 9 and 10 (python tests/golden/make_golden_wide.py --c9)
model_9spk.npz : a full ConvTasNet forward + PIT loss + backward at C = 9 (small dims, --c9)
model_5spk.npz : a full ConvTasNet forward + PIT loss + backward at C = 5 (small dims)
"""
import numpy as np
import torch

import make_golden as mg
from oracle import ctn_oracle as O


def pit_wide_fixtures():
    rng = np.random.default_rng(310)
    out = {}
    for C, T in ((5, 1000), (6, 700), (8, 400)):
        for tag, lens in (("eq", [T, T]), ("neq", [T, T * 2 // 3])):
            src = rng.standard_normal((2, C, T)).astype(np.float32)
            for b, l in enumerate(lens):
                src[b, :, l:] = 0
            perm = [list(rng.permutation(C)) for _ in range(2)]
            est = np.stack([src[b, perm[b]] for b in range(2)]) * 0.8 + \
                0.5 * rng.standard_normal((2, C, T)).astype(np.float32) + 0.3
            s = torch.from_numpy(src)
            e = torch.from_numpy(est.astype(np.float32)).requires_grad_(True)
            e2 = e * 1.0
            lengths = torch.tensor(lens)
            loss, max_snr, est_m, reord = mg.ref_pit.cal_loss(s, e2, lengths)
            loss.backward()
            k = f"pit.C{C}.{tag}"
            out.update({k + ".src": s, k + ".est": e.detach(), k + ".len": lengths,
                        k + ".loss": loss.detach(), k + ".max_snr": max_snr.detach(),
                        k + ".est_m": est_m.detach(), k + ".reord": reord.detach(),
                        k + ".gest": e.grad, k + ".perm": np.array(perm)})
    mg.save("pit_wide.npz", **out)


def pit_c9_c10_fixtures():
    """pit_c9_10.npz: cal_loss at C = 9 and 10 (C! = 362,880 and 3,628,800 permutations,
    the reference's own one-hot enumeration: 1.45 GB at C = 10), equal and unequal
    lengths; beyond C = 10 the reference cannot build its table (tests/test_gpu_pit_wide.py
    checks the assignment path against scipy on the oracle's pairwise SI-SNR instead)."""
    rng = np.random.default_rng(911)
    out = {}
    for C, T in ((9, 300), (10, 240)):
        for tag, lens in (("eq", [T, T]), ("neq", [T, T * 2 // 3])):
            src = rng.standard_normal((2, C, T)).astype(np.float32)
            for b, l in enumerate(lens):
                src[b, :, l:] = 0
            perm = [list(rng.permutation(C)) for _ in range(2)]
            est = np.stack([src[b, perm[b]] for b in range(2)]) * 0.8 + \
                0.5 * rng.standard_normal((2, C, T)).astype(np.float32) + 0.3
            s = torch.from_numpy(src)
            e = torch.from_numpy(est.astype(np.float32)).requires_grad_(True)
            e2 = e * 1.0
            lengths = torch.tensor(lens)
            loss, max_snr, est_m, reord = mg.ref_pit.cal_loss(s, e2, lengths)
            loss.backward()
            _, _, idx = mg.ref_pit.cal_si_snr_with_pit(s, (e * 1.0).detach(), lengths)
            k = f"pit.C{C}.{tag}"
            out.update({k + ".src": s, k + ".est": e.detach(), k + ".len": lengths,
                        k + ".loss": loss.detach(), k + ".max_snr": max_snr.detach(),
                        k + ".est_m": est_m.detach(), k + ".reord": reord.detach(),
                        k + ".gest": e.grad, k + ".idx": idx, k + ".perm": np.array(perm)})
    mg.save("pit_c9_10.npz", **out)


if __name__ == "__main__":
    import sys
    torch.manual_seed(0)
    if "--c9" in sys.argv:   # only the round-5 fixtures (C = 9, 10 PIT; the C = 9 model)
        pit_c9_c10_fixtures()
        model_9spk()
        sys.exit(0)
    pit_wide_fixtures()
    pit_c9_c10_fixtures()
    mg.model_fixture("model_5spk.npz", O.Cfg(64, 20, 64, 128, 3, 2, 2, 5), 2, 4000, 6,
                     lens=[4000, 3300], full=True)
    model_9spk()


def model_9spk():
    """model_9spk.npz (round 5): the full model at C = 9 (mask and decoder kernels with 16
    speakers per row, PIT over 362,880 permutations), small dims"""
    mg.model_fixture("model_9spk.npz", O.Cfg(32, 20, 32, 64, 3, 2, 1, 9), 2, 2000, 8,
                     lens=[2000, 1500], full=True)
