"""Loader for the separating trained-weight fixtures made by
tests/golden/make_golden_paper_trained.py: model_paper_trained.npz (paper config, c2)
and model_c4_trained.npz (causal cLN, L=16, c4): dequantized weights and the
regenerated held-out batch, checked against the fixture's checksum."""
import os

import numpy as np
import torch

from conftest import GOLDEN
from oracle import ctn_oracle as O

CFG = O.Cfg(256, 20, 256, 512, 3, 8, 4, 2)
PATH = os.path.join(GOLDEN, "model_paper_trained.npz")
CFG_C4 = O.Cfg(256, 16, 256, 512, 3, 8, 4, 2, "cLN", True)
PATH_C4 = os.path.join(GOLDEN, "model_c4_trained.npz")


def available(path=PATH):
    return os.path.exists(path)


def load(path=PATH, cfg=CFG):
    import synthetic
    g = np.load(path)
    params = {}
    for n, _ in O.param_shapes(cfg):
        if "f:" + n in g.files:
            params[n] = torch.from_numpy(np.array(g["f:" + n]))
        else:
            q, s = g["q:" + n], g["s:" + n]
            w = q.astype(np.float32) * s[:, None]
            params[n] = torch.from_numpy(w)
    shapes = dict(O.param_shapes(cfg))
    params = {n: v.reshape(shapes[n]) for n, v in params.items()}
    M, T = int(g["M"]), int(g["T"])
    mix, src = synthetic.speech_like(M, 2, T, int(g["seed"]))
    assert abs(float(mix.double().abs().sum()) - float(g["mix_abs_sum"])) < 1e-6 * float(g["mix_abs_sum"]), \
        "synthetic batch drifted from the fixture's"
    np.testing.assert_array_equal(mix[:, :16].numpy(), g["mix_head"])
    return params, mix, src, g
