"""Diagnostic: per-parameter relative error of bf16-mode gradients vs fp32-mode
gradients (both HIP) on a golden model fixture."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "conv-tasnet_amd"), os.path.join(ROOT, "tests")]
import test_gpu_model as tg
from oracle import ctn_oracle as O

name = sys.argv[1] if len(sys.argv) > 1 else "model_paper_short.npz"
g = tg.load(name)
cfg = tg.cfg_of(g)
res = {}
for bf in (False, True):
    m = tg.build(cfg, g)
    est, loss, ms, _ = tg.run(m, g, bf16=bf)
    res[bf] = (est.detach().cpu().numpy(), float(loss), {n: p.grad.detach().cpu().numpy().copy() for n, p in m.named_parameters()})
print("loss fp32 %.6f bf16 %.6f golden %.6f" % (res[False][1], res[True][1], float(g["loss"])))
print("est rel", tg.rel(res[True][0], res[False][0]))
for n, _ in O.param_shapes(cfg):
    a, b = res[True][2][n], res[False][2][n]
    print("%-50s rel %.3e  |g| %.3e  gold-norm %.3e fp32-norm %.3e" % (n, tg.rel(a, b), np.linalg.norm(b), float(g["gnorm:" + n]), np.linalg.norm(b)))
