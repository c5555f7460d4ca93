"""Run-to-run bit equality of one bf16 TemporalBlock fwd+bwd (paper dims), per path."""
import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "conv-tasnet_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import ctn_lib as L
import ctn_ops as ops
from test_gpu_tblock import _paper_block
torch.manual_seed(0)
params = _paper_block(3)
M, B, K = 2, 256, 700
fr = ops.Frames.of(M, K)
x = ops.ncw_to_rows(torch.randn(M, B, K, device="cuda"), fr, torch.bfloat16)
cfg = (B, 512, 3, 4, False, L.NORM_GLN)
ps = [p.to("cuda").clone().requires_grad_(True) for p in params]
def run(pack):
    for p in ps:
        p.grad = None
    xx = x.clone().requires_grad_(True)
    y = ops.TBlockFn.apply(xx, fr, cfg, pack, None, *ps)
    y.float().square().sum().backward()
    return [y.detach(), xx.grad.detach()] + [p.grad.detach().clone() for p in ps]
packs = ops.WeightPacks()
pk = packs.get([(ps[0], ps[8])], x.device)[0]
r = [run(None), run(None), run(pk), run(pk)]
names = ["y", "gx"] + [f"p{i}" for i in range(9)]
for i, n in enumerate(names):
    print(n, "none-none", torch.equal(r[0][i], r[1][i]), "pk-pk", torch.equal(r[2][i], r[3][i]), "none-pk", torch.equal(r[0][i], r[2][i]))
