"""Host-side cost of one training step: time to ISSUE k steps (no sync inside)
vs the synchronized wall time.  If issue time ~ wall time, the step is bound by
the host (Python + launch overhead), not by the GPU."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "conv-tasnet_amd")]
import bench  # noqa: E402
import conv_tasnet as ct  # noqa: E402
import ctn_optim  # noqa: E402
import pit_criterion as pc  # noqa: E402
import synthetic  # noqa: E402

dev = torch.device("cuda")
cfg = bench.PAPER
M, T = 8, 32000
torch.manual_seed(0)
model = ct.ConvTasNet(**cfg).to(dev)
model.act_dtype = torch.bfloat16
opt = ctn_optim.Adam(model.parameters(), lr=1e-3)
mix, src = synthetic.speech_like(M, cfg["C"], T, 1)
mix, src = mix.to(dev), src.to(dev)
lens = torch.full((M,), T, dtype=torch.int64, device=dev)


def step(parts):
    t = time.perf_counter()
    est = model(mix)
    loss = pc.cal_loss(src, est, lens)[0]
    t1 = time.perf_counter()
    opt.zero_grad(set_to_none=True)
    loss.backward()
    t2 = time.perf_counter()
    ctn_optim.clip_grad_norm_(model.parameters(), 5.0)
    opt.step()
    t3 = time.perf_counter()
    parts[0] += t1 - t; parts[1] += t2 - t1; parts[2] += t3 - t2


p = [0.0, 0.0, 0.0]
for _ in range(3):
    step(p)
torch.cuda.synchronize()
K = 10
p = [0.0, 0.0, 0.0]
t0 = time.perf_counter()
for _ in range(K):
    step(p)
t_issue = time.perf_counter() - t0
torch.cuda.synchronize()
t_wall = time.perf_counter() - t0
print(f"M={M}: issue {t_issue / K * 1e3:.2f} ms/step (fwd {p[0] / K * 1e3:.2f}, bwd {p[1] / K * 1e3:.2f}, "
      f"update {p[2] / K * 1e3:.2f}); wall {t_wall / K * 1e3:.2f} ms/step")
