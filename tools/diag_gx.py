"""Diagnose the per-utterance fp32 gx outlier of test_gpu_benchshape (GPU)."""
import sys, os
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "conv-tasnet_amd"), os.path.join(ROOT, "tests")]
import test_gpu_benchshape as T

for (M, K, d, causal, norm) in [(7, 3000, 4, 0, "gLN"), (3, 3199, 16, 1, "cLN"), (2, 1000, 4, 0, "gLN")]:
    torch.manual_seed(M * 1000 + d)
    params = T._block_params(11 + d, 256, 512)
    x = torch.randn(M, 256, K)
    G = torch.randn(M, 256, K)
    y, gx, gp = T._hip_block(x, G, params, d, causal, norm, torch.float32, packed=False)
    yr, gxr, gpr = T._oracle_block(x, G, params, d, causal, norm)
    eg = np.array([T.rel(gx[m], gxr[m]) for m in range(M)])
    m = int(eg.argmax())
    diff = (gx[m] - gxr[m]).abs()          # [B, K]
    per_frame = diff.max(0).values.numpy()
    per_chan = diff.max(1).values.numpy()
    bad = np.nonzero(per_frame > 1e-3 * float(gxr[m].abs().max()))[0]
    print(f"M={M} K={K} d={d} {norm} c={causal}: per-utt gx err {np.array2string(eg, precision=2)}; worst utt {m}")
    print("  frames with large err:", bad[:20], "... count", len(bad), " chans max err argmax", per_chan.argmax(),
          "max", per_chan.max(), "ref scale", float(gxr[m].abs().max()))
    for n, a, b in zip(T._names(causal), gp, gpr):
        print(f"  {n}: {T.rel(a.reshape(b.shape), b):.2e}")
