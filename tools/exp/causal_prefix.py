"""Causal TemporalBlock: outputs on a K-frame prefix must equal the first K outputs on the
full sequence.  Prints (dilation, K, stage, max diff) for mismatches."""
import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "conv-tasnet_amd"))
import conv_tasnet as ct, ctn_ops as ops, ctn_lib as L
torch.manual_seed(0)
B, H = 16, 32
for norm in ("cLN",):
    for d in (1, 2, 4, 8):
        blk = ct.TemporalBlock(B, H, 3, 1, 2 * d, d, norm_type=norm, causal=True).cuda()
        with torch.no_grad():
            for p in blk.parameters():
                p.add_(0.1 * torch.randn_like(p))
        full = torch.randn(1, 60, B, device="cuda")
        def run(seq):
            rows, fr = None, ops.Frames.of(1, seq.shape[1])
            r = seq.new_zeros(1, fr.Kp, B); r[:, :seq.shape[1]] = seq
            with torch.no_grad():
                y = blk._forward_rows(r.view(fr.Kp, B), fr, L.NORM_CLN)
            return y.view(1, fr.Kp, B)[:, :seq.shape[1]]
        yf = run(full)
        bad = []
        for K in range(1, 40):
            yk = run(full[:, :K])
            dd = (yk - yf[:, :K]).abs().amax(dim=(0, 2))
            if float(dd.max()) > 1e-5:
                bad.append((K, int((dd > 1e-5).nonzero()[0]), round(float(dd.max()), 3)))
        print(norm, "d", d, "mismatch (K, first frame, maxdiff):", bad[:12])
