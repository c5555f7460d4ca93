# locate the first streamed sample that departs from the whole forward (small model)
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "conv-tasnet_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import conv_tasnet as ct, streaming
DEV = "cuda"
def model(H=32, B=16, N=32, X=4):
    torch.manual_seed(0)
    m = ct.ConvTasNet(N=N, L=16, B=B, H=H, P=3, X=X, R=2, C=2, norm_type="cLN", causal=True).to(DEV)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("gamma") or n.endswith("beta") or n.endswith(".weight") and p.dim() == 1:
                p.add_(0.2 * torch.randn_like(p))
    return m.eval()
for (H, B, N, X) in [(32, 16, 32, 4), (512, 256, 256, 4), (32, 16, 32, 1)]:
    m = model(H, B, N, X)
    for M in (1, 3):
        mix = torch.randn(M, 4000, device=DEV)
        with torch.no_grad():
            full = m(mix)
        for chunk, mf in ((8, 64), (100, 64), (100, 8), (100, 1), (1000, 64)):
            out = streaming.StreamingSeparator(m, max_frames=mf).separate(mix, chunk)
            d = (out - full).abs().amax(dim=(0, 1))
            bad = (d > 1e-4 * full.abs().max()).nonzero()
            first = int(bad[0]) if len(bad) else -1
            print(f"H={H} B={B} N={N} X={X} M={M} chunk={chunk} max_frames={mf}: first bad sample {first} "
                  f"(frame {first // 8 if first >= 0 else -1}), max diff {float(d.max()):.3e}", flush=True)
