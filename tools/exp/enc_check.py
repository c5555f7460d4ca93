"""Encoder forward: MFMA (bf16) vs VALU (bf16) vs fp32 outputs, relative L2 per path."""
import os, sys
sys.path.insert(0, "conv-tasnet_amd")
import torch
import conv_tasnet as ct
torch.manual_seed(0)
for N, L in ((256, 20), (256, 16), (512, 20)):
    enc = ct.Encoder(L, N).cuda()
    x = torch.randn(3, 5003, device="cuda")
    outs = {}
    for name, dt, mf in (("f32", torch.float32, "1"), ("valu", torch.bfloat16, "0"), ("mfma", torch.bfloat16, "1")):
        os.environ["CTN_ENC_MFMA"] = mf
        enc.act_dtype = dt
        with torch.no_grad():
            outs[name] = enc(x).float()
    r = lambda a, b: float((a - b).norm() / b.norm())
    print(N, L, "valu-f32 %.2e  mfma-f32 %.2e  mfma-valu %.2e" % (r(outs["valu"], outs["f32"]), r(outs["mfma"], outs["f32"]), r(outs["mfma"], outs["valu"])),
          "zeros f32 %d valu %d mfma %d" % tuple(int((o == 0).sum()) for o in (outs["f32"], outs["valu"], outs["mfma"])))
