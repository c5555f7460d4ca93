"""Debug: one TemporalBlock forward through the C-ABI with CTN_DW_WAVE=1 and =0; where do
h1, d, the saved statistics and y differ (utterance, frame, channel pattern)."""
import ctypes, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "conv-tasnet_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import ctn_lib as L
import ctn_ops as ops
from test_gpu_benchshape import _block_params

M, K, d, causal = [int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (32, 3199, 1, 0))]
norm = L.NORM_CLN if len(sys.argv) > 5 and sys.argv[5] == "cLN" else L.NORM_GLN
lib = L.load()
dev = torch.device("cuda")
torch.manual_seed(3)
params = [p.to(dev) for p in _block_params(41 + d, 256, 512)]
fr = ops.Frames.of(M, K)
x = ops.ncw_to_rows(torch.randn(M, 256, K, device=dev), fr, torch.bfloat16)
pack = ops.WeightPacks().get([(params[0], params[8])], dev)[0]

def fwd():
    desc = L.TBlockDesc(fr.M, fr.K, fr.Kp, 256, 512, 3, d, causal, norm, L.dtype_code(torch.bfloat16))
    ps = L.TBlockParams(*[p.data_ptr() for p in params], *pack[:4], *ops._NO_BN, *pack[4:8])
    y = torch.empty_like(x); h1 = x.new_empty(fr.rows, 512); dd = x.new_empty(fr.rows, 512)
    st = torch.empty(lib.ctn_tblock_stats_floats(ctypes.byref(desc)), dtype=torch.float32, device=dev)
    sv = L.TBlockSaved(h1.data_ptr(), dd.data_ptr(), st.data_ptr())
    nb = lib.ctn_tblock_workspace_bytes(ctypes.byref(desc), 0)
    ws = L.workspace(nb, dev)
    L.check(lib.ctn_tblock_forward(ctypes.byref(desc), ctypes.byref(ps), x.data_ptr(), y.data_ptr(), ctypes.byref(sv),
                                   ws.data_ptr(), nb, L.stream_handle(dev)), "fwd")
    torch.cuda.synchronize()
    return y.float(), h1.float(), dd.float(), st

out = {}
for v in ("1", "0"):
    os.environ["CTN_DW_WAVE"] = v
    out[v] = fwd()
for name, a, b in zip(("y", "h1", "d", "stats"), out["1"], out["0"]):
    bad = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
    n = int(bad.sum())
    print(name, "mismatches", n, "of", a.numel(), "nan", int(torch.isnan(a).sum()), int(torch.isnan(b).sum()))
    if n and a.dim() == 2:
        rows = bad.any(1).nonzero().flatten()
        utt = (rows // fr.Kp).tolist(); frm = (rows % fr.Kp).tolist()
        import collections
        print("  rows", len(rows), "utterances", sorted(collections.Counter(utt).items())[:12])
        print("  frames (first 40)", frm[:40])
        ch = bad.any(0).nonzero().flatten()
        print("  channels", len(ch), ch[:20].tolist())
        r0 = int(rows[0]); print("  row", r0, "new", a[r0, :8].tolist(), "old", b[r0, :8].tolist())
    elif n:
        idx = bad.nonzero().flatten()[:20].tolist(); print("  idx", idx, a.flatten()[idx[:4]].tolist(), b.flatten()[idx[:4]].tolist())
