"""Reference points for the 1x1 GEMM shapes of the paper block (M*Kp=102400 rows):
hipBLASLt (torch.mm) time and a torch copy of the same bytes, bf16."""
import torch
rows = 102400
def t(f, n=20):
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3
for kin, nout in ((256, 512), (512, 256), (512, 512)):
    a = torch.randn(rows, kin, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(nout, kin, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(rows, nout, device="cuda", dtype=torch.bfloat16)
    us = t(lambda: torch.mm(a, w.t(), out=c))
    by = rows * (kin + nout) * 2
    print(f"mm rows x {kin} -> {nout}: {us:7.1f} us  {by / us / 1e3:7.0f} GB/s")
    # weight-gradient shape: w' = c^T a  (reduction over rows)
    g = torch.empty(nout, kin, device="cuda", dtype=torch.float32)
    us = t(lambda: torch.mm(c.t(), a, out=g.to(torch.bfloat16)))
    print(f"mm^T rows reduction {nout}x{kin}: {us:7.1f} us  {by / us / 1e3:7.0f} GB/s")
x = torch.randn(rows * 768, device="cuda", dtype=torch.bfloat16)
y = torch.empty_like(x)
us = t(lambda: y.copy_(x))
print(f"copy {x.numel()*2/1e6:.0f} MB r+w: {us:7.1f} us  {2 * x.numel() * 2 / us / 1e3:7.0f} GB/s")
