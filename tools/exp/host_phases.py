"""Host-side issue time per phase of the bench step (no syncs added inside the step;
--sync drains the GPU before each phase, so each phase's host time is free of queue
back-pressure):
a phase whose host time jumps to GPU-time scale contains a synchronization.  Also runs
three steps under torch.cuda.set_sync_debug_mode("warn") to name synchronizing calls."""
import sys, time, warnings
sys.path.insert(0, "conv-tasnet_amd"); sys.path.insert(0, ".")
import torch
import conv_tasnet as ct
import ctn_optim
import pit_criterion as pc
import synthetic
from bench import PAPER

dev = torch.device("cuda:0")
M, C, T = 32, 2, 32000
torch.manual_seed(0)
model = ct.ConvTasNet(**PAPER).to(dev)
model.act_dtype = torch.bfloat16
opt = ctn_optim.Adam(model.parameters(), lr=1e-3)
mix, src = synthetic.speech_like(M, C, T, 1234)
mix, src = mix.to(dev), src.to(dev)
lens = torch.full((M,), T, dtype=torch.int64, device=dev)
ph = {}
plist = list(model.parameters())   # as bench.py
SYNC = "--sync" in sys.argv   # drain the GPU before each phase: host cost without queue back-pressure


def step(rec):
    times = []

    def run(name, fn):
        if SYNC:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        times.append((name, (time.perf_counter() - t0) * 1e3))
        return r

    est = run("forward", lambda: model(mix))
    loss = run("loss", lambda: pc.cal_loss(src, est, lens)[0])
    run("zero_grad", lambda: opt.zero_grad(set_to_none=True))
    run("backward", lambda: loss.backward())
    run("clip", lambda: ctn_optim.clip_grad_norm_(plist, 5.0))
    run("adam", lambda: opt.step())
    if rec:
        for n, v in times:
            ph.setdefault(n, []).append(v)


for _ in range(5):
    step(False)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    step(True)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host issue {1e3 * (t1 - t0) / 10:.2f} ms/step, wall {1e3 * (t2 - t0) / 10:.2f} ms/step")
for n, v in ph.items():
    v = sorted(v)
    print(f"  {n:10s} median {v[len(v) // 2]:7.3f} ms  max {v[-1]:7.3f} ms")
torch.cuda.set_sync_debug_mode("warn")
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    for _ in range(2):
        step(False)
    torch.cuda.synchronize()
torch.cuda.set_sync_debug_mode(0)
seen = set()
for x in w:
    k = str(x.message)[:160] + " @ " + f"{x.filename}:{x.lineno}"
    if k not in seen:
        seen.add(k)
        print("SYNC:", k)
print(f"{len(w)} sync warnings in 2 steps")
print("optimizer fast paths:", ctn_optim.FAST_STATS, "(sync mode)" if SYNC else "")
if "--cprofile" in sys.argv:   # where the host time of 5 steps goes, by function
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        step(False)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
