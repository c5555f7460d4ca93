#!/usr/bin/env python3
"""Conv-TasNet training-step throughput on MI355X (BASELINE.json metric).

One step = forward + PIT SI-SNR loss + backward + clip_grad_norm_(5) + Adam
(src/solver.py:178-186) over one per-GPU batch of synthetic speech-like
mixtures already resident in HBM.  Workload: paper config (N=256 L=20 B=256
H=512 P=3 X=8 R=4 gLN, 2 speakers, 4 s @ 8 kHz), 32 utterances per GPU, bf16
activations (fp32 params/stats/accumulation).  N GPUs = one process per GPU
under torchrun, the gradients averaged over RCCL with one flat all-reduce after
backward (ctn_dist.FlatGradAllReduce; CTN_GRAD_SYNC=ddp for DistributedDataParallel)
(weak scaling: per-GPU batch fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W]

With --gpus N > 1 and no WORLD_SIZE in the environment (no torchrun), bench.py
starts the N ranks itself as child processes (spawn_ranks); under torchrun it
is one of the ranks.

Prints ONE JSON line (rank 0).  `roofline` is measured live: the dominant
kernel's launches inside the timed region are bracketed by hipEvents on their
own stream (ctn_timer_*), and achieved = algorithmic bytes per launch / mean
launch time.  `cpu_baseline` times the fp32 CPU oracle (oracle/, test
infrastructure — never part of the GPU path) on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "conv-tasnet_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA

PAPER = dict(N=256, L=20, B=256, H=512, P=3, X=8, R=4, C=2, norm_type="gLN", causal=False,
             mask_nonlinear="relu")
# BASELINE.json configs runnable on one GPU: c2 is the metric's workload (the
# default); c4 (causal cLN, L=16, 16 kHz) and c5 (3 speakers, N=512, 8 s) are
# measured per GPU at their per-GPU batch for the record, never as the bench line.
CONFIGS = {
    "c2": (PAPER, 8000, 4.0, 32),
    "c4": (dict(PAPER, L=16, norm_type="cLN", causal=True), 16000, 4.0, 64),
    "c5": (dict(PAPER, N=512, C=3), 8000, 8.0, 16),
}

# timer kinds (include/ctn.h CTN_TIMER_*): the TemporalBlock's seven kernel families
TIMER_GEMM1, TIMER_DW_FWD, TIMER_GEMM_BWD_A, TIMER_DW_BWD, TIMER_GEMM_GX, TIMER_COLS_W1, TIMER_GEMM2 = range(1, 8)
TIMER_NAMES = {
    TIMER_GEMM1: "gemm_ws fwd 1x1 B->H (PReLU-stats epilogue)",
    TIMER_DW_FWD: "dw_fwd (norm1 + depthwise + PReLU-2 stats)",
    TIMER_GEMM_BWD_A: "gemm_dual bwd g_n2 = gy.W2 (norm-backward epilogue) + dW2 = gy^T.n2",
    TIMER_DW_BWD: "dw_bwd (norm2/PReLU2 bwd + transposed depthwise + dW_dw + norm1 sums)",
    TIMER_GEMM_GX: "gemm_ws bwd gx = n1bwd(g).W1 + gy (stores dL/dh1)",
    TIMER_COLS_W1: "gemm_cols bwd dW1 = (dL/dh1)^T.x",
    TIMER_GEMM2: "gemm_ws fwd 1x1 H->B (norm2 operand, residual)",
}


def kernel_bytes(kind, M, K, cfg, s=2):
    """Algorithmic HBM bytes per launch of the timed kernel family:
    each operand row read once and each output row written once, weights once."""
    B, H = cfg["B"], cfg["H"]
    rows = M * K
    if kind == TIMER_GEMM1:        # x[B] in, h1[H] out, W1 once
        return rows * (B + H) * s + B * H * s
    if kind == TIMER_DW_FWD:       # h1[H] in, d[H] out
        return rows * 2 * H * s
    if kind == TIMER_GEMM_BWD_A:   # gy[B] in, d[H] in, g[H] out, W2t once (+ dW2 fp32 once: dual kernel)
        return rows * (B + 2 * H) * s + B * H * s + (B * H * 4 if dual_pair_a() else 0)
    if kind == TIMER_DW_BWD:       # d, g_n2, h1 in, dL/d(hat a1) out
        return rows * 4 * H * s
    if kind == TIMER_GEMM_GX:      # g, h1, gy in; dL/dh1, gx out; W1 once
        return rows * (3 * H + 2 * B) * s + B * H * s
    if kind == TIMER_COLS_W1:      # dL/dh1, x in (dW1 partials fp32: 32 chunks)
        return rows * (B + H) * s
    if kind == TIMER_GEMM2:        # d in, x in (residual), y out; W2 once
        return rows * (H + 2 * B) * s + B * H * s
    raise ValueError(kind)


def copy_peak_gbs(dev, lib, sizes_mib=(256, 512, 1024), reps=10):
    """Measured streaming ceiling of this GPU: device-to-device copies (read + write bytes
    / time, best of `reps`) by torch's copy_ and by the library's 16-B-per-lane copy kernel
    (ctn_copy_bytes: grid-stride or one chunk per lane, with and without the nontemporal
    hint, 4 or 8 loads in flight) over buffers of 256 MiB to 1 GiB — the block kernels move
    157-420 MB per launch — SURVEY.md §8(d)'s measured peak beside the 8 TB/s datasheet
    value.  The best rate over all of them is the ceiling.  Returns (GB/s, which copy)."""
    import ctn_lib as L
    stream = torch.cuda.current_stream(dev).cuda_stream
    res = {}
    for mib in sizes_mib:
        n = mib * (1 << 20) // 4
        a = torch.empty(n, dtype=torch.float32, device=dev).uniform_()
        b = torch.empty_like(a)
        ways = {"torch copy_": lambda: b.copy_(a)}
        for fl in range(4):   # flags: nontemporal, 8 loads in flight
            per_wg = 256 * (8 if fl & 2 else 4) * 4          # floats one workgroup moves per round
            for wgs in (2048, 4096, min(65536, (n + per_wg - 1) // per_wg)):
                ways[f"ctn_copy_bytes wg={wgs} flags={fl}"] = (lambda w, f: lambda: L.check(
                    lib.ctn_copy_bytes(b.data_ptr(), a.data_ptr(), n * 4, w, f, stream), "ctn_copy_bytes"))(wgs, fl)
        for name, fn in ways.items():
            best = float("inf")
            for _ in range(reps + 2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1))
            res[f"{name} {mib} MiB"] = 2 * n * 4 / (best * 1e-3) / 1e9
        if not torch.equal(a, b):
            raise RuntimeError("bench.py: the calibration copy is wrong")
        del a, b
    name = max(res, key=res.get)
    if os.environ.get("CTN_COPY_VERBOSE"):
        print(json.dumps({k: round(v, 1) for k, v in res.items()}), file=sys.stderr)
    return res[name], name


def mfma_peak_tflops(dev, lib, reps=5):
    """Measured matrix peak of this GPU (a measured MFMA microbenchmark
    beside the 2.5 PF/s datasheet value): ctn_mfma_peak, back-to-back bf16 MFMAs on random
    register operands, 2 workgroups of 4 waves per CU, best of `reps` launches per shape.
    Returns {shape: TFLOP/s}."""
    import ctn_lib as L
    stream = torch.cuda.current_stream(dev).cuda_stream
    wgs = 2 * torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.empty(wgs * 256, dtype=torch.float32, device=dev)
    res = {}
    for shape, name, iters in ((0, "v_mfma_f32_16x16x32_bf16", 8000), (1, "v_mfma_f32_32x32x16_bf16", 8000)):
        flops = ctypes.c_double(0.0)
        best = float("inf")
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.check(lib.ctn_mfma_peak(shape, wgs, iters, out.data_ptr(), ctypes.byref(flops), stream), "ctn_mfma_peak")
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1))
        res[name] = round(flops.value / (best * 1e-3) / 1e12, 1)
    if not torch.isfinite(out).all():
        raise RuntimeError("bench.py: the MFMA microbenchmark produced non-finite values")
    return res


def dual_pair_a():
    """Pair A of the dual GEMM (ctn_gemm_dual.hip) is on unless CTN_GEMM_DUAL clears bit 0."""
    return bool(int(os.environ.get("CTN_GEMM_DUAL", "1")) & 1)


def step_alg_bytes(M, K, T, cfg, s=2):
    """SURVEY.md §8(d) compulsory bytes of one fwd+bwd step: X*R*(12H+7B)*K*s + edges."""
    N, B, H, C, X, R = cfg["N"], cfg["B"], cfg["H"], cfg["C"], cfg["X"], cfg["R"]
    per_utt = X * R * (12 * H + 7 * B) * K * s + (3 * N * K + 3 * B * K + 6 * C * N * K + 3 * C * T + 2 * T) * s
    return M * per_utt


def step_flops(M, K, cfg):
    N, L, B, H, P, X, R, C = (cfg[k] for k in ("N", "L", "B", "H", "P", "X", "R", "C"))
    f = 2 * K * (N * L + N * B + X * R * (2 * B * H + H * P) + B * C * N + C * N * L)
    return 3 * f * M


def _cpu_model():
    """CPU model name, the host's physical cores, the logical CPUs this process may run
    on, and the physical cores among those (lscpu's view, from /proc/cpuinfo)."""
    name, cores, core_of = "unknown", set(), {}
    try:
        with open("/proc/cpuinfo") as f:
            proc = phys = core = None
            for line in f.read().splitlines() + [""]:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    proc = int(v)
                elif k == "model name" and name == "unknown":
                    name = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    core = v
                elif not k and proc is not None:
                    cores.add((phys, core))
                    core_of[proc] = (phys, core)
                    proc = phys = core = None
    except OSError:
        pass
    allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    phys_allowed = len({core_of.get(c, c) for c in allowed})
    return name, len(cores) or None, len(allowed), phys_allowed


def _time_train_steps(cfg_d, T, seconds):
    from oracle import ctn_oracle as O
    import synthetic
    cfg = O.Cfg(**{k: cfg_d[k] for k in ("N", "L", "B", "H", "P", "X", "R", "C")})
    params = O.init_params(cfg, 0)
    mix, src = synthetic.speech_like(1, cfg.C, T, 99)
    lens = torch.tensor([T])
    O.train_step(cfg, params, mix, src, lens)                 # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        _, params = O.train_step(cfg, params, mix, src, lens)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return n, el


def cpu_baseline(seconds=10.0):
    """fp32 CPU oracle train step (fwd + loss + bwd + clip + Adam), M=1, on this box's host
    cores: the paper config (the reported value) and c1 (BASELINE.json configs[0]).

    SURVEY.md §8(d): torch.set_num_threads(n), n = the physical cores this process may
    run on.  The step is also timed at the process's default thread count (the box's
    per-GPU CPU share, OMP_NUM_THREADS); `value` is the faster of the two, and both are
    recorded."""
    default_threads = torch.get_num_threads()
    name, phys, allowed, phys_allowed = _cpu_model()
    runs = {}
    try:
        for threads in sorted({phys_allowed, default_threads}, reverse=True):
            torch.set_num_threads(threads)
            n, el = _time_train_steps(PAPER, 32000, seconds)
            runs[threads] = (n, el)
        best = max(runs, key=lambda th: runs[th][0] / runs[th][1])
        torch.set_num_threads(best)
        n1, el1 = _time_train_steps(dict(PAPER, N=64, B=64, H=128, X=2, R=2), 32000, seconds / 3)
    finally:
        torch.set_num_threads(default_threads)
    n, el = runs[best]
    return {"value": n / el, "unit": "utterances/sec", "cores": best, "kind": "port",
            "cpu": name, "physical_cores_on_host": phys, "cpus_allowed": allowed,
            "physical_cores_allowed": phys_allowed,
            "by_threads": {str(th): round(v[0] / v[1], 3) for th, v in runs.items()},
            "sample": f"{n} training steps (fwd+PIT loss+bwd+clip+Adam) of 1 utterance, paper config, "
                      f"4 s @ 8 kHz, fp32 oracle/ctn_oracle.py on {best} threads, {el:.1f} s "
                      f"(faster of {sorted(runs)} threads; {phys_allowed} physical cores allowed)",
            "c1": {"value": n1 / el1, "unit": "utterances/sec",
                   "sample": f"{n1} c1 training steps (N=64 B=64 H=128 X=2 R=2), 1 utterance 4 s @ 8 kHz, "
                             f"{best} threads, {el1:.1f} s"}}


def spawn_ranks(n, cmd, port=None, env=None):
    """Start `cmd` as n ranks of one job (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*), wait for
    all of them and return the first non-zero exit code (0 when every rank succeeded).

    The parent never touches the GPU and never execs: each rank is a fresh child process
    (the reference's multi-GPU path, src/train.py:120-122, is nn.DataParallel over the
    --id GPUs inside one process; here one process per GPU, DDP over RCCL)."""
    import socket
    import subprocess
    if port is None:
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=e))
    # Poll every rank: a rank that dies while another is blocked inside a collective
    # (which would only return at the RCCL timeout) must still end the job at once.
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.05)
    finally:
        for q in procs:                  # one rank failed: the others would wait forever
            if q.poll() is None:
                q.terminate()
        for q in procs:
            try:
                q.wait(timeout=30)
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()
    return rc


def _rehearsal() -> bool:
    """CTN_BENCH_REHEARSAL=1: the N-rank job on ONE GPU over gloo, to exercise the
    multi-rank code path (launcher, exchange, timing reduction) on a one-GPU box; its
    numbers are not a measurement."""
    return os.environ.get("CTN_BENCH_REHEARSAL", "0") == "1"


def visible_gpus():
    """GPUs this process may use, without initialising HIP in this process: the
    *_VISIBLE_DEVICES lists if set, else the GPU nodes of the KFD topology (sysfs)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() not in ("", "-1")])
    nodes = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for d in os.listdir(nodes):
            try:
                with open(os.path.join(nodes, d, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:    # CPU nodes have no SIMDs
                n += 1
    except OSError:
        return 0
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="BASELINE.json config (c2 = the metric's workload)")
    ap.add_argument("--batch", type=int, default=None, help="utterances per GPU (config default)")
    ap.add_argument("--seconds", type=float, default=None, help="utterance length (config default)")
    ap.add_argument("--fp32", action="store_true", help="fp32 activations (parity mode) instead of bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-copy-peak", action="store_true",
                    help="skip the calibration kernels after the timed steps (copy_peak and mfma_peak: null); "
                         "profiling runs use it so that no calibration kernel lands in a kernel trace")
    ap.add_argument("--timer-kind", type=int, default=0,
                    help="kernel timed in the timed region (default: the dominant one of the profile pass)")
    ap.add_argument("--timer-stride", type=int, default=9,
                    help="in the timed region, bracket every n-th launch of the timed kernel with "
                         "hipEvents (each bracket idles the GPU a few us around the launch); 9 is "
                         "coprime with the 32 launches per step, so the samples visit every block")
    ap.add_argument("--profile-steps", type=int, default=5,
                    help="untimed steps with every kernel family timed (the per-kernel table)")
    ap.add_argument("--ddp", action="store_true",
                    help="the data-parallel path over RCCL even at world size 1 (process-group init, "
                         "gradient exchange)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole step as a HIP graph after warmup and time its replays "
                         "(ctn_graph.StepGraph; one GPU, no exchange)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no outside launcher: start one rank per GPU ourselves (children, no exec); the
        # GPUs are counted from the environment / sysfs, so this parent never loads HIP
        visible = visible_gpus()
        if args.gpus > visible and not _rehearsal():
            sys.exit(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) visible")
        sys.exit(spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world and "WORLD_SIZE" in os.environ and args.gpus != 1:
        sys.exit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if _rehearsal():
        local = 0     # every rank on the one GPU (gloo: RCCL refuses two ranks per device)
    use_ddp = world > 1 or args.ddp
    if use_ddp:
        if "RANK" not in os.environ:      # --ddp without a launcher: a world of one rank
            import socket
            with socket.socket() as so:
                so.bind(("127.0.0.1", 0))
                port = so.getsockname()[1]
            os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(port))
        torch.cuda.set_device(local)
        if _rehearsal():
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()    # what RCCL reports
    dev = torch.device("cuda", local)

    import conv_tasnet as ct
    import ctn_lib as L
    import ctn_optim
    import pit_criterion as pc
    import synthetic

    cfg, rate, secs, batch = CONFIGS[args.config]
    if args.config != "c2":
        args.no_cpu_baseline = True   # the CPU baseline leg times the c2 workload only
    args.batch = batch if args.batch is None else args.batch
    args.seconds = secs if args.seconds is None else args.seconds
    M, C = args.batch, cfg["C"]
    T = int(args.seconds * rate)
    K = (T - cfg["L"]) // (cfg["L"] // 2) + 1

    torch.manual_seed(0)
    model = ct.ConvTasNet(**cfg).to(dev)
    model.act_dtype = torch.float32 if args.fp32 else torch.bfloat16
    # parameter-gradient tails on a second stream (ctn_ops._split_ok): off, the overlap
    # slowed the step by 6 % at this batch; CTN_WGRAD_STREAM=1 for A/B
    model.wgrad_stream = os.environ.get("CTN_WGRAD_STREAM", "0") == "1"
    # parameter-gradient reductions of all blocks batched at the end of backward (on by
    # default; CTN_DEFER_REDUCE=0 for A/B against the per-block reductions)
    model.defer_grad_reduce = os.environ.get("CTN_DEFER_REDUCE", "1") == "1"
    # gradient exchange across ranks: "flat" (default) = all-reduces of a persistent flat
    # gradient buffer, CTN_FLAT_CHUNKS - 1 of them during backward as groups of deferred
    # block reductions finish, the rest after it (ctn_dist.FlatGradAllReduce),
    # "ddp" = DistributedDataParallel's bucket hooks during backward (per-block reductions)
    sync_kind = os.environ.get("CTN_GRAD_SYNC", "flat")
    if sync_kind not in ("flat", "ddp"):
        sys.exit(f"bench.py: CTN_GRAD_SYNC={sync_kind} (flat|ddp)")
    grad_sync = None
    if use_ddp and sync_kind == "flat":
        import ctn_dist
        grad_sync = ctn_dist.FlatGradAllReduce(model.parameters(),
                                               chunks=int(os.environ.get("CTN_FLAT_CHUNKS", "4")))
    elif use_ddp:
        # gradients as views into the RCCL buckets (no per-step copy into the buckets),
        # one fixed graph (the reducer skips its unused-parameter search each step)
        model = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[local], bucket_cap_mb=int(os.environ.get("CTN_DDP_BUCKET_MB", "25")),
            gradient_as_bucket_view=os.environ.get("CTN_DDP_VIEW", "1") == "1",
            static_graph=os.environ.get("CTN_DDP_STATIC", "1") == "1")
    # the solver's update (src/solver.py:184-186) on the HIP path: one launch for
    # the clip norm, one for the clip scale, one for Adam over all 294 tensors
    opt = ctn_optim.Adam(model.parameters(), lr=1e-3, capturable=args.graph)
    mix, src = synthetic.speech_like(M, C, T, 1234 + rank)
    mix, src = mix.to(dev), src.to(dev)
    lens = torch.full((M,), T, dtype=torch.int64, device=dev)

    plist = list(model.parameters())   # (model.parameters() walks every module each call)

    def step():
        est = model(mix)
        loss = pc.cal_loss(src, est, lens)[0]
        opt.zero_grad(set_to_none=True)
        loss.backward()
        if grad_sync is not None:
            grad_sync.sync()
        ctn_optim.clip_grad_norm_(plist, 5.0)
        opt.step()
        return loss

    import ctn_ops
    for _ in range(args.warmup):
        step()
    lib = L.load()
    s_el = 4 if args.fp32 else 2
    # profile pass (untimed): every kernel family bracketed by hipEvents -> per-kernel table
    table = {}
    if args.profile_steps > 0:
        torch.cuda.synchronize(dev)
        L.check(lib.ctn_timer_enable_mask(sum(1 << k for k in TIMER_NAMES), args.profile_steps * 64),
                "ctn_timer_enable_mask")
        for _ in range(args.profile_steps):
            step()
        torch.cuda.synchronize(dev)
        for k in TIMER_NAMES:
            tk, nk = ctypes.c_double(0.0), ctypes.c_int(0)
            L.check(lib.ctn_timer_read_kind(k, ctypes.byref(tk), ctypes.byref(nk)), "ctn_timer_read_kind")
            if nk.value:
                mean_k = tk.value / nk.value
                kb_k = kernel_bytes(k, M, K, cfg, s_el)
                table[k] = {"kernel": TIMER_NAMES[k], "mean_us": round(mean_k * 1e3, 2),
                            "launches_per_step": round(nk.value / args.profile_steps, 2),
                            "ms_per_step": round(tk.value / args.profile_steps, 4),
                            "alg_bytes": kb_k, "GBps": round(kb_k / (mean_k * 1e-3) / 1e9, 1),
                            "frac": round(kb_k / (mean_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        lib.ctn_timer_enable(0, 0)
    if not args.timer_kind:   # the kernel family with the most time per step
        args.timer_kind = max(table, key=lambda k: table[k]["ms_per_step"]) if table else TIMER_GEMM_BWD_A
    n_def0 = ctn_ops.DEFERRED_BLOCKS
    graph = None
    if args.graph:
        if use_ddp:
            sys.exit("bench.py: --graph runs one process on one GPU (no exchange inside the graph)")
        import ctn_graph
        graph = ctn_graph.StepGraph(step, warmup=1)   # one more eager step on a side stream, then capture
    torch.cuda.synchronize(dev)
    if graph is None:   # (a replay re-runs the captured launches: the live timer sees none of them)
        L.check(lib.ctn_timer_set_stride(args.timer_stride), "ctn_timer_set_stride")
        L.check(lib.ctn_timer_enable(args.timer_kind, args.steps * 64), "ctn_timer_enable")
    if use_ddp:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step() if graph is None else graph.replay()
    torch.cuda.synchronize(dev)
    if use_ddp:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tot = ctypes.c_double(0.0)
    nl = ctypes.c_int(0)
    L.check(lib.ctn_timer_read(ctypes.byref(tot), ctypes.byref(nl)), "ctn_timer_read")
    lib.ctn_timer_enable(0, 0)
    lib.ctn_timer_set_stride(1)
    # a generation-word timeout anywhere in the run fails the bench (ctn_device_status)
    L.check(lib.ctn_device_status(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), None, 0),
            "ctn_device_status")
    rank_ms = [round(elapsed / args.steps * 1e3, 3)]
    if use_ddp:
        # every rank's time (max = the job's time); the list's length is RCCL's world size
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        ts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(ts, t)
        rank_ms = [round(float(x) / args.steps * 1e3, 3) for x in ts]
        elapsed = max(float(x) for x in ts)
    final_loss = float(loss.detach())
    deferred = (ctn_ops.DEFERRED_BLOCKS - n_def0) / args.steps
    copy_gbs, copy_how = copy_peak_gbs(dev, lib) if rank == 0 and not args.no_copy_peak else (None, None)
    mfma_peak = mfma_peak_tflops(dev, lib) if rank == 0 and not args.no_copy_peak else None

    if rank == 0:
        s = s_el
        ms = elapsed / args.steps * 1e3
        utt_s = world * M * args.steps / elapsed
        kb = kernel_bytes(args.timer_kind, M, K, cfg, s)
        mean_ms = tot.value / max(nl.value, 1)
        if graph is not None and args.timer_kind in table:   # graph: the eager profile pass's timing
            mean_ms = table[args.timer_kind]["mean_us"] * 1e-3
            nl.value = int(round(table[args.timer_kind]["launches_per_step"] * args.steps))
        achieved = kb / (mean_ms * 1e-3) / 1e9
        traffic = mfma = step_pmc = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")   # c2 FETCH_SIZE/WRITE_SIZE passes
        if os.path.exists(pmc) and args.config == "c2":
            with open(pmc) as f:
                traffic = json.load(f).get(str(args.timer_kind))
        pmc = os.path.join(ROOT, "profiles", "pmc_step.json")      # the same passes, whole step (tools/pmc_step.py)
        if os.path.exists(pmc) and args.config == "c2" and not args.fp32:
            with open(pmc) as f:
                step_pmc = json.load(f).get("step_GB")
        pmc = os.path.join(ROOT, "profiles", "pmc_mfma.json")   # tools/gpu.sh prof, MFMA pass
        if os.path.exists(pmc):
            with open(pmc) as f:
                mfma = json.load(f).get(str(args.timer_kind))
        out = {
            "metric": ("utterances/sec (4s, 8kHz, 2-spk) fwd+bwd" if args.config == "c2" else
                       f"utterances/sec ({args.seconds:g}s, {rate // 1000}kHz, {C}-spk) fwd+bwd, {args.config}"),
            "value": round(utt_s, 2),
            "unit": "utterances/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if args.fp32 else "bf16",
            "data": "synthetic (AR(2) speech-like sources, random-init weights)",
            "config": {"workload": ("paper config train step c2: N=256 L=20 B=256 H=512 P=3 X=8 R=4 gLN "
                                    "non-causal relu-mask, 2 spk, 4 s @ 8 kHz, fwd+PIT loss+bwd+clip+Adam"
                                    if args.config == "c2" else
                                    f"{args.config} train step: N={cfg['N']} L={cfg['L']} B={cfg['B']} H={cfg['H']} "
                                    f"P={cfg['P']} X={cfg['X']} R={cfg['R']} {cfg['norm_type']} "
                                    f"{'causal' if cfg['causal'] else 'non-causal'} relu-mask, {C} spk, "
                                    f"{args.seconds:g} s @ {rate // 1000} kHz, fwd+PIT loss+bwd+clip+Adam"),
                       "per_gpu_batch": M, "global_batch": M * world, "samples": T, "frames": K,
                       "parallelism": f"dp{world}" + ((" (DDP/" if grad_sync is None else " (flat all-reduce/")
                                                      + ("gloo)" if _rehearsal() else "RCCL)") if use_ddp else "")
                                      + (" REHEARSAL: all ranks on one GPU over gloo" if _rehearsal() else ""),
                       "rccl_world_size": dist.get_world_size() if use_ddp and not _rehearsal() else None,
                       "rank_ms_per_step": rank_ms,
                       # timed steps as replays of one captured HIP graph (--graph)
                       "hip_graph": graph is not None,
                       # TemporalBlock backwards per step whose parameter-gradient reductions
                       # ran batched at the end of backward (ctn_tblock_reduce_grads)
                       "deferred_grad_reduce_blocks": deferred},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": TIMER_NAMES[args.timer_kind] if not (args.timer_kind == TIMER_GEMM_BWD_A and
                                                                        not dual_pair_a()) else
                         "gemm_ws bwd g_n2 = gy.W2 (norm-backward epilogue)",
                         # measured streaming ceiling on this GPU (device copy, read + write)
                         "copy_peak": round(copy_gbs, 1) if copy_gbs else None, "copy_peak_by": copy_how,
                         "frac_of_copy_peak": round(achieved / copy_gbs, 4) if copy_gbs else None,
                         "launches": nl.value, "timer_stride": args.timer_stride, "mean_ms": round(mean_ms, 4), "bytes_per_launch": kb,
                         # rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs) of
                         # this kernel, from the committed PMC pass (profiles/pmc_mfma.json)
                         "mfma_util": mfma.get("mfma_util") if mfma else None,
                         # measured matrix peak (ctn_mfma_peak) beside the dense bf16 datasheet value
                         "mfma_peak": {"measured_tflops": mfma_peak, "datasheet_tflops": BF16_PEAK_TFLOPS},
                         # the whole step against the same peak: SURVEY §8d compulsory bytes
                         "step_frac": round(step_alg_bytes(M, K, T, cfg, s) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         # every TemporalBlock kernel family, timed live in the untimed profile
                         # pass (hipEvents on the launch stream), sorted by time per step
                         "kernels": sorted(table.values(), key=lambda r: -r["ms_per_step"])},
            "step_model": {"alg_bytes_GB": round(step_alg_bytes(M, K, T, cfg, s) / 1e9, 3),
                           "alg_GBps": round(step_alg_bytes(M, K, T, cfg, s) / (ms * 1e-3) / 1e9, 1),
                           "tflops": round(step_flops(M, K, cfg) / (ms * 1e-3) / 1e12, 1),
                           # HBM bytes of one whole step measured by rocprofv3 (committed PMC passes)
                           "pmc_GB": round(step_pmc, 2) if step_pmc else None},
            "final_loss": round(final_loss, 4),
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    if use_ddp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
