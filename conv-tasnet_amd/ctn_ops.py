"""torch.autograd.Function wrappers around the C ABI (one native call per
forward and per backward).  Activations travel between ops in the frame-row
layout [M*Kp, C]; parameters stay fp32 in reference shapes."""
from __future__ import annotations

import ctypes
import os
import sys
import weakref
from dataclasses import dataclass

import torch

import ctn_lib as L


@dataclass(frozen=True)
class Frames:
    """Frame-row geometry of one batch: M utterances, K frames, Kp padded."""
    M: int
    K: int
    Kp: int

    @property
    def rows(self) -> int:
        return self.M * self.Kp

    @staticmethod
    def of(M: int, K: int) -> "Frames":
        return Frames(M, K, L.padded_frames(K))


def _f32(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32 or not t.is_contiguous():
        t = t.float().contiguous()
    return t


# ----------------------------------------------------------------------------
# TemporalBlock (conv_tasnet.py:212-272)
# ----------------------------------------------------------------------------
class WeightPacks:
    """bf16 compute copies of the TemporalBlocks' 1x1 weights (W1 [H,B], W2 [B,H]
    and both transposes, row-major and, when B and H are multiples of 32, in the
    MFMA fragment order the weight-stationary kernels load from: include/ctn.h
    ctn_weight_pack), refreshed for all stale blocks in ONE native call per
    step (ctn_pack_weights) instead of a conversion inside every block call.
    A copy is stale when its fp32 parameter's version counter moved: every
    in-place update bumps it (torch optimizers, load_state_dict, and
    ctn_optim.Adam, which bumps it explicitly)."""

    def __init__(self):
        self.key = None
        self.buf = None
        self.vers = []
        self.ptrs = []

    def get(self, pairs: list, device) -> list:
        """pairs: [(w1, w2)] fp32 parameters -> [(w1s, w2s, w1t, w2t, w1f, w2f, w1tf, w2tf,
        buf)]: eight device pointers into ``buf`` (the fragment-order four None when B
        or H is not a multiple of 32), returned WITH the buffer so that every autograd
        node that saves a pack keeps its storage alive until its backward has run (the
        cache may reallocate ``buf`` between forward and backward)."""
        key = (device, tuple((w1.data_ptr(), w2.data_ptr(), tuple(w1.shape), tuple(w2.shape)) for w1, w2 in pairs))
        if key != self.key:
            frag = os.environ.get("CTN_WEIGHT_FRAG", "1") != "0"   # 0: row-major copies only (A/B)
            sizes = [(w1.numel(), w2.numel(), frag and w1.shape[0] % 32 == 0 and w1.shape[1] % 32 == 0)
                     for w1, w2 in pairs]
            total = sum((4 if fr else 2) * (a + b) for a, b, fr in sizes)
            self.buf = torch.empty(total, dtype=torch.bfloat16, device=device)
            base, off, self.ptrs = self.buf.data_ptr(), 0, []
            for a, b, fr in sizes:
                n = 2 if fr else 1
                ptrs = []
                for _ in range(n):   # row-major (w1s, w2s, w1t, w2t), then the fragment-order four
                    ptrs += [base + 2 * o for o in (off, off + a, off + a + b, off + 2 * a + b)]
                    off += 2 * (a + b)
                self.ptrs.append(tuple(ptrs) + (None,) * (8 - len(ptrs)))
            self.key = key
            self.vers = [None] * len(pairs)
        packs = []
        for i, (w1, w2) in enumerate(pairs):
            v = (w1._version, w2._version)
            if self.vers[i] != v:
                w1s, w2s, w1t, w2t, w1f, w2f, w1tf, w2tf = self.ptrs[i]
                H, B = w1.shape[0], w1.shape[1]
                packs.append(L.WeightPack(_f32(w1).data_ptr(), H, B, w1s, w1t, w1f, w1tf))
                packs.append(L.WeightPack(_f32(w2).data_ptr(), B, H, w2s, w2t, w2f, w2tf))
                self.vers[i] = v
        if packs:
            arr = (L.WeightPack * len(packs))(*packs)
            L.check(L.load().ctn_pack_weights(arr, len(packs), L.stream_handle(device)), "ctn_pack_weights")
        return [(*p, self.buf) for p in self.ptrs]


class PackCache:
    """One WeightPacks per device.  nn.DataParallel replicas share their module's
    __dict__ (src/train.py:121 replicates per forward), so a single shared cache
    would be re-keyed and overwritten concurrently by the per-GPU threads; keyed by
    device, each thread only ever touches its own entry."""

    def __init__(self):
        self.by_dev = {}

    def get(self, pairs: list, device) -> list:
        wp = self.by_dev.get(device)
        if wp is None:
            wp = self.by_dev.setdefault(device, WeightPacks())
        return wp.get(pairs, device)


_NO_BN = (None, None, None, None, 0, 0.0, 0.0, 0.0, 0.0)


def bn_state(bn1: torch.nn.BatchNorm1d, bn2: torch.nn.BatchNorm1d) -> tuple:
    """The ctn_tblock_params BatchNorm fields for a block's two nn.BatchNorm1d
    (conv_tasnet.py:302-303), following torch.nn.modules.batchnorm._BatchNorm.forward:
    a training-mode call counts num_batches_tracked and uses momentum (or the
    cumulative factor 1/num_batches_tracked when momentum is None); batch statistics
    are used in training mode or when there are no running statistics."""
    training = bn1.training
    out_ptrs, facs, epss = [], [], []
    for bn in (bn1, bn2):
        fac = 0.0 if bn.momentum is None else float(bn.momentum)
        if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
            if bn.momentum is None:
                fac = 1.0 / float(bn.num_batches_tracked)
        use_running = (not bn.training or bn.track_running_stats) and bn.running_mean is not None
        for t in (bn.running_mean, bn.running_var):
            if use_running and (t.dtype != torch.float32 or not t.is_contiguous()):
                raise L.CtnLibraryError("BatchNorm running statistics must be contiguous float32")
        out_ptrs += [bn.running_mean.data_ptr() if use_running else None,
                     bn.running_var.data_ptr() if use_running else None]
        facs.append(fac)
        epss.append(float(bn.eps))
    return (*out_ptrs, int(training), facs[0], facs[1], epss[0], epss[1])


# ----------------------------------------------------------------------------
# parameter gradients on a second stream (ctn_tblock_backward_split)
# ----------------------------------------------------------------------------
_WGRAD_STREAMS = {}
# (device, autograd graph task) pairs whose end-of-backward join is queued.  Keyed by the
# graph task, not just the device: a backward that raises after queueing drops its
# callbacks, and a stale device-only entry would stop every later backward from joining.
_WGRAD_PENDING = set()


def _wgrad_stream(device) -> torch.cuda.Stream:
    st = _WGRAD_STREAMS.get(device)
    if st is None:
        st = _WGRAD_STREAMS.setdefault(device, torch.cuda.Stream(device=device))
    return st


def _join_wgrad(device, key):
    """End of the backward pass: the caller's stream waits for the parameter-gradient
    stream, so every consumer of .grad (clip, optimizer, user code) sees them done."""
    _WGRAD_PENDING.discard(key)
    torch.cuda.current_stream(device).wait_stream(_wgrad_stream(device))


# parameter -> the live forward records (TBlockFn contexts) that use it.  A late .grad
# write is safe only for a parameter that exactly one pending TemporalBlock backward uses:
# with two (the model run twice before one backward, a shared weight) the other use's
# AccumulateGrad would add into a gradient that the late write then overwrites.
# Keyed by id(parameter) with a weak reference to it (a WeakKeyDictionary would compare
# tensors with ==); an entry whose parameter died is replaced on the next registration.
_USES = {}


class _Use:
    """Token held by one TBlockFn context; dies with its autograd graph, or is spent
    (dead) at the end of the backward pass that ran the context's backward."""
    __slots__ = ("__weakref__", "dead")

    def __init__(self):
        self.dead = False


def _register_uses(ctx, params):
    ctx.use_token = tok = _Use()
    for p in params:
        e = _USES.get(id(p))
        if e is None or e[0]() is not p:
            e = _USES[id(p)] = (weakref.ref(p), weakref.WeakSet())
        e[1].add(tok)


def _pending_uses(p) -> int:
    e = _USES.get(id(p))
    return sum(1 for t in e[1] if not t.dead) if e is not None and e[0]() is p else 0


DEFERRED_BLOCKS = 0   # block backwards that took the deferred path (tests, bench)

# parameters whose gradients a post-backward exchange (ctn_dist.FlatGradAllReduce)
# consumes: id -> (weak reference, the exchange's persistent gradient view or None); under
# torch.distributed only these may be written late, and a deferred block backward writes
# their gradients straight into the exchange's buffer
_SYNCED = {}


def register_synced_after_backward(params, grad_views=None):
    for i, p in enumerate(params):
        # the view by weak reference: the exchange object owns its buffer
        _SYNCED[id(p)] = (weakref.ref(p), None if grad_views is None else weakref.ref(grad_views[i]))


def _synced_after_backward(p) -> bool:
    e = _SYNCED.get(id(p))
    return e is not None and e[0]() is p


def _grad_buffer(p):
    """A new gradient for parameter p: its view of the exchange buffer, or fresh memory."""
    e = _SYNCED.get(id(p))
    if e is not None and e[1] is not None and e[0]() is p:
        v = e[1]()
        if v is not None:
            return v
    return torch.empty_like(p)


class _TaskState:
    """What one backward pass (device, autograd graph task) leaves for its end: the
    contexts whose parameter uses it spent, and its deferred block backwards (entries
    before `flushed` were already reduced for an exchange hook)."""
    __slots__ = ("tokens", "deferred", "flushed")

    def __init__(self):
        self.tokens, self.deferred = [], []   # weak references: a dropped graph's tokens die
        self.flushed = 0


# Post-backward gradient exchanges that overlap the backward pass (ctn_dist.FlatGradAllReduce
# with chunks > 1): device -> hook.  Every `hook.group_blocks` deferred block backwards the
# pass reduces those blocks' gradients at once (instead of all at the pass's end) and calls
# hook.on_reduced(params), so the exchange can all-reduce them while the rest of the
# backward runs.
_EXCHANGE_HOOKS = {}


def register_exchange_hook(device, hook):
    _EXCHANGE_HOOKS[torch.device(device)] = hook


def unregister_exchange_hook(device, hook):
    if _EXCHANGE_HOOKS.get(torch.device(device)) is hook:
        del _EXCHANGE_HOOKS[torch.device(device)]


def _reduce_entries(entries):
    """One batched reduction (ctn_tblock_reduce_grads) of deferred block backwards."""
    if not entries:
        return
    lib = L.load()
    n = len(entries)
    descs = (L.TBlockDesc * n)(*[e[0] for e in entries])
    grads = (L.TBlockGrads * n)(*[e[1] for e in entries])
    parts = (ctypes.c_void_p * n)(*[e[2].data_ptr() for e in entries])
    L.check(lib.ctn_tblock_reduce_grads(descs, grads, parts, n, entries[0][4]), "ctn_tblock_reduce_grads")


_TASKS = {}


def _nested_backward() -> bool:
    """This thread is running a backward pass from inside another one's node (a reentrant
    torch.utils.checkpoint, a Function whose backward calls autograd): the outer pass's
    torch.autograd backward entry is on this thread's Python stack.  A top-level pass runs
    its nodes on the engine's device thread, whose stack holds no such frame."""
    f = sys._getframe(1)
    while f is not None:
        if f.f_code.co_name in ("_engine_run_backward", "run_backward") and "autograd" in f.f_code.co_filename:
            return True
        f = f.f_back
    return False


def _task_state(dev) -> "_TaskState":
    key = (dev, torch._C._current_graph_task_id())
    st = _TASKS.get(key)
    if st is None:
        # State of another pass on this device: the pass around this one (nested: keep it,
        # it ends after this one) or a pass that raised before its end (top-level: drop it;
        # its callback never ran).  The stack walk runs only in that rare case.
        others = [k for k in _TASKS if k[0] == dev]
        nested = bool(others) and _nested_backward()
        if others and not nested:
            for k in others:
                del _TASKS[k]
        st = _TASKS[key] = _TaskState()
        hook = _EXCHANGE_HOOKS.get(dev)
        if hook is not None and not nested:
            hook.on_pass_start()   # a second pass before the exchange's sync(): no early chunks
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _end_of_backward(key))
    return st


def _end_of_backward(key):
    """End of the backward pass: every deferred block's parameter gradients in one batched
    reduction, on the stream the block backwards ran on, before any consumer of .grad; then
    the pass's parameter uses are spent (a graph kept alive by a returned loss must not
    count as a pending use in the next step; released here and not at each node, because
    an immediate node's gradient is accumulated only after the node returns)."""
    # only this pass's own state: a nested pass ends before the pass around it, whose
    # deferred blocks must survive it (stale state of a raised pass is dropped by the next
    # top-level pass, _task_state)
    st = _TASKS.pop(key, None)
    if st is None:
        return
    _reduce_entries(st.deferred[st.flushed:])
    for r in st.tokens:
        t = r()
        if t is not None:
            t.dead = True


def _grads_unobserved(ctx) -> bool:
    """.grad of this block's parameters may be written late (after this node) only when
    nothing can observe the gradients before the backward pass ends: a plain
    .backward() that will accumulate into every one of these leaves (not
    autograd.grad), no gradient yet (no accumulation), no hooks, fp32 contiguous
    leaves; under torch.distributed only parameters a post-backward exchange consumes
    (ctn_dist.FlatGradAllReduce: DDP's hooks read gradients as they arrive)."""
    if torch.is_grad_enabled() or not hasattr(ctx, "param_refs"):
        return False
    dist_on = torch.distributed.is_available() and torch.distributed.is_initialized()
    for p, node in zip(ctx.param_refs, ctx.acc_nodes):
        if dist_on and not _synced_after_backward(p):
            return False
        if _pending_uses(p) != 1:    # another pending use of this parameter
            return False
        if (node is None or p.grad is not None or p.dtype != torch.float32 or not p.is_contiguous()
                or p._backward_hooks or getattr(p, "_post_accumulate_grad_hooks", None)):
            return False
        try:
            if not torch._C._will_engine_execute_node(node):
                return False
        except RuntimeError:   # autograd.grad() with these leaves as inputs
            return False
    return True


def _split_ok(ctx) -> bool:
    """The parameter-gradient tail may run on the side stream and write .grad directly
    only when the gradients are unobservable until the backward pass ends."""
    return ctx.wgrad_split and _grads_unobserved(ctx)


class TBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, fr: Frames, cfg: tuple, pack, bn, w1, a1, g1, b1, wd, a2, g2, b2, w2):
        """pack: (w1s, w2s, w1t, w2t, w1f, w2f, w1tf, w2tf, buf) bf16 copies from
        WeightPacks, or None.
        bn: BatchNorm state for norm_type BN (bn_state()), else None.
        cfg[6] (optional, ConvTasNet.wgrad_stream): let the backward run its
        parameter-gradient tail on a second stream when that is unobservable (_split_ok).
        cfg[7] (optional, ConvTasNet.defer_grad_reduce): leave the parameter-gradient
        reductions to one batched call at the end of the backward pass when that is
        unobservable (_grads_unobserved; not with the side stream).
        cfg[8] (optional): the parameters' AccumulateGrad nodes, cached by the caller."""
        B, H, P, dil, causal, norm = cfg[:6]
        ctx.wgrad_split = len(cfg) > 6 and bool(cfg[6])
        ctx.defer = len(cfg) > 7 and bool(cfg[7]) and norm != L.NORM_BN
        if ctx.wgrad_split or ctx.defer:
            ctx.param_refs = (w1, a1, g1, b1, wd, a2, g2, b2, w2)
            # cfg[8]: the nodes cached by the module (conv_tasnet.TemporalBlock._acc_nodes)
            nodes = cfg[8] if len(cfg) > 8 else None
            ctx.acc_nodes = nodes if nodes is not None else tuple(
                torch.autograd.graph.get_gradient_edge(t).node if t.requires_grad and t.is_leaf else None
                for t in ctx.param_refs)
            _register_uses(ctx, ctx.param_refs)
        lib = L.load()
        L.require_device(x, "TemporalBlock")
        x = x.contiguous()
        params = [_f32(t) for t in (w1, a1, g1, b1, wd, a2, g2, b2, w2)]
        desc = L.TBlockDesc(fr.M, fr.K, fr.Kp, B, H, P, dil, int(causal), norm, L.dtype_code(x.dtype))
        pack = pack if x.dtype == torch.bfloat16 else None
        ctx.pack = pack          # (8 pointers, buf): keeps the packed storage alive until backward
        ctx.bn = bn or _NO_BN
        pstruct = L.TBlockParams(*[p.data_ptr() for p in params], *(pack[:4] if pack else (None,) * 4), *ctx.bn,
                                 *(pack[4:8] if pack else (None,) * 4))
        y = torch.empty_like(x)
        h1 = x.new_empty(fr.rows, H)
        d = x.new_empty(fr.rows, H)
        stats = torch.empty(lib.ctn_tblock_stats_floats(ctypes.byref(desc)), dtype=torch.float32,
                            device=x.device)
        saved = L.TBlockSaved(h1.data_ptr(), d.data_ptr(), stats.data_ptr())
        nb = lib.ctn_tblock_workspace_bytes(ctypes.byref(desc), 0)
        ws = L.workspace(nb, x.device)
        L.check(lib.ctn_tblock_forward(ctypes.byref(desc), ctypes.byref(pstruct), x.data_ptr(), y.data_ptr(),
                                       ctypes.byref(saved), ws.data_ptr(), nb, L.stream_handle(x.device)),
                "ctn_tblock_forward")
        ctx.desc = (fr.M, fr.K, fr.Kp, B, H, P, dil, int(causal), norm, L.dtype_code(x.dtype))
        ctx.save_for_backward(x, h1, d, stats, *params)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = L.load()
        x, h1, d, stats, *params = ctx.saved_tensors
        gy = gy.contiguous()
        if gy.dtype != x.dtype:
            gy = gy.to(x.dtype)
        desc = L.TBlockDesc(*ctx.desc)
        pstruct = L.TBlockParams(*[p.data_ptr() for p in params], *(ctx.pack[:4] if ctx.pack else (None,) * 4),
                                 *ctx.bn, *(ctx.pack[4:8] if ctx.pack else (None,) * 4))
        saved = L.TBlockSaved(h1.data_ptr(), d.data_ptr(), stats.data_ptr())
        gx = torch.empty_like(x)
        late_ok = (ctx.defer or ctx.wgrad_split) and _grads_unobserved(ctx)
        if getattr(ctx, "use_token", None) is not None:
            _task_state(x.device).tokens.append(weakref.ref(ctx.use_token))   # spent at the pass's end
        if ctx.defer and not ctx.wgrad_split and late_ok:
            grads = [_grad_buffer(p) for p in ctx.param_refs]
            gstruct = L.TBlockGrads(*[g.data_ptr() for g in grads])
            return TBlockFn._backward_deferred(ctx, lib, desc, pstruct, saved, x, gy, gx, grads, gstruct)
        grads = [torch.empty_like(p) for p in params]
        gstruct = L.TBlockGrads(*[g.data_ptr() for g in grads])
        nb = lib.ctn_tblock_workspace_bytes(ctypes.byref(desc), 1)
        ws = L.workspace(nb, x.device)
        if not (ctx.wgrad_split and late_ok):
            L.check(lib.ctn_tblock_backward(ctypes.byref(desc), ctypes.byref(pstruct), x.data_ptr(),
                                            ctypes.byref(saved), gy.data_ptr(), gx.data_ptr(), ctypes.byref(gstruct),
                                            ws.data_ptr(), nb, L.stream_handle(x.device)),
                    "ctn_tblock_backward")
            return (gx, None, None, None, None, *grads)
        # the dW1 GEMM and the parameter-gradient reductions overlap the next block's
        # backward on the side stream; they read x and ws and write the gradients, whose
        # memory the caching allocator must not hand out again before they finish
        side = _wgrad_stream(x.device)
        L.check(lib.ctn_tblock_backward_split(ctypes.byref(desc), ctypes.byref(pstruct), x.data_ptr(),
                                              ctypes.byref(saved), gy.data_ptr(), gx.data_ptr(),
                                              ctypes.byref(gstruct), ws.data_ptr(), nb, L.stream_handle(x.device),
                                              side.cuda_stream),
                "ctn_tblock_backward_split")
        for t in (x, ws, *grads):
            t.record_stream(side)
        for p, g in zip(ctx.param_refs, grads):
            p.grad = g
        key = (x.device, torch._C._current_graph_task_id())
        if key not in _WGRAD_PENDING:
            _WGRAD_PENDING.add(key)
            dev = x.device
            torch.autograd.Variable._execution_engine.queue_callback(lambda: _join_wgrad(dev, key))
        return (gx, None, None, None, None) + (None,) * 9

    @staticmethod
    def _backward_deferred(ctx, lib, desc, pstruct, saved, x, gy, gx, grads, gstruct):
        """gx now; the parameter gradients' partials go to their own buffer and one batched
        reduction at the end of the backward pass writes .grad (_end_of_backward)."""
        global DEFERRED_BLOCKS
        DEFERRED_BLOCKS += 1
        dev = x.device
        stream = L.stream_handle(dev)
        nb = lib.ctn_tblock_deferred_workspace_bytes(ctypes.byref(desc))
        ws = L.workspace(nb, dev)
        npart = lib.ctn_tblock_partials_bytes(ctypes.byref(desc))
        part = L.workspace(npart, dev)
        L.check(lib.ctn_tblock_backward_deferred(ctypes.byref(desc), ctypes.byref(pstruct), x.data_ptr(),
                                                 ctypes.byref(saved), gy.data_ptr(), gx.data_ptr(),
                                                 ctypes.byref(gstruct), ws.data_ptr(), nb, part.data_ptr(), npart,
                                                 stream),
                "ctn_tblock_backward_deferred")
        for p, g in zip(ctx.param_refs, grads):
            p.grad = g
        # the partials, gradients and their descriptors stay alive until they are reduced
        st = _task_state(dev)
        st.deferred.append((L.TBlockDesc(*ctx.desc), gstruct, part, grads, stream, ctx.param_refs))
        hook = _EXCHANGE_HOOKS.get(dev)
        if hook is not None and len(st.deferred) - st.flushed >= hook.group_blocks:
            group = st.deferred[st.flushed:]
            _reduce_entries(group)
            st.deferred[st.flushed:] = [None] * len(group)   # partials: free once enqueued
            st.flushed = len(st.deferred)
            hook.on_reduced([p for e in group for p in e[5]])
        return (gx, None, None, None, None) + (None,) * 9


# ----------------------------------------------------------------------------
# layout helpers for standalone (sub)module calls: reference NCW <-> frame rows
# ----------------------------------------------------------------------------
def ncw_to_rows(x: torch.Tensor, fr: Frames, dtype) -> torch.Tensor:
    """[M, C, K] -> [M*Kp, C] with zero padded rows."""
    M, C, K = x.shape
    out = x.new_zeros(M, fr.Kp, C, dtype=dtype)
    out[:, :K].copy_(x.transpose(1, 2))
    return out.view(M * fr.Kp, C)


def rows_to_ncw(r: torch.Tensor, fr: Frames, dtype=None) -> torch.Tensor:
    C = r.shape[1]
    t = r.view(fr.M, fr.Kp, C)[:, :fr.K].transpose(1, 2)
    return t.to(dtype) if dtype is not None else t


# ----------------------------------------------------------------------------
# front: Encoder (conv_tasnet.py:97-117) + separator cLN (:167) + bottleneck (:169)
# ----------------------------------------------------------------------------
def codec_desc(fr: Frames, T, N, Lf, B, C, mask_type, dtype):
    return L.CodecDesc(fr.M, T, fr.K, fr.Kp, N, Lf, B, C, mask_type, L.dtype_code(dtype))


class EncoderFn(torch.autograd.Function):
    """mixture [M,T] fp32 -> (w_rows [M*Kp,N], x0 [M*Kp,B] or None).  Wb None: encoder only."""

    @staticmethod
    def forward(ctx, mixture, fr: Frames, geo: tuple, act_dtype, U, gamma0, beta0, Wb):
        N, Lf, B, C = geo
        lib = L.load()
        L.require_device(mixture, "Encoder")
        mixture = _f32(mixture)
        T = mixture.shape[-1]
        U = _f32(U)
        has_b = Wb is not None
        g0, b0, wb = (_f32(gamma0), _f32(beta0), _f32(Wb)) if has_b else (None, None, None)
        desc = codec_desc(fr, T, N, Lf, B if has_b else 8, C, L.MASK_RELU, act_dtype)
        dev = mixture.device
        w_rows = torch.empty(fr.rows, N, dtype=act_dtype, device=dev)
        stats = torch.empty(fr.rows, 2, dtype=torch.float32, device=dev) if has_b else None
        x0 = torch.empty(fr.rows, B, dtype=act_dtype, device=dev) if has_b else None
        nb = lib.ctn_encoder_workspace_bytes(ctypes.byref(desc), 0)
        ws = L.workspace(nb, dev)
        L.check(lib.ctn_encoder_forward(ctypes.byref(desc), mixture.data_ptr(), U.data_ptr(), L.ptr(g0), L.ptr(b0),
                                        L.ptr(wb), w_rows.data_ptr(), L.ptr(stats), L.ptr(x0), ws.data_ptr(), nb,
                                        L.stream_handle(dev)), "ctn_encoder_forward")
        ctx.desc = tuple(getattr(desc, f) for f, _ in L.CodecDesc._fields_)
        ctx.has_b = has_b
        ctx.save_for_backward(mixture, U, g0, b0, wb, w_rows, stats)
        if not has_b:
            return w_rows, w_rows.new_empty(0)
        return w_rows, x0

    @staticmethod
    def backward(ctx, g_w, g_x0):
        lib = L.load()
        mixture, U, g0, b0, wb, w_rows, stats = ctx.saved_tensors
        desc = L.CodecDesc(*ctx.desc)
        dev = mixture.device
        if g_w is not None:
            g_w = g_w.to(w_rows.dtype).contiguous()
        if not ctx.has_b or g_x0 is None or g_x0.numel() == 0:
            g_x0 = None
        else:
            g_x0 = g_x0.to(w_rows.dtype).contiguous()
        gU = torch.empty_like(U)
        gg0 = torch.empty_like(g0) if g_x0 is not None else None
        gb0 = torch.empty_like(b0) if g_x0 is not None else None
        gwb = torch.empty_like(wb) if g_x0 is not None else None
        nb = lib.ctn_encoder_workspace_bytes(ctypes.byref(desc), 1)
        ws = L.workspace(nb, dev)
        L.check(lib.ctn_encoder_backward(ctypes.byref(desc), mixture.data_ptr(), U.data_ptr(), L.ptr(g0),
                                         L.ptr(b0), L.ptr(wb), w_rows.data_ptr(), L.ptr(stats), L.ptr(g_w),
                                         L.ptr(g_x0), gU.data_ptr(), L.ptr(gg0), L.ptr(gb0), L.ptr(gwb),
                                         ws.data_ptr(), nb, L.stream_handle(dev)), "ctn_encoder_backward")
        if ctx.has_b and g_x0 is None:        # bottleneck output unused: zero grads
            gg0, gb0, gwb = torch.zeros_like(g0), torch.zeros_like(b0), torch.zeros_like(wb)
        return None, None, None, None, gU, gg0, gb0, gwb


# ----------------------------------------------------------------------------
# back: mask conv (:185) + nonlinearity (:202-208) + Decoder (:120-142) + OLA + pad
# ----------------------------------------------------------------------------
class DecoderFn(torch.autograd.Function):
    """(x_last [M*Kp,B], w_rows [M*Kp,N]) -> est [M,C,T] fp32.
    Wm None: standalone Decoder; x_last then holds mask rows [M*Kp, C*N]."""

    @staticmethod
    def forward(ctx, x_last, w_rows, fr: Frames, geo: tuple, Wm, V):
        T, N, Lf, B, C, mask_type = geo
        lib = L.load()
        L.require_device(x_last, "Decoder")
        x_last, w_rows = x_last.contiguous(), w_rows.contiguous()
        V = _f32(V)
        wm = _f32(Wm) if Wm is not None else None
        desc = codec_desc(fr, T, N, Lf, B, C, mask_type, w_rows.dtype)
        dev = w_rows.device
        score = torch.empty(fr.rows, C * N, dtype=w_rows.dtype, device=dev) if wm is not None else None
        est = torch.empty(fr.M, C, T, dtype=torch.float32, device=dev)
        nb = lib.ctn_decoder_workspace_bytes(ctypes.byref(desc), 0)
        ws = L.workspace(nb, dev)
        L.check(lib.ctn_decoder_forward(ctypes.byref(desc), x_last.data_ptr(), w_rows.data_ptr(), L.ptr(wm),
                                        V.data_ptr(), L.ptr(score), est.data_ptr(), ws.data_ptr(), nb,
                                        L.stream_handle(dev)), "ctn_decoder_forward")
        ctx.desc = tuple(getattr(desc, f) for f, _ in L.CodecDesc._fields_)
        ctx.save_for_backward(x_last, w_rows, wm, V, score)
        return est

    @staticmethod
    def backward(ctx, g_est):
        lib = L.load()
        x_last, w_rows, wm, V, score = ctx.saved_tensors
        desc = L.CodecDesc(*ctx.desc)
        dev = w_rows.device
        g_est = _f32(g_est)
        g_x = torch.empty_like(x_last)
        g_w = torch.empty_like(w_rows)
        gwm = torch.empty_like(wm) if wm is not None else None
        gV = torch.empty_like(V)
        nb = lib.ctn_decoder_workspace_bytes(ctypes.byref(desc), 1)
        ws = L.workspace(nb, dev)
        L.check(lib.ctn_decoder_backward(ctypes.byref(desc), x_last.data_ptr(), w_rows.data_ptr(), L.ptr(wm),
                                         V.data_ptr(), L.ptr(score), g_est.data_ptr(), g_x.data_ptr(),
                                         g_w.data_ptr(), L.ptr(gwm), gV.data_ptr(), ws.data_ptr(), nb,
                                         L.stream_handle(dev)), "ctn_decoder_backward")
        return g_x, g_w, None, None, gwm, gV


# ----------------------------------------------------------------------------
# PIT SI-SNR loss (pit_criterion.py:12-113)
# ----------------------------------------------------------------------------
class PITFn(torch.autograd.Function):
    """(source, est, lengths) -> (loss, max_snr [M,1], est (masked in place), best perm idx,
    the reordered estimate [M,C,T] (pit_criterion.py:79-98, written by the same kernel pass
    that masks est))."""

    @staticmethod
    def forward(ctx, source, est, lengths):
        lib = L.load()
        L.require_device(est, "cal_loss")
        if source.shape != est.shape:
            raise AssertionError("source and estimate_source sizes differ")   # pit_criterion.py:34
        if est.dtype != torch.float32 or not est.is_contiguous():
            raise L.CtnLibraryError("estimate_source must be a contiguous float32 tensor")
        source = _f32(source)
        lengths = lengths.to(device=est.device, dtype=torch.int64).contiguous()
        M, C, T = est.shape
        desc = L.PitDesc(M, C, T)
        dev = est.device
        loss = torch.empty((), dtype=torch.float32, device=dev)
        max_snr = torch.empty(M, 1, dtype=torch.float32, device=dev)
        best = torch.empty(M, dtype=torch.int64, device=dev)
        coef = torch.empty(M, C, 4, dtype=torch.float32, device=dev)
        reordered = torch.empty_like(est)
        nb = lib.ctn_pit_workspace_bytes(ctypes.byref(desc))
        ws = L.workspace(nb, dev)
        L.check(lib.ctn_pit_forward(ctypes.byref(desc), source.data_ptr(), est.data_ptr(), lengths.data_ptr(),
                                    loss.data_ptr(), max_snr.data_ptr(), best.data_ptr(), reordered.data_ptr(),
                                    coef.data_ptr(), ws.data_ptr(), nb, L.stream_handle(dev)), "ctn_pit_forward")
        ctx.mark_dirty(est)
        ctx.mark_non_differentiable(best, reordered)
        # outputs the caller does not differentiate (max_snr, the masked estimate) arrive
        # in backward as None instead of zero-filled tensors
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(source, est, lengths, coef)
        return loss, max_snr, est, best, reordered

    @staticmethod
    def backward(ctx, g_loss, g_max_snr, g_est_out, _g_best, _g_reordered):
        lib = L.load()
        source, est, lengths, coef = ctx.saved_tensors
        M, C, T = est.shape
        desc = L.PitDesc(M, C, T)
        dev = est.device
        g_est = torch.empty_like(est)
        gl = _f32(g_loss.reshape(1)) if g_loss is not None else torch.zeros(1, device=dev)
        gm = _f32(g_max_snr.reshape(M)) if g_max_snr is not None else None
        L.check(lib.ctn_pit_backward(ctypes.byref(desc), source.data_ptr(), est.data_ptr(), lengths.data_ptr(),
                                     coef.data_ptr(), gl.data_ptr(), L.ptr(gm), g_est.data_ptr(),
                                     L.stream_handle(dev)), "ctn_pit_backward")
        if g_est_out is not None:   # the in-place mask's gradient: zero beyond each length
            mask = (torch.arange(T, device=dev).unsqueeze(0) < lengths.unsqueeze(1)).unsqueeze(1)
            g_est.addcmul_(g_est_out, mask)
        return None, g_est, None


# ----------------------------------------------------------------------------
# stand-alone separator layers on frame rows (ctn_layers.hip; include/ctn.h ABI v4):
# the module forwards of TemporalConvNet / DepthwiseSeparableConv / gLN / cLN when
# they are called on their own (conv_tasnet.py:192-209, 265-272, 319-329, 344-355)
# ----------------------------------------------------------------------------
def rows_desc(fr: Frames, C: int, dtype) -> "L.RowsDesc":
    return L.RowsDesc(fr.M, fr.K, fr.Kp, C, L.dtype_code(dtype))


class LayerNormFn(torch.autograd.Function):
    """rows [M*Kp, C] -> gLN / cLN rows (norm: L.NORM_GLN / L.NORM_CLN)."""

    @staticmethod
    def forward(ctx, x, fr: Frames, norm: int, gamma, beta):
        lib = L.load()
        L.require_device(x, "LayerNorm")
        x = x.contiguous()
        C = x.shape[1]
        g, b = _f32(gamma), _f32(beta)
        d = rows_desc(fr, C, x.dtype)
        y = torch.empty_like(x)
        G = fr.M if norm == L.NORM_GLN else fr.rows
        stats = torch.empty(G, 2, dtype=torch.float32, device=x.device)
        nb = lib.ctn_layernorm_workspace_bytes(ctypes.byref(d), norm, 0)
        ws = L.workspace(nb, x.device)
        L.check(lib.ctn_layernorm_forward(ctypes.byref(d), norm, x.data_ptr(), g.data_ptr(), b.data_ptr(),
                                          y.data_ptr(), stats.data_ptr(), ws.data_ptr(), nb,
                                          L.stream_handle(x.device)), "ctn_layernorm_forward")
        ctx.fr, ctx.norm = fr, norm
        ctx.save_for_backward(x, g, stats)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = L.load()
        x, g, stats = ctx.saved_tensors
        gy = gy.to(x.dtype).contiguous()
        d = rows_desc(ctx.fr, x.shape[1], x.dtype)
        gx = torch.empty_like(x)
        gg = torch.empty_like(g)
        gb = torch.empty_like(g)
        nb = lib.ctn_layernorm_workspace_bytes(ctypes.byref(d), ctx.norm, 1)
        ws = L.workspace(nb, x.device)
        L.check(lib.ctn_layernorm_backward(ctypes.byref(d), ctx.norm, x.data_ptr(), g.data_ptr(), stats.data_ptr(),
                                           gy.data_ptr(), gx.data_ptr(), gg.data_ptr(), gb.data_ptr(),
                                           ws.data_ptr(), nb, L.stream_handle(x.device)), "ctn_layernorm_backward")
        return gx, None, None, gg, gb


class PReLUFn(torch.autograd.Function):
    """rows -> nn.PReLU() rows (one shared alpha)."""

    @staticmethod
    def forward(ctx, x, fr: Frames, alpha):
        lib = L.load()
        L.require_device(x, "PReLU")
        x = x.contiguous()
        a = _f32(alpha)
        d = rows_desc(fr, x.shape[1], x.dtype)
        y = torch.empty_like(x)
        L.check(lib.ctn_prelu_forward(ctypes.byref(d), x.data_ptr(), a.data_ptr(), y.data_ptr(),
                                      L.stream_handle(x.device)), "ctn_prelu_forward")
        ctx.fr = fr
        ctx.save_for_backward(x, a)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = L.load()
        x, a = ctx.saved_tensors
        gy = gy.to(x.dtype).contiguous()
        d = rows_desc(ctx.fr, x.shape[1], x.dtype)
        gx = torch.empty_like(x)
        ga = torch.empty_like(a)
        nb = lib.ctn_prelu_workspace_bytes(ctypes.byref(d))
        ws = L.workspace(nb, x.device)
        L.check(lib.ctn_prelu_backward(ctypes.byref(d), x.data_ptr(), a.data_ptr(), gy.data_ptr(), gx.data_ptr(),
                                       ga.data_ptr(), ws.data_ptr(), nb, L.stream_handle(x.device)),
                "ctn_prelu_backward")
        return gx, None, ga


class DepthwiseFn(torch.autograd.Function):
    """rows -> depthwise dilated conv rows (reference padding; causal = + Chomp1d)."""

    @staticmethod
    def forward(ctx, x, fr: Frames, geo: tuple, w):
        P, dil, causal = geo
        lib = L.load()
        L.require_device(x, "DepthwiseConv")
        x = x.contiguous()
        wf = _f32(w)
        d = rows_desc(fr, x.shape[1], x.dtype)
        y = torch.empty_like(x)
        L.check(lib.ctn_depthwise_forward(ctypes.byref(d), P, dil, int(causal), x.data_ptr(), wf.data_ptr(),
                                          y.data_ptr(), L.stream_handle(x.device)), "ctn_depthwise_forward")
        ctx.fr, ctx.geo = fr, geo
        ctx.save_for_backward(x, wf)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = L.load()
        x, wf = ctx.saved_tensors
        P, dil, causal = ctx.geo
        gy = gy.to(x.dtype).contiguous()
        d = rows_desc(ctx.fr, x.shape[1], x.dtype)
        gx = torch.empty_like(x)
        gw = torch.empty_like(wf)
        nb = lib.ctn_depthwise_workspace_bytes(ctypes.byref(d), P)
        ws = L.workspace(nb, x.device)
        L.check(lib.ctn_depthwise_backward(ctypes.byref(d), P, dil, int(causal), x.data_ptr(), wf.data_ptr(),
                                           gy.data_ptr(), gx.data_ptr(), gw.data_ptr(), ws.data_ptr(), nb,
                                           L.stream_handle(x.device)), "ctn_depthwise_backward")
        return gx, None, None, gw


class Conv1x1Fn(torch.autograd.Function):
    """rows [.., C] -> rows [.., cout] of a bias-free 1x1 conv (weight [cout, C, 1])."""

    @staticmethod
    def forward(ctx, x, fr: Frames, w):
        lib = L.load()
        L.require_device(x, "Conv1x1")
        x = x.contiguous()
        wf = _f32(w)
        cout, C = wf.shape[0], x.shape[1]
        d = rows_desc(fr, C, x.dtype)
        y = x.new_empty(fr.rows, cout)
        nb = lib.ctn_conv1x1_workspace_bytes(ctypes.byref(d), cout, 0)
        ws = L.workspace(nb, x.device)
        L.check(lib.ctn_conv1x1_forward(ctypes.byref(d), cout, x.data_ptr(), wf.data_ptr(), y.data_ptr(),
                                        ws.data_ptr(), nb, L.stream_handle(x.device)), "ctn_conv1x1_forward")
        ctx.fr = fr
        ctx.save_for_backward(x, wf)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = L.load()
        x, wf = ctx.saved_tensors
        cout, C = wf.shape[0], x.shape[1]
        gy = gy.to(x.dtype).contiguous()
        d = rows_desc(ctx.fr, C, x.dtype)
        gx = torch.empty_like(x)
        gw = torch.empty_like(wf)
        nb = lib.ctn_conv1x1_workspace_bytes(ctypes.byref(d), cout, 1)
        ws = L.workspace(nb, x.device)
        L.check(lib.ctn_conv1x1_backward(ctypes.byref(d), cout, x.data_ptr(), wf.data_ptr(), gy.data_ptr(),
                                         gx.data_ptr(), gw.data_ptr(), ws.data_ptr(), nb,
                                         L.stream_handle(x.device)), "ctn_conv1x1_backward")
        return gx, None, gw


class MaskFn(torch.autograd.Function):
    """score rows [.., S*N] -> mask rows (ReLU, or softmax over the S speakers)."""

    @staticmethod
    def forward(ctx, score, fr: Frames, nspk: int, mask_type: int):
        lib = L.load()
        L.require_device(score, "mask")
        score = score.contiguous()
        d = rows_desc(fr, score.shape[1], score.dtype)
        mask = torch.empty_like(score)
        L.check(lib.ctn_mask_forward(ctypes.byref(d), nspk, mask_type, score.data_ptr(), mask.data_ptr(),
                                     L.stream_handle(score.device)), "ctn_mask_forward")
        ctx.fr, ctx.nspk, ctx.mask_type = fr, nspk, mask_type
        ctx.save_for_backward(score)
        return mask

    @staticmethod
    def backward(ctx, gm):
        lib = L.load()
        (score,) = ctx.saved_tensors
        gm = gm.to(score.dtype).contiguous()
        d = rows_desc(ctx.fr, score.shape[1], score.dtype)
        gs = torch.empty_like(score)
        L.check(lib.ctn_mask_backward(ctypes.byref(d), ctx.nspk, ctx.mask_type, score.data_ptr(), gm.data_ptr(),
                                      gs.data_ptr(), L.stream_handle(score.device)), "ctn_mask_backward")
        return gs, None, None, None
