"""Data-parallel gradient exchange after the backward pass (one process per GPU,
torch.distributed over RCCL).

The reference trains data-parallel with nn.DataParallel (src/train.py:120-122): the
batch is split over the GPUs and the replicas' parameter gradients are summed onto one
device before the optimizer step (src/solver.py:178-186).  Here each rank holds a
replica and its shard of the global batch, and the gradients are averaged across ranks
before clip + Adam.  DistributedDataParallel does that with hooks that read each
gradient as it arrives during backward, which forces every TemporalBlock backward to
write its parameter gradients immediately (68 reduction launches per step at the bench
shape) instead of the batched reductions of the deferred path
(ConvTasNet.defer_grad_reduce, ctn_ops._end_of_backward).  ``FlatGradAllReduce``
owns one persistent gradient buffer in which every parameter has a view; the deferred
block backwards write their gradients straight into it.

Chunked exchange (default 4 chunks): the deferred blocks are reduced in groups during
the backward pass (ctn_ops exchange hook: every ``group_blocks`` block backwards), and
each group's contiguous slice of the buffer is all-reduced asynchronously (RCCL's own
stream) as soon as it is final, while the backward of the earlier blocks goes on; what
is left when ``backward()`` returns (the first blocks, the encoder, bottleneck, mask and
decoder gradients) is one more all-reduce in :meth:`sync`.  The layout is learnt in the
first step, in which every deferred block is reduced and reported on its own: the
reported blocks in report order, split into ``chunks - 1`` groups of consecutive blocks,
then everything else, so every chunk is one contiguous message (at the paper
configuration 4 messages of ≈8.7 MB, still large enough for the point-to-point xGMI
rings).  Chunks go out in the same order on every rank.  ``chunks=1`` is one all-reduce
of the whole buffer after backward.

Averaging matches DDP's: every gradient is divided by the world size, then summed
across ranks (exact for power-of-two world sizes), so both give the same bits.

An early chunk is all-reduced out of place (a scaled copy of the slice), so the views
keep this rank's local gradients until :meth:`sync` copies the reduced values in.  A
second backward pass before ``sync()`` (gradient accumulation, or a step abandoned
without ``sync()``) therefore finds its views untouched by RCCL: the pass waits for the
early chunks, drops them and turns the overlap off until the next ``sync()``, which
all-reduces the whole buffer once (ctn_ops calls :meth:`on_pass_start`).

The learnt layout decides the sequence of all-reduces every rank issues, so after it is
learnt the ranks compare it (a hash of every chunk's parameter list, one all-reduce)
and all raise if any rank learnt another one, instead of deadlocking in RCCL.
"""
import hashlib

import torch
import torch.distributed as dist
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

import ctn_ops


class FlatGradAllReduce:
    """Averages the ``.grad`` of ``params`` across the ranks of ``group`` after the
    backward pass; call :meth:`sync` between ``loss.backward()`` and the optimizer.

    On construction the parameters are broadcast from rank 0 (every replica starts from
    the same weights, as DDP's constructor does) and registered with ctn_ops as consumed
    after backward, which lets the TemporalBlock backwards defer their gradient
    reductions under torch.distributed.  Do not also wrap the same parameters in
    DistributedDataParallel: its hooks read gradients during backward."""

    LEARN = 1   # group_blocks while the layout is learnt: every block reported on its own

    def __init__(self, params, group=None, chunks=4):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("FlatGradAllReduce: torch.distributed is not initialized")
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group)
        self.chunks = max(1, int(chunks))
        with torch.no_grad():
            for bucket in self._buckets(self.params):
                flat = _flatten_dense_tensors(bucket)
                dist.broadcast(flat, src=dist.get_global_rank(group, 0) if group is not None else 0,
                               group=group)
                for p, v in zip(bucket, _unflatten_dense_tensors(flat, bucket)):
                    p.copy_(v)
        self._layout(self._buckets(self.params), None)
        self._reported = []     # this step's hook reports (lists of parameters), in order
        self._final = set()     # ids of parameters final in their views this step
        self._launched = {}     # (arena, chunk) -> (async all-reduce work, reduced copy, view slice)
        self._passes = 0        # backward passes since the last sync()
        self._accumulating = False   # a second pass before sync(): no early chunks this step
        self._learnt = False
        self.early_chunks = 0   # chunks all-reduced during a backward pass (overlapped)
        self._hook_devs = []
        self.group_blocks = self.LEARN
        if self.chunks > 1:
            for bucket in self._buckets(self.params):
                if bucket[0].is_cuda and bucket[0].device not in self._hook_devs:
                    ctn_ops.register_exchange_hook(bucket[0].device, self)
                    self._hook_devs.append(bucket[0].device)

    def close(self):
        """Stop overlapping with the backward pass (unregister the ctn_ops hook)."""
        for d in self._hook_devs:
            ctn_ops.unregister_exchange_hook(d, self)
        self._hook_devs = []

    def _layout(self, buckets, bounds):
        """One persistent gradient buffer per (device, dtype) bucket, in the bucket's
        parameter order, each parameter owning a view; bounds[i] = the chunks of bucket i
        as (first, end) parameter index ranges (None: one chunk)."""
        self._arenas = []
        views = {}
        for i, g in enumerate(buckets):
            flat = torch.empty(sum(p.numel() for p in g), device=g[0].device, dtype=g[0].dtype)
            vs = _unflatten_dense_tensors(flat, g)
            offs = [0]
            for p in g:
                offs.append(offs[-1] + p.numel())
            chunks = bounds[i] if bounds is not None else [(0, len(g))]
            self._arenas.append((g, flat, vs, [(a, b, offs[a], offs[b]) for a, b in chunks]))
            views.update({id(p): v for p, v in zip(g, vs)})
        ctn_ops.register_synced_after_backward(self.params, [views[id(p)] for p in self.params])

    @staticmethod
    def _buckets(tensors):
        by = {}
        for t in tensors:
            by.setdefault((t.device, t.dtype), []).append(t)
        return list(by.values())

    # ---- ctn_ops exchange hook (called from the backward pass, in block order)
    def on_pass_start(self):
        """A backward pass begins (ctn_ops: the pass's first TemporalBlock backward).  If an
        earlier pass since the last sync() already ran (gradient accumulation, or a step
        abandoned without sync()), its early chunks are waited for and dropped — their views
        still hold the local gradients — and this step exchanges everything in sync()."""
        self._passes += 1
        if self._passes > 1:
            self._drop_early()
            self._accumulating = True

    def _drop_early(self):
        for work, _, _ in self._launched.values():
            work.wait()               # RCCL is done with the reduced copies before they are freed
        self._launched, self._final, self._reported = {}, set(), []

    def on_reduced(self, params):
        """A group of deferred blocks' gradients is final, in place in their views: launch
        every chunk, in order, whose parameters are all final."""
        if self._accumulating:
            return
        self._reported.append(list(params))
        self._final.update(id(p) for p in params)
        if self._learnt:
            self._launch(final_only=True)

    def _launch(self, final_only):
        for ai, (g, flat, vs, chunks) in enumerate(self._arenas):
            for ci, (a, b, o0, o1) in enumerate(chunks):
                if (ai, ci) in self._launched:
                    continue
                if final_only and not all(id(p) in self._final for p in g[a:b]):
                    return            # in order: every rank issues the same sequence
                part = flat[o0:o1]
                if final_only:
                    # out of place: the views keep the local gradients until sync()
                    red = part / self.world
                    self._launched[(ai, ci)] = (dist.all_reduce(red, group=self.group, async_op=True), red, part)
                    self.early_chunks += 1
                else:
                    self._gather(g[a:b], vs[a:b])
                    part.div_(self.world)
                    self._launched[(ai, ci)] = (dist.all_reduce(part, group=self.group, async_op=True), None, None)

    @staticmethod
    def _gather(params, views):
        for p, v in zip(params, views):
            g = p.grad
            if g is v:               # written in place by a deferred block backward
                continue
            if g is None:
                v.zero_()            # an unused parameter contributes zeros (as DDP)
            else:                    # accumulated elsewhere (encoder, decoder, ...)
                v.copy_(g)

    @torch.no_grad()
    def sync(self):
        """All-reduce (mean) every parameter gradient; a parameter without a gradient on
        this rank contributes zeros (DDP's treatment of an unused parameter) and receives
        the mean.  Afterwards each ``p.grad`` is the parameter's view of the persistent
        buffer (as DDP's gradient_as_bucket_view makes them): keep a copy, not the tensor,
        to hold a gradient past the next step."""
        self._launch(final_only=False)
        for work, red, part in self._launched.values():
            work.wait()              # the current stream waits for RCCL's
            if red is not None:      # an early chunk, reduced out of place
                part.copy_(red)
        for g, flat, vs, _ in self._arenas:
            for p, v in zip(g, vs):
                p.grad = v
        # learnt collectively at the first sync() after a single-pass step (the layout check
        # is an all-reduce every rank joins: CUDA buckets always learn, whatever they reported)
        if not self._learnt and not self._accumulating and self.chunks > 1 and (self._hook_devs or self._reported):
            self._learn()
        self._reported, self._final, self._launched = [], set(), {}
        self._passes, self._accumulating = 0, False

    def _learn(self):
        """After the first step: the blocks the hook reported, in report order, in
        `chunks - 1` groups of consecutive blocks, then every other parameter."""
        blocks = [grp for grp in self._reported if grp]
        self._learnt = True
        if len(blocks) < 2:
            self.group_blocks = 1 << 30   # nothing to overlap: one exchange after backward
            self._check_layout()
            return
        per = -(-len(blocks) // (self.chunks - 1))
        self.group_blocks = per
        groups = [[p for grp in blocks[i:i + per] for p in grp] for i in range(0, len(blocks), per)]
        seen = {id(p) for grp in groups for p in grp}
        groups.append([p for p in self.params if id(p) not in seen])
        buckets, bounds = {}, {}
        for grp in groups:
            firsts = {}
            for p in grp:
                key = (p.device, p.dtype)
                lst = buckets.setdefault(key, [])
                firsts.setdefault(key, len(lst))
                lst.append(p)
            for key, a in firsts.items():
                bounds.setdefault(key, []).append((a, len(buckets[key])))
        keys = list(buckets)
        self._layout([buckets[k] for k in keys], [bounds[k] for k in keys])
        self._check_layout()

    def layout_signature(self):
        """A hash of the learnt layout: every chunk's parameters (as indices into the
        constructor's list), in the order the chunks are all-reduced."""
        idx = {id(p): i for i, p in enumerate(self.params)}
        desc = [(ai, [idx[id(p)] for p in g[a:b]]) for ai, (g, _, _, chunks) in enumerate(self._arenas)
                for a, b, _, _ in chunks]
        # 62 bits, non-negative: -h below stays inside int64
        return int.from_bytes(hashlib.sha1(repr(desc).encode()).digest()[:8], "little") >> 2

    def _check_layout(self):
        """Every rank must issue the same all-reduce sequence: compare the layout hashes
        (max of h and of -h over the ranks: equal iff every rank holds the same h) and
        raise on every rank if they differ, instead of deadlocking in RCCL later."""
        h = self.layout_signature()
        t = torch.tensor([h, -h], dtype=torch.int64, device=self.params[0].device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        hi, lo = int(t[0]), -int(t[1])
        if hi != h or lo != h:
            raise RuntimeError(
                "FlatGradAllReduce: the ranks learnt different gradient-chunk layouts in the first "
                f"step (this rank {h:#x}, max {hi:#x}, min {lo:#x}); their all-reduce sequences would "
                "not match.  Every rank must run the same model with the same deferred TemporalBlock "
                "backwards in its first step (or use chunks=1).")
