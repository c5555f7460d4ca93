"""Data-parallel gradient exchange after the backward pass (one process per GPU,
torch.distributed over RCCL).

The reference trains data-parallel with nn.DataParallel (src/train.py:120-122): the
batch is split over the GPUs and the replicas' parameter gradients are summed onto one
device before the optimizer step (src/solver.py:178-186).  Here each rank holds a
replica and its shard of the global batch, and the gradients are averaged across ranks
before clip + Adam.  DistributedDataParallel does that with hooks that read each
gradient as it arrives during backward, which forces every TemporalBlock backward to
write its parameter gradients immediately (68 reduction launches per step at the bench
shape) instead of the one batched reduction at the end of the pass
(ConvTasNet.defer_grad_reduce, ctn_ops._end_of_backward).  ``FlatGradAllReduce``
consumes the gradients only after ``backward()`` returns, so the deferred reductions
stay on and write straight into its persistent gradient buffer, and exchanges that
buffer with ONE all-reduce per dtype: one ring all-reduce of the whole model (≈35 MB fp32 for the paper configuration) — a single large message is what
point-to-point xGMI rings move at full link rate.

Averaging matches DDP's: every gradient is divided by the world size, then summed
across ranks (exact for power-of-two world sizes), so both give the same bits.
"""
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

    def __init__(self, params, group=None):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("FlatGradAllReduce: torch.distributed is not initialized")
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group)
        with torch.no_grad():
            for bucket in self._buckets(self.params):
                flat = _flatten_dense_tensors(bucket)
                dist.broadcast(flat, src=dist.get_global_rank(group, 0) if group is not None else 0,
                               group=group)
                for p, v in zip(bucket, _unflatten_dense_tensors(flat, bucket)):
                    p.copy_(v)
        # one persistent gradient buffer per (device, dtype); each parameter owns a view.
        # The deferred TemporalBlock backwards write their gradients straight into it, so
        # after a backward pass most gradients are already in place.
        self._arenas = []
        views = {}
        for bucket in self._buckets(self.params):
            flat = torch.empty(sum(p.numel() for p in bucket), device=bucket[0].device, dtype=bucket[0].dtype)
            vs = _unflatten_dense_tensors(flat, bucket)
            self._arenas.append((bucket, flat, vs))
            views.update({id(p): v for p, v in zip(bucket, vs)})
        ctn_ops.register_synced_after_backward(self.params, [views[id(p)] for p in self.params])

    @staticmethod
    def _buckets(tensors):
        by = {}
        for t in tensors:
            by.setdefault((t.device, t.dtype), []).append(t)
        return list(by.values())

    @torch.no_grad()
    def sync(self):
        """All-reduce (mean) every parameter gradient; a parameter without a gradient on
        this rank contributes zeros (DDP's treatment of an unused parameter) and receives
        the mean.  Afterwards each ``p.grad`` is the parameter's view of the persistent
        buffer (as DDP's gradient_as_bucket_view makes them): keep a copy, not the tensor,
        to hold a gradient past the next step."""
        for bucket, flat, views in self._arenas:
            for p, v in zip(bucket, views):
                g = p.grad
                if g is v:               # written in place by a deferred block backward
                    continue
                if g is None:
                    v.zero_()
                else:                    # accumulated elsewhere (encoder, decoder, ...)
                    v.copy_(g)
                p.grad = v
            flat.div_(self.world)
            dist.all_reduce(flat, group=self.group)
