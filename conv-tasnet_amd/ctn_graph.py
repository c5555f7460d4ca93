"""Whole training steps as HIP graphs (torch.cuda.CUDAGraph is a hipGraph on ROCm).

A training step of this package (forward, PIT loss, backward with the deferred
parameter-gradient reductions, clip, Adam) issues ~600 kernel launches from Python:
about 9 ms of host time per step at the paper configuration (tools/exp/host_phases.py).
Captured once, a replay is one graph launch and the host is off the critical path.
Nothing in the step synchronises or reads host memory from the device at replay time:
segment tables are written by kernels whose arguments carry them
(ctn_opt_write_segments), and Adam(capturable=True) keeps its step count and lr on the
device and computes the bias corrections there (ctn_adam_step_dev), so every replay is
the next step, with no step limit.

Errors: the wave-specialised kernels report a timed-out wait in the device error word
(CTN_DEVERR_SPIN, include/ctn.h), which eager steps check at the end of every backward
pass (ctn_tblock_reduce_grads) — a replay runs no host code, so ``replay()`` checks the
word itself every ``check_every`` replays (one stream synchronisation; 0 = never) and
``check()`` does it on demand.

Requirements (the CUDA-graph rules of torch.cuda.graph): inputs in static tensors (copy
each new batch into them), the optimizer built with capturable=True, the same shapes at
every replay, no torch.distributed exchange inside the step (one process, one GPU).
A schedule that changes lr between replays writes ``opt.lr_tensor(group)`` (outside
the graph); betas are captured as kernel arguments (change them, then capture again).
"""
import torch

import ctn_lib as L


class StepGraph:
    """Captures ``step_fn`` (no arguments, returns the tensors to keep) after ``warmup``
    eager calls on a side stream, as torch.cuda.graph requires; ``replay()`` runs one
    more step and returns the captured outputs (overwritten in place by each replay)."""

    def __init__(self, step_fn, warmup: int = 2, check_every: int = 100):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                step_fn()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.outputs = step_fn()
        self.warmup = warmup
        self.check_every = int(check_every)
        self.replays = 0

    def check(self):
        """Synchronise the current stream and raise (CtnLibraryError) if a kernel of any
        earlier replay set a device error bit (ctn_device_status)."""
        stream = torch.cuda.current_stream()
        L.check(L.load().ctn_device_status(L.c_void_p(stream.cuda_stream), None, 0), "ctn_device_status")

    def replay(self):
        self.graph.replay()
        self.replays += 1
        if self.check_every > 0 and self.replays % self.check_every == 0:
            self.check()
        return self.outputs
