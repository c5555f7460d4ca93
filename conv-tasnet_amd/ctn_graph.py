"""Whole training steps as HIP graphs (torch.cuda.CUDAGraph is a hipGraph on ROCm).

A training step of this package (forward, PIT loss, backward with the deferred
parameter-gradient reductions, clip, Adam) issues ~600 kernel launches from Python:
about 9 ms of host time per step at the paper configuration (tools/exp/host_phases.py).
Captured once, a replay is one graph launch and the host is off the critical path.
Nothing in the step synchronises or reads host memory from the device at replay time:
segment tables are written by kernels whose arguments carry them
(ctn_opt_write_segments), and Adam(capturable=True) keeps its step count on the device
with a bias-correction table (ctn_adam_step_dev), so every replay is the next step.

Requirements (the CUDA-graph rules of torch.cuda.graph): inputs in static tensors (copy
each new batch into them), the optimizer built with capturable=True, the same shapes at
every replay, no torch.distributed exchange inside the step (one process, one GPU).
Changing lr or betas needs one eager step before the next capture
(ctn_optim.Adam._capture_state rebuilds the table outside capture).
"""
import torch


class StepGraph:
    """Captures ``step_fn`` (no arguments, returns the tensors to keep) after ``warmup``
    eager calls on a side stream, as torch.cuda.graph requires; ``replay()`` runs one
    more step and returns the captured outputs (overwritten in place by each replay)."""

    def __init__(self, step_fn, warmup: int = 2):
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

    def replay(self):
        self.graph.replay()
        return self.outputs
