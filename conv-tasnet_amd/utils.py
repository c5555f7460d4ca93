"""Drop-in for ``src/utils.py``.

``overlap_and_add`` here is the standalone utility (any leading dims, any
frame_step <= frame_length).  The model's own overlap-add is fused into the
HIP decoder kernel (ctn_decoder_forward) and never calls this.  This version
is a deterministic gather (no index_add_ atomics, no per-call host->device
index copy, utils.py:39-44) and works on any device.
"""
from __future__ import annotations

import torch


def overlap_and_add(signal, frame_step):
    """utils.py:9-46: out[..., k*frame_step + j] += signal[..., k, j]."""
    *outer, frames, frame_length = signal.shape
    out_len = frame_step * (frames - 1) + frame_length
    out = signal.new_zeros(*outer, out_len)
    base = torch.arange(frames, device=signal.device) * frame_step
    for j0 in range(0, frame_length, frame_step):
        s = min(frame_step, frame_length - j0)
        # within one column group the target indices are unique: plain gather-add
        idx = (base + j0).unsqueeze(1) + torch.arange(s, device=signal.device)
        out[..., idx.reshape(-1)] += signal[..., j0:j0 + s].reshape(*outer, frames * s)
    return out


def remove_pad(inputs, inputs_lengths):
    """utils.py:49-66 -> list of numpy arrays [C, T_b] (or [T_b])."""
    results = []
    dim = inputs.dim()
    if dim == 3:
        C = inputs.size(1)
    for input, length in zip(inputs, inputs_lengths):
        if dim == 3:
            results.append(input[:, :length].view(C, -1).cpu().numpy())
        elif dim == 2:
            results.append(input[:length].view(-1).cpu().numpy())
    return results
