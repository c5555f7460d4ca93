"""Synthetic speech-like mixtures for benchmarks and smoke runs.

Each source: Gaussian noise through a random resonant AR(2) filter, times a
slow random envelope, unit RMS, random gain in [-2.5, 2.5] dB.  Mixture = sum
of sources.  Deterministic per seed (numpy PCG64); generated on the host once
and copied to the device before any timed region.
"""
from __future__ import annotations

import math

import numpy as np
import torch
from scipy.signal import lfilter


def speech_like(M: int, C: int, T: int, seed: int):
    """-> (mixture [M, T], sources [M, C, T]) float32 CPU tensors."""
    rng = np.random.default_rng(seed)
    src = np.empty((M, C, T), dtype=np.float32)
    t = np.arange(T)
    for m in range(M):
        for c in range(C):
            r, th = rng.uniform(0.85, 0.97), rng.uniform(0.05, 0.6)
            y = lfilter([1.0], [1.0, -2 * r * math.cos(th), r * r], rng.standard_normal(T))
            nk = max(2, T // 800)
            env = np.interp(t, np.linspace(0, T - 1, nk), np.abs(rng.standard_normal(nk)) + 0.1)
            y = y * env
            y /= np.sqrt(np.mean(y ** 2)) + 1e-12
            src[m, c] = y * 10 ** (rng.uniform(-2.5, 2.5) / 20)
    src_t = torch.from_numpy(src)
    return src_t.sum(1), src_t
