"""torch.autograd.Function wrappers around the C ABI (one native call per
forward and per backward).  Activations travel between ops in the frame-row
layout [M*Kp, C]; parameters stay fp32 in reference shapes."""
from __future__ import annotations

import ctypes
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
class TBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, fr: Frames, cfg: tuple, w1, a1, g1, b1, wd, a2, g2, b2, w2):
        B, H, P, dil, causal, norm = cfg
        lib = L.load()
        L.require_device(x, "TemporalBlock")
        x = x.contiguous()
        params = [_f32(t) for t in (w1, a1, g1, b1, wd, a2, g2, b2, w2)]
        desc = L.TBlockDesc(fr.M, fr.K, fr.Kp, B, H, P, dil, int(causal), norm, L.dtype_code(x.dtype))
        pstruct = L.TBlockParams(*[p.data_ptr() for p in params])
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
        pstruct = L.TBlockParams(*[p.data_ptr() for p in params])
        saved = L.TBlockSaved(h1.data_ptr(), d.data_ptr(), stats.data_ptr())
        gx = torch.empty_like(x)
        grads = [torch.empty_like(p) for p in params]
        gstruct = L.TBlockGrads(*[g.data_ptr() for g in grads])
        nb = lib.ctn_tblock_workspace_bytes(ctypes.byref(desc), 1)
        ws = L.workspace(nb, x.device)
        L.check(lib.ctn_tblock_backward(ctypes.byref(desc), ctypes.byref(pstruct), x.data_ptr(),
                                        ctypes.byref(saved), gy.data_ptr(), gx.data_ptr(), ctypes.byref(gstruct),
                                        ws.data_ptr(), nb, L.stream_handle(x.device)),
                "ctn_tblock_backward")
        return (gx, None, None, *grads)


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
