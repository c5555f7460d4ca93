"""Streaming (chunk-by-chunk) separation with a causal Conv-TasNet (SURVEY.md §8f
row 4): audio arrives in chunks of any length, separated audio leaves with a fixed
delay of one encoder stride, and the concatenated output equals
``ConvTasNet.forward`` on the whole signal (the reference's separate.py:35-79 run
on a causal model, conv_tasnet.py:176, 251-260, 289).

Why a causal model streams: with ``causal=True`` every operation is either per
frame (encoder, cLN, 1x1 convs, PReLU, mask and its nonlinearity, decoder basis)
or looks only BACKWARD in time (the dilated depthwise conv after Chomp1d reaches
(P-1)*d frames into the past).  gLN normalizes over the whole utterance and
cannot stream; BatchNorm streams in eval mode (running statistics, per frame).

State kept between chunks (all on the device, fp32), nothing re-run:
* ``samples``: input samples not yet consumed by a whole encoder frame;
* per TemporalBlock a RING of its depthwise-conv input frames (after conv1x1,
  PReLU and norm 1): a new frame is computed once, written to slot g % R, and
  read by the depthwise taps of the frames g .. g + (P-1)*d; taps before the
  stream start read as zero (the reference's causal zero padding);
* ``tail``: the last L/2 overlap-add samples of the previous chunk.

Per chunk of K new frames (cut into calls of at most ``max_frames``): one
``ctn_stream_call`` (include/ctn.h ABI v7, csrc/ctn_stream.hip): an encode kernel,
two kernels per TemporalBlock and two decode kernels, every 1x1 conv split over
32-output column chunks so a call with one new frame still spreads over many CUs —
work proportional to the NEW frames only, no padding of a call to 128-frame tiles.  Forward only (torch.no_grad);
the weights are snapshotted (transposed 1x1 weights, folded BatchNorm) when the
streamer is built or ``refresh_weights()`` is called.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

import ctn_lib as L
from conv_tasnet import ConvTasNet, _mask_code, _norm_code


def _t1x1(conv: nn.Conv1d) -> torch.Tensor:
    """Conv1d(cin, cout, 1).weight [cout, cin, 1] -> [cin, cout] fp32 contiguous."""
    return conv.weight.detach()[:, :, 0].t().contiguous().float()


def _norm_pair(norm: nn.Module):
    """cLN -> (gamma, beta); eval BatchNorm1d -> (scale, shift) with its running stats."""
    if isinstance(norm, nn.BatchNorm1d):
        scale = norm.weight.detach() / torch.sqrt(norm.running_var.detach() + norm.eps)
        return scale.float().contiguous(), (norm.bias.detach() - norm.running_mean.detach() * scale).float().contiguous()
    return norm.gamma.detach().reshape(-1).float().contiguous(), norm.beta.detach().reshape(-1).float().contiguous()


class StreamingSeparator:
    """Wraps a causal ConvTasNet for chunked inference.

    >>> s = StreamingSeparator(model)          # model.causal, norm_type cLN (or BN in eval)
    >>> outs = [s.push(chunk) for chunk in chunks]   # chunk [M, n] -> [M, C, m] (m may be 0)
    >>> outs.append(s.flush())                  # the last L/2 samples
    """

    def __init__(self, model: ConvTasNet, act_dtype=None, max_frames: int = 64):
        """act_dtype: None or torch.float32 — the stream kernels compute and keep their
        state in fp32 (the round-2 bf16 streamer was replaced; bf16 raises ValueError)."""
        if not model.causal:
            raise ValueError("streaming needs a causal model (ConvTasNet(causal=True))")
        norm = _norm_code(model.norm_type)
        if norm == L.NORM_GLN:
            raise ValueError("gLN normalizes over the whole utterance: a gLN model cannot stream")
        if norm == L.NORM_BN and model.training:
            raise ValueError("BatchNorm streams only in eval mode (running statistics)")
        if model.L % 2:
            raise ValueError("the encoder stride L//2 must tile the frame (even L)")
        if act_dtype not in (None, torch.float32):
            raise ValueError("streaming computes in fp32")
        self.model = model
        self.norm = norm
        self.stride = model.L // 2
        self.max_frames = int(max_frames)
        # one ctn_stream_call per chunk (ABI v7); False: the v5 per-stage entries
        self.one_call = True
        self.lib = L.load()
        self.refresh_weights()
        self.reset()

    def refresh_weights(self):
        """Snapshot the model's parameters in the layouts the stream kernels read."""
        m = self.model
        sep = m.separator
        cln, bott, _, mask = sep.network
        self.U = m.encoder.conv1d_U.weight.detach()[:, 0, :].float().contiguous()          # [N][L]
        self.g0, self.b0 = _norm_pair(cln)
        self.wb_t = _t1x1(bott)                                                             # [N][B]
        self.wm_t = _t1x1(mask)                                                             # [B][C*N]
        self.V = m.decoder.basis_signals.weight.detach().float().contiguous()              # [L][N]
        self.blocks = []
        for blk in sep.blocks():
            B, H, P, dil, _, _ = blk._geo
            ds = blk.net[3].net
            n1, n2 = blk._norms()
            a1, b1 = _norm_pair(n1)
            a2, b2 = _norm_pair(n2)
            self.blocks.append(dict(
                dil=dil, P=P, w1_t=_t1x1(blk.net[0]), alpha1=blk.net[1].weight.detach().float().contiguous(),
                n1a=a1, n1b=b1, wd=ds[0].weight.detach()[:, 0, :].float().contiguous(),
                alpha2=ds[2].weight.detach().float().contiguous(), n2a=a2, n2b=b2, w2_t=_t1x1(ds[4])))
        self.B, self.H = self.blocks[0]["w1_t"].shape if self.blocks else (bott.weight.shape[0], 0)
        # the ctn_stream_model holds pointers into this snapshot: rebuild it (the old
        # tensors are freed; a cached struct would hand the library dangling pointers)
        self._wver = getattr(self, "_wver", 0) + 1
        self._mkey = None

    def reset(self):
        self.samples = None          # [M, s] pending input samples
        self.rings = None            # per block [M, R, H]
        self._mkey = None
        self.tail = None             # [M, C, stride] pending overlap-add samples
        self.frames = 0              # frames emitted so far (= pos of the next frame)
        self._tails = None           # one_call: the tail ping-pong pair
        self._stage = {}             # one_call: (M, K, device) -> input / output / workspace buffers

    @property
    def latency_samples(self) -> int:
        """Output trails input by one stride: the last L/2 samples wait for the next frame."""
        return self.stride

    def _desc(self, M, K):
        m = self.model
        return L.StreamDesc(M, K, m.N, m.L, self.B, self.H, m.P, m.C,
                            L.NORM_CLN if self.norm == L.NORM_CLN else L.NORM_BN, _mask_code(m.mask_nonlinear))

    def _alloc(self, M, dev):
        self.rings = []
        for b in self.blocks:
            need = (b["P"] - 1) * b["dil"] + self.max_frames
            R = 1 << max(0, (need - 1).bit_length())
            self.rings.append(torch.zeros(M, R, self.H, device=dev))
        self.tail = torch.zeros(M, self.model.C, self.stride, device=dev)

    def _model_struct(self):
        """ctn_stream_model for ctn_stream_call (ABI v7): pointers into the snapshot and
        the rings, rebuilt when either changes."""
        key = (id(self.rings), self._wver)
        if getattr(self, "_mkey", None) != key:
            blocks = (L.StreamBlockParams * max(1, len(self.blocks)))()
            for i, (b, ring) in enumerate(zip(self.blocks, self.rings)):
                blocks[i] = L.StreamBlockParams(b["dil"], ring.shape[1],
                                                *(b[k].data_ptr() for k in ("w1_t", "alpha1", "n1a", "n1b", "wd",
                                                                            "alpha2", "n2a", "n2b", "w2_t")),
                                                ring.data_ptr())
            self._mblocks = blocks   # keeps the host array alive
            self._mstruct = L.StreamModel(self.U.data_ptr(), self.g0.data_ptr(), self.b0.data_ptr(),
                                          self.wb_t.data_ptr(), self.wm_t.data_ptr(), self.V.data_ptr(),
                                          ctypes.cast(blocks, ctypes.c_void_p), len(self.blocks))
            self._mkey = key
        return self._mstruct

    def _call(self, buf: torch.Tensor, K: int) -> torch.Tensor:
        """K frames whose samples start at buf[:, 0] -> [M, C, K*stride] finished samples:
        one ctn_stream_call (ABI v7: the whole network, 1x1 convs split over column chunks)."""
        m, lib = self.model, self.lib
        M, dev = buf.shape[0], buf.device
        d = self._desc(M, K)
        st = L.stream_handle(dev)
        if self.one_call:
            # persistent staging buffers per (M, K) and a tail pair per M: the library
            # replays one captured graph per argument set (ctn_stream_call), so equal
            # pointers from call to call make every call after the first a replay
            nb = lib.ctn_stream_workspace_bytes(ctypes.byref(d))
            sk = (M, K, dev)
            stg = self._stage.get(sk)
            if stg is None:
                # bounded like the library's graph cache (8 argument sets): chunk sizes
                # that keep changing must not grow device memory without limit
                while len(self._stage) >= 8:
                    self._stage.pop(next(iter(self._stage)))
                ns = (K - 1) * self.stride + m.L
                stg = self._stage[sk] = dict(inp=torch.empty(M, ns, device=dev),
                                             out=torch.empty(M, m.C, K * self.stride, device=dev),
                                             ws=torch.empty(nb, dtype=torch.uint8, device=dev))
            if self._tails is None or self._tails[0].shape != self.tail.shape:
                self._tails = [self.tail, torch.empty_like(self.tail)]
            inp = stg["inp"]
            inp.copy_(buf[:, :inp.shape[1]])
            tail = self._tails[1] if self.tail.data_ptr() == self._tails[0].data_ptr() else self._tails[0]
            L.check(lib.ctn_stream_call(ctypes.byref(d), ctypes.byref(self._model_struct()), self.frames,
                                        inp.data_ptr(), inp.stride(0), self.tail.data_ptr(), tail.data_ptr(),
                                        stg["out"].data_ptr(), stg["ws"].data_ptr(), nb, st), "ctn_stream_call")
            self.tail = tail
            self.frames += K
            return stg["out"].clone()
        w = torch.empty(M, K, m.N, device=dev)
        x = torch.empty(M, K, self.B, device=dev)
        L.check(lib.ctn_stream_encode(ctypes.byref(d), buf.data_ptr(), buf.stride(0), self.U.data_ptr(),
                                      self.g0.data_ptr(), self.b0.data_ptr(), self.wb_t.data_ptr(), w.data_ptr(),
                                      x.data_ptr(), st), "ctn_stream_encode")
        y = torch.empty_like(x)
        for b, ring in zip(self.blocks, self.rings):
            L.check(lib.ctn_stream_block(ctypes.byref(d), b["dil"], self.frames, ring.shape[1], x.data_ptr(),
                                         *(b[k].data_ptr() for k in ("w1_t", "alpha1", "n1a", "n1b", "wd", "alpha2",
                                                                     "n2a", "n2b", "w2_t")),
                                         ring.data_ptr(), y.data_ptr(), st), "ctn_stream_block")
            x, y = y, x
        out = torch.empty(M, m.C, K * self.stride, device=dev)
        frames = torch.empty(M, m.C, K, m.L, device=dev)
        tail = torch.empty_like(self.tail)
        L.check(lib.ctn_stream_decode(ctypes.byref(d), x.data_ptr(), w.data_ptr(), self.wm_t.data_ptr(),
                                      self.V.data_ptr(), self.tail.data_ptr(), tail.data_ptr(), frames.data_ptr(),
                                      out.data_ptr(), st), "ctn_stream_decode")
        self.tail = tail
        self.frames += K
        return out

    # -- streaming -------------------------------------------------------------
    @torch.no_grad()
    def push(self, chunk: torch.Tensor) -> torch.Tensor:
        """chunk [M, n] fp32 samples -> the next finished output samples [M, C, m]."""
        m = self.model
        L.require_device(chunk, "StreamingSeparator")
        chunk = chunk.float()
        buf = chunk if self.samples is None else torch.cat([self.samples, chunk], dim=1)
        M, T = buf.shape
        if self.rings is None:
            self._alloc(M, buf.device)
        elif self.tail.shape[0] != M:
            raise ValueError("the number of streams changed; call reset() first")
        K = (T - m.L) // self.stride + 1 if T >= m.L else 0
        if K <= 0:
            self.samples = buf
            return buf.new_zeros(M, m.C, 0)
        outs = []
        for k0 in range(0, K, self.max_frames):
            k = min(self.max_frames, K - k0)
            outs.append(self._call(buf[:, k0 * self.stride:].contiguous(), k))
        self.samples = buf[:, K * self.stride:].contiguous()    # the overlap of the next frame onwards
        return outs[0] if len(outs) == 1 else torch.cat(outs, dim=2)

    @torch.no_grad()
    def flush(self) -> torch.Tensor:
        """The remaining overlap-add samples (call once after the last chunk).  The
        streamer is reset afterwards: the next push() starts a new stream."""
        out = self.tail if self.frames else None
        self.reset()
        if out is None:
            return torch.zeros(0)
        return out

    def separate(self, mixture: torch.Tensor, chunk: int) -> torch.Tensor:
        """Whole signal [M, T] in chunks of ``chunk`` samples -> [M, C, T] (zero tail as the
        reference's F.pad to the input length, conv_tasnet.py:56-58)."""
        self.reset()
        parts = [self.push(mixture[:, i:i + chunk]) for i in range(0, mixture.shape[1], chunk)]
        tail = self.flush()
        if tail.numel():
            parts.append(tail)
        out = torch.cat(parts, dim=2)
        T = mixture.shape[1]
        if out.shape[2] < T:
            out = torch.nn.functional.pad(out, (0, T - out.shape[2]))
        return out[:, :, :T]
