"""Streaming (chunk-by-chunk) separation with a causal Conv-TasNet (SURVEY.md
§8f row 4, stretch item): audio arrives in chunks of any length, separated
audio leaves with a fixed delay of one encoder stride, and the concatenated
output equals ``ConvTasNet.forward`` on the whole signal.

Why a causal model streams (conv_tasnet.py:176, 251-260, 289): with
``causal=True`` every operation is either per frame (encoder, cLN, 1x1 convs,
PReLU, mask and its nonlinearity, decoder basis) or looks only BACKWARD in time
(the dilated depthwise conv after Chomp1d reaches (P-1)*d frames into the
past).  gLN normalizes over the whole utterance and cannot stream; BatchNorm
streams in eval mode (running statistics, per frame).

State kept between chunks (all on the device):
* ``samples``: input samples not yet consumed by a whole encoder frame
  (< L; frame k covers samples [k*L/2, k*L/2 + L));
* per TemporalBlock, a ring of its last (P-1)*d INPUT frames — the block is
  re-run on [history | new frames] and only the new frames are kept, so the
  depthwise taps of every new frame see exactly the frames the full forward
  gives them, and the kernel's causal zero padding stands in for the frames
  before the start of the stream (history shorter than (P-1)*d);
* ``tail``: the last L/2 output samples of the previous chunk's overlap-add,
  which the next chunk's first frame completes.

Each chunk runs the same native calls as the model forward (EncoderFn,
TBlockFn per block, DecoderFn: include/ctn.h) on the chunk's frames plus the
block histories; rows are re-laid out per block with torch copies.  Forward
only (torch.no_grad).
"""
from __future__ import annotations

import torch

import ctn_lib as L
import ctn_ops as ops
from conv_tasnet import ConvTasNet, _act_dtype, _mask_code, _norm_code


class StreamingSeparator:
    """Wraps a causal ConvTasNet for chunked inference.

    >>> s = StreamingSeparator(model)          # model.causal, norm_type cLN (or BN in eval)
    >>> outs = [s.push(chunk) for chunk in chunks]   # chunk [M, n] -> [M, C, m] (m may be 0)
    >>> outs.append(s.flush())                  # the last L/2 samples
    """

    def __init__(self, model: ConvTasNet, act_dtype=None):
        if not model.causal:
            raise ValueError("streaming needs a causal model (ConvTasNet(causal=True))")
        norm = _norm_code(model.norm_type)
        if norm == L.NORM_GLN:
            raise ValueError("gLN normalizes over the whole utterance: a gLN model cannot stream")
        if norm == L.NORM_BN and model.training:
            raise ValueError("BatchNorm streams only in eval mode (running statistics)")
        if model.L % 2:
            raise ValueError("the encoder stride L//2 must tile the frame (even L)")
        self.model = model
        self.norm = norm
        self.dt = _act_dtype(act_dtype if act_dtype is not None else model.act_dtype)
        self.stride = model.L // 2
        self.blocks = list(model.separator.blocks())
        # frames of history per block: (P-1)*dilation (the causal receptive field)
        self.ctx = [(b._geo[2] - 1) * b._geo[3] for b in self.blocks]
        self.reset()

    def reset(self):
        self.samples = None          # [M, s] pending input samples
        self.hist = [None] * len(self.blocks)   # [M, h, B] block-input history
        self.tail = None             # [M, C, stride] pending overlap-add samples
        self.frames = 0              # frames emitted so far

    @property
    def latency_samples(self) -> int:
        """Output trails input by one stride: the last L/2 samples wait for the next frame."""
        return self.stride

    # -- helpers ---------------------------------------------------------------
    def _pad_rows(self, seq: torch.Tensor) -> tuple:
        """[M, K, C] frames -> ([M*Kp, C] rows with zero padded rows, Frames)."""
        M, K, C = seq.shape
        fr = ops.Frames.of(M, K)
        rows = seq.new_zeros(M, fr.Kp, C)
        rows[:, :K] = seq
        return rows.view(M * fr.Kp, C), fr

    @staticmethod
    def _frames(rows: torch.Tensor, fr: ops.Frames, first: int = 0) -> torch.Tensor:
        return rows.view(fr.M, fr.Kp, -1)[:, first:fr.K]

    # -- streaming -------------------------------------------------------------
    @torch.no_grad()
    def push(self, chunk: torch.Tensor) -> torch.Tensor:
        """chunk [M, n] fp32 samples -> the next finished output samples [M, C, m]."""
        m = self.model
        L.require_device(chunk, "StreamingSeparator")
        chunk = chunk.float()
        buf = chunk if self.samples is None else torch.cat([self.samples, chunk], dim=1)
        M, T = buf.shape
        K = (T - m.L) // self.stride + 1 if T >= m.L else 0
        if K <= 0:
            self.samples = buf
            return buf.new_zeros(M, m.C, 0)
        used = (K - 1) * self.stride + m.L
        self.samples = buf[:, K * self.stride:]        # the overlap of the next frame onwards
        enc_in = buf[:, :used].contiguous()

        sep = m.separator
        cln, bott = sep.network[0], sep.network[1]
        fr = ops.Frames.of(M, K)
        w_rows, x = ops.EncoderFn.apply(enc_in, fr, (m.N, m.L, m.B, m.C), self.dt, m.encoder.conv1d_U.weight,
                                        cln.gamma, cln.beta, bott.weight)
        new = self._frames(x, fr)                       # [M, K, B]
        for i, blk in enumerate(self.blocks):
            h = self.hist[i]
            seq = new if h is None else torch.cat([h, new], dim=1)
            rows, fr_b = self._pad_rows(seq)
            y = blk._forward_rows(rows, fr_b, self.norm)
            hn = seq.shape[1] - K                       # history frames in front of the new ones
            keep = self.ctx[i]
            self.hist[i] = seq[:, max(0, seq.shape[1] - keep):].clone() if keep > 0 else None
            new = self._frames(y, fr_b, hn)
        x_last, _ = self._pad_rows(new)
        Tc = (K - 1) * self.stride + m.L
        est = ops.DecoderFn.apply(x_last, w_rows, fr, (Tc, m.N, m.L, m.B, m.C, _mask_code(m.mask_nonlinear)),
                                  sep.network[3].weight, m.decoder.basis_signals.weight)   # [M, C, Tc]
        if self.tail is not None:
            est[:, :, :self.stride] += self.tail
        self.tail = est[:, :, K * self.stride:].clone()
        self.frames += K
        return est[:, :, :K * self.stride]

    @torch.no_grad()
    def flush(self) -> torch.Tensor:
        """The remaining overlap-add samples (call once after the last chunk)."""
        out = self.tail
        self.tail = None
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
