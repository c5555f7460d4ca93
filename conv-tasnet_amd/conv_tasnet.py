"""Drop-in for jwr1995/Conv-TasNet ``src/conv_tasnet.py`` on MI355X.

Same classes, constructor signatures, attributes, submodule tree, parameter
names/shapes/order and init as the reference, so
``from conv_tasnet import ConvTasNet`` with ``PYTHONPATH=conv-tasnet_amd``
replaces the reference import (src/train.py:12, evaluate.py:16, separate.py:14)
and reference checkpoints load unchanged.  ``forward`` runs the hand-written
HIP kernels of ``libctn_hip.so`` (include/ctn.h) on a ROCm device:

    EncoderFn  : encoder + separator cLN + bottleneck        (one native call)
    TBlockFn   : each of the R*X TemporalBlocks               (one native call)
    DecoderFn  : mask conv + nonlinearity + decoder + OLA/pad (one native call)

Activation dtype: float32, or bfloat16 when the forward runs under
``torch.autocast("cuda", dtype=torch.bfloat16)`` (statistics, accumulation and
parameters stay fp32).  CPU tensors raise: there is no CPU fallback.
"""
from __future__ import annotations

import torch
import torch.nn as nn

import ctn_lib as L
import ctn_ops as ops

EPS = 1e-8   # conv_tasnet.py:10 (used by the kernels)


def _act_dtype(explicit=None):
    if explicit is not None:
        return explicit
    if torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16:
        return torch.bfloat16
    return torch.float32


def _norm_code(norm_type):
    if norm_type == "gLN":
        return L.NORM_GLN
    if norm_type == "cLN":
        return L.NORM_CLN
    return L.NORM_BN      # chose_norm's fallback branch: nn.BatchNorm1d (conv_tasnet.py:302-303)


def _mask_code(mask_nonlinear):
    if mask_nonlinear == "softmax":
        return L.MASK_SOFTMAX
    if mask_nonlinear == "relu":
        return L.MASK_RELU
    raise ValueError("Unsupported mask non-linear function")      # conv_tasnet.py:207-208


def _io_dtype(t):
    return t.dtype if t.dtype in (torch.float32, torch.bfloat16) else torch.float32


def _norm_rows(norm_mod, rows, fr):
    """A block norm module applied to frame rows: gLN / cLN on the HIP path
    (ctn_layernorm_*); nn.BatchNorm1d — chose_norm's fallback, a torch module in the
    reference as well — on the NCW view of the rows."""
    if isinstance(norm_mod, (GlobalLayerNorm, ChannelwiseLayerNorm)):
        code = L.NORM_GLN if isinstance(norm_mod, GlobalLayerNorm) else L.NORM_CLN
        return ops.LayerNormFn.apply(rows, fr, code, norm_mod.gamma, norm_mod.beta)
    y = norm_mod(ops.rows_to_ncw(rows, fr, torch.float32))
    return ops.ncw_to_rows(y, fr, rows.dtype)


class ConvTasNet(nn.Module):
    def __init__(self, N, L, B, H, P, X, R, C, norm_type="gLN", causal=False,
                 mask_nonlinear='relu'):
        """conv_tasnet.py:14-43 — same arguments, attributes, submodules and init."""
        super(ConvTasNet, self).__init__()
        self.N, self.L, self.B, self.H, self.P, self.X, self.R, self.C = N, L, B, H, P, X, R, C
        self.norm_type = norm_type
        self.causal = causal
        self.mask_nonlinear = mask_nonlinear
        self.encoder = Encoder(L, N)
        self.separator = TemporalConvNet(N, B, H, P, X, R, C, norm_type, causal, mask_nonlinear)
        self.decoder = Decoder(N, L)
        # conv_tasnet.py:41-43: xavier_normal_ on every param with dim > 1, which also
        # overwrites the [1,C,1] gLN/cLN gamma/beta
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_normal_(p)
        self.act_dtype = None     # None: follow autocast; or torch.float32 / torch.bfloat16
        # True: in a plain .backward() with no gradients yet, each TemporalBlock's
        # parameter-gradient tail runs on a second stream and writes .grad directly,
        # overlapping the next block's backward (ctn_ops._split_ok lists the conditions;
        # otherwise the one-stream path runs).  Off by default: at the paper batch the
        # overlapped kernels slow each other down more than the overlap saves (§11).
        self.wgrad_stream = False
        # True: in a plain .backward() with no gradients yet (the same conditions), each
        # TemporalBlock leaves its parameter-gradient reductions for one batched call at
        # the end of the backward pass (ctn_tblock_reduce_grads: a few launches instead of
        # two per block); bit-identical gradients.
        self.defer_grad_reduce = True

    def forward(self, mixture):
        """mixture [M, T] -> est_source [M, C, T] (conv_tasnet.py:45-60)."""
        L.require_device(mixture, "ConvTasNet")
        _mask_code(self.mask_nonlinear)
        norm = _norm_code(self.norm_type)
        dt = _act_dtype(self.act_dtype)
        M, T = mixture.shape
        K = (T - self.L) // (self.L // 2) + 1
        fr = ops.Frames.of(M, K)
        sep = self.separator
        cln, bott = sep.network[0], sep.network[1]
        w_rows, x = ops.EncoderFn.apply(mixture, fr, (self.N, self.L, self.B, self.C), dt,
                                        self.encoder.conv1d_U.weight, cln.gamma, cln.beta, bott.weight)
        blocks = list(sep.blocks())
        packs = [None] * len(blocks)
        if dt == torch.bfloat16:   # bf16 weight copies for every block: one launch per step
            if not hasattr(self, "_packs"):
                self._packs = ops.PackCache()
            packs = self._packs.get([(b.net[0].weight, b._params()[8]) for b in blocks], mixture.device)
        split = self.wgrad_stream and torch.is_grad_enabled()
        defer = self.defer_grad_reduce and torch.is_grad_enabled() and norm != L.NORM_BN
        for blk, pk in zip(blocks, packs):
            x = blk._forward_rows(x, fr, norm, pk, split, defer)
        return ops.DecoderFn.apply(x, w_rows, fr, (T, self.N, self.L, self.B, self.C, _mask_code(self.mask_nonlinear)),
                                   sep.network[3].weight, self.decoder.basis_signals.weight)

    @classmethod
    def load_model(cls, path):
        """conv_tasnet.py:62-67 (maps to CPU; weights-only load)."""
        package = torch.load(path, map_location=lambda storage, loc: storage, weights_only=True)
        return cls.load_model_from_package(package)

    @classmethod
    def load_model_from_package(cls, package):
        """conv_tasnet.py:69-76."""
        model = cls(package['N'], package['L'], package['B'], package['H'],
                    package['P'], package['X'], package['R'], package['C'],
                    norm_type=package['norm_type'], causal=package['causal'],
                    mask_nonlinear=package['mask_nonlinear'])
        model.load_state_dict(package['state_dict'])
        return model

    @staticmethod
    def serialize(model, optimizer, epoch, tr_loss=None, cv_loss=None):
        """conv_tasnet.py:78-94 — identical package keys."""
        package = {
            'N': model.N, 'L': model.L, 'B': model.B, 'H': model.H,
            'P': model.P, 'X': model.X, 'R': model.R, 'C': model.C,
            'norm_type': model.norm_type, 'causal': model.causal,
            'mask_nonlinear': model.mask_nonlinear,
            'state_dict': model.state_dict(),
            'optim_dict': optimizer.state_dict(),
            'epoch': epoch
        }
        if tr_loss is not None:
            package['tr_loss'] = tr_loss
            package['cv_loss'] = cv_loss
        return package


class Encoder(nn.Module):
    """conv_tasnet.py:97-117: ReLU(Conv1d(1, N, L, stride=L//2, bias=False))."""

    def __init__(self, L, N):
        super(Encoder, self).__init__()
        self.L, self.N = L, N
        self.conv1d_U = nn.Conv1d(1, N, kernel_size=L, stride=L // 2, bias=False)
        self.act_dtype = None

    def forward(self, mixture):
        """mixture [M, T] -> mixture_w [M, N, K]."""
        L.require_device(mixture, "Encoder")
        M, T = mixture.shape
        K = (T - self.L) // (self.L // 2) + 1
        fr = ops.Frames.of(M, K)
        w_rows, _ = ops.EncoderFn.apply(mixture, fr, (self.N, self.L, 8, 1), _act_dtype(self.act_dtype),
                                        self.conv1d_U.weight, None, None, None)
        return ops.rows_to_ncw(w_rows, fr)


class Decoder(nn.Module):
    """conv_tasnet.py:120-142: (w ⊙ mask) · basisᵀ, overlap-add with step L//2."""

    def __init__(self, N, L):
        super(Decoder, self).__init__()
        self.N, self.L = N, L
        self.basis_signals = nn.Linear(N, L, bias=False)

    def forward(self, mixture_w, est_mask):
        """mixture_w [M, N, K], est_mask [M, C, N, K] -> est_source [M, C, (K-1)*L/2 + L]."""
        L.require_device(mixture_w, "Decoder")
        M, N, K = mixture_w.shape
        C = est_mask.shape[1]
        fr = ops.Frames.of(M, K)
        dt = mixture_w.dtype if mixture_w.dtype in (torch.float32, torch.bfloat16) else torch.float32
        w_rows = ops.ncw_to_rows(mixture_w, fr, dt)
        m_rows = ops.ncw_to_rows(est_mask.reshape(M, C * N, K), fr, dt)
        T = (K - 1) * (self.L // 2) + self.L
        return ops.DecoderFn.apply(m_rows, w_rows, fr, (T, N, self.L, 8, C, L.MASK_IDENTITY), None,
                                   self.basis_signals.weight)


class TemporalConvNet(nn.Module):
    """conv_tasnet.py:145-209 — same network layout:
    [cLN(N), Conv1x1 N->B, R x [X x TemporalBlock], Conv1x1 B->C*N]."""

    def __init__(self, N, B, H, P, X, R, C, norm_type="gLN", causal=False,
                 mask_nonlinear='relu'):
        super(TemporalConvNet, self).__init__()
        self.C = C
        self.mask_nonlinear = mask_nonlinear
        layer_norm = ChannelwiseLayerNorm(N)
        bottleneck_conv1x1 = nn.Conv1d(N, B, 1, bias=False)
        repeats = []
        for r in range(R):
            blocks = []
            for x in range(X):
                dilation = 2 ** x
                padding = (P - 1) * dilation if causal else (P - 1) * dilation // 2
                blocks += [TemporalBlock(B, H, P, stride=1, padding=padding, dilation=dilation,
                                         norm_type=norm_type, causal=causal)]
            repeats += [nn.Sequential(*blocks)]
        temporal_conv_net = nn.Sequential(*repeats)
        mask_conv1x1 = nn.Conv1d(B, C * N, 1, bias=False)
        self.network = nn.Sequential(layer_norm, bottleneck_conv1x1, temporal_conv_net, mask_conv1x1)
        self._norm_type = norm_type

    def blocks(self):
        for rep in self.network[2]:
            for blk in rep:
                yield blk

    def forward(self, mixture_w):
        """mixture_w [M, N, K] -> est_mask [M, C, N, K] (conv_tasnet.py:192-209).

        Stand-alone call: cLN, bottleneck, mask conv and nonlinearity as separate
        native layers (ctn_layernorm / ctn_conv1x1 / ctn_mask), the blocks as in
        ConvTasNet.forward (ctn_tblock).  Activations in fp32, or bf16 under
        torch.autocast; the mask is returned in that dtype."""
        L.require_device(mixture_w, "TemporalConvNet")
        M, N, K = mixture_w.shape
        fr = ops.Frames.of(M, K)
        dt = _act_dtype(getattr(self, "act_dtype", None))
        cln, bott, _, mask_conv = self.network
        r = ops.ncw_to_rows(mixture_w, fr, dt)
        r = ops.LayerNormFn.apply(r, fr, L.NORM_CLN, cln.gamma, cln.beta)
        r = ops.Conv1x1Fn.apply(r, fr, bott.weight)
        norm = _norm_code(self._norm_type)
        for blk in self.blocks():
            r = blk._forward_rows(r, fr, norm)
        score = ops.Conv1x1Fn.apply(r, fr, mask_conv.weight)
        mask = ops.MaskFn.apply(score, fr, self.C, _mask_code(self.mask_nonlinear))
        return ops.rows_to_ncw(mask, fr).reshape(M, self.C, N, K)


class TemporalBlock(nn.Module):
    """conv_tasnet.py:212-238: x + DSConv(norm(PReLU(Conv1x1_{B->H}(x))))."""

    def __init__(self, in_channels, out_channels, kernel_size,
                 stride, padding, dilation, norm_type="gLN", causal=False):
        super(TemporalBlock, self).__init__()
        conv1x1 = nn.Conv1d(in_channels, out_channels, 1, bias=False)
        prelu = nn.PReLU()
        norm = chose_norm(norm_type, out_channels)
        dsconv = DepthwiseSeparableConv(out_channels, in_channels, kernel_size,
                                        stride, padding, dilation, norm_type, causal)
        self.net = nn.Sequential(conv1x1, prelu, norm, dsconv)
        self._geo = (in_channels, out_channels, kernel_size, dilation, bool(causal), norm_type)
        if stride != 1:
            raise ValueError("TemporalBlock: only stride 1 is used by the reference (conv_tasnet.py:177)")

    # Sub-modules by their Sequential keys (dict lookups: this runs for every block on
    # every step, and nn.Sequential indexing goes through islice)
    def _norms(self):
        m = self.net._modules
        return m['2'], m['3'].net._modules['3' if self._geo[4] else '2']

    def _params(self):
        m = self.net._modules
        ds = m['3'].net._modules
        off = 1 if self._geo[4] else 0
        n1, n2 = m['2'], ds[str(2 + off)]
        if isinstance(n1, nn.BatchNorm1d):
            g1, b1, g2, b2 = n1.weight, n1.bias, n2.weight, n2.bias
        else:
            g1, b1, g2, b2 = n1.gamma, n1.beta, n2.gamma, n2.beta
        return (m['0'].weight, m['1'].weight, g1, b1, ds['0'].weight,
                ds[str(1 + off)].weight, g2, b2, ds[str(3 + off)].weight)

    def _acc_nodes(self, params):
        """The parameters' AccumulateGrad nodes (what ctn_ops reads to decide whether a late
        gradient write is unobservable), held by this module: the same node objects every
        step (autograd keeps a leaf's accumulator while anyone holds it), found once instead
        of per forward; recomputed when a parameter was replaced."""
        c = getattr(self, "_acc_cache", None)
        if c is None or len(c[0]) != len(params) or any(a is not b for a, b in zip(c[0], params)):
            nodes = tuple(torch.autograd.graph.get_gradient_edge(t).node if t.requires_grad and t.is_leaf else None
                          for t in params)
            object.__setattr__(self, "_acc_cache", c := (tuple(params), nodes))
        return c[1]

    def _forward_rows(self, x_rows, fr, norm, pack=None, wgrad_split=False, defer=False):
        B, H, P, dil, causal, _ = self._geo
        bn = ops.bn_state(*self._norms()) if norm == L.NORM_BN else None
        params = self._params()
        nodes = self._acc_nodes(params) if (wgrad_split or defer) and torch.is_grad_enabled() else None
        return ops.TBlockFn.apply(x_rows, fr, (B, H, P, dil, causal, norm, wgrad_split, defer, nodes), pack, bn,
                                  *params)

    def forward(self, x):
        """x [M, B, K] -> [M, B, K]."""
        L.require_device(x, "TemporalBlock")
        M, B, K = x.shape
        fr = ops.Frames.of(M, K)
        dt = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        y = self._forward_rows(ops.ncw_to_rows(x, fr, dt), fr, _norm_code(self._geo[5]))
        return ops.rows_to_ncw(y, fr)


class DepthwiseSeparableConv(nn.Module):
    """conv_tasnet.py:241-272.  Inside a TemporalBlock its compute is fused into the
    block kernels (ctn_tblock_*); called on its own it runs the stand-alone layers
    (ctn_depthwise / ctn_prelu / ctn_layernorm / ctn_conv1x1)."""

    def __init__(self, in_channels, out_channels, kernel_size,
                 stride, padding, dilation, norm_type="gLN", causal=False):
        super(DepthwiseSeparableConv, self).__init__()
        depthwise_conv = nn.Conv1d(in_channels, in_channels, kernel_size,
                                   stride=stride, padding=padding,
                                   dilation=dilation, groups=in_channels,
                                   bias=False)
        if causal:
            chomp = Chomp1d(padding)
        prelu = nn.PReLU()
        norm = chose_norm(norm_type, in_channels)
        pointwise_conv = nn.Conv1d(in_channels, out_channels, 1, bias=False)
        if causal:
            self.net = nn.Sequential(depthwise_conv, chomp, prelu, norm, pointwise_conv)
        else:
            self.net = nn.Sequential(depthwise_conv, prelu, norm, pointwise_conv)

    def forward(self, x):
        """x [M, C_in, K] -> [M, C_out, K] (conv_tasnet.py:265-272)."""
        L.require_device(x, "DepthwiseSeparableConv")
        M, C, K = x.shape
        fr = ops.Frames.of(M, K)
        causal = isinstance(self.net[1], Chomp1d)
        dw = self.net[0]
        P, dil = dw.kernel_size[0], dw.dilation[0]
        if dw.stride[0] != 1 or dw.padding[0] != ((P - 1) * dil if causal else (P - 1) * dil // 2):
            raise L.CtnLibraryError("DepthwiseSeparableConv: only the reference's stride 1 and padding "
                                    "(conv_tasnet.py:177,188) are implemented")
        prelu, norm, pw = self.net[2 if causal else 1], self.net[3 if causal else 2], self.net[-1]
        r = ops.ncw_to_rows(x, fr, _io_dtype(x))
        r = ops.DepthwiseFn.apply(r, fr, (P, dil, causal), dw.weight)
        r = ops.PReLUFn.apply(r, fr, prelu.weight)
        r = _norm_rows(norm, r, fr)
        r = ops.Conv1x1Fn.apply(r, fr, pw.weight)
        return ops.rows_to_ncw(r, fr)


class Chomp1d(nn.Module):
    """conv_tasnet.py:275-289.  The HIP depthwise kernel pads on the left only,
    which is identical to symmetric padding followed by this chomp."""

    def __init__(self, chomp_size):
        super(Chomp1d, self).__init__()
        self.chomp_size = chomp_size

    def forward(self, x):
        return x[:, :, :-self.chomp_size].contiguous()


def chose_norm(norm_type, channel_size):
    """conv_tasnet.py:292-303."""
    if norm_type == "gLN":
        return GlobalLayerNorm(channel_size)
    elif norm_type == "cLN":
        return ChannelwiseLayerNorm(channel_size)
    else:
        return nn.BatchNorm1d(channel_size)


class ChannelwiseLayerNorm(nn.Module):
    """Channel-wise Layer Normalization (cLN), conv_tasnet.py:307-329 (per-frame
    statistics, biased variance, EPS=1e-8).  Fused into the encoder/block kernels
    inside the model; on its own ctn_layernorm_* (CTN_NORM_CLN)."""

    def __init__(self, channel_size):
        super(ChannelwiseLayerNorm, self).__init__()
        self.gamma = nn.Parameter(torch.Tensor(1, channel_size, 1))
        self.beta = nn.Parameter(torch.Tensor(1, channel_size, 1))
        self.reset_parameters()

    def reset_parameters(self):
        self.gamma.data.fill_(1)
        self.beta.data.zero_()

    def forward(self, y):
        """y [M, N, K] -> cLN(y) (conv_tasnet.py:319-329)."""
        return _layer_norm_ncw(y, L.NORM_CLN, self.gamma, self.beta)


def _layer_norm_ncw(y, code, gamma, beta):
    L.require_device(y, "LayerNorm")
    M, C, K = y.shape
    fr = ops.Frames.of(M, K)
    r = ops.LayerNormFn.apply(ops.ncw_to_rows(y, fr, _io_dtype(y)), fr, code, gamma, beta)
    return ops.rows_to_ncw(r, fr)


class GlobalLayerNorm(nn.Module):
    """Global Layer Normalization (gLN), conv_tasnet.py:332-355 (per-utterance
    statistics over [N, K], EPS=1e-8).  Fused into the block kernels inside the
    model; on its own ctn_layernorm_* (CTN_NORM_GLN)."""

    def __init__(self, channel_size):
        super(GlobalLayerNorm, self).__init__()
        self.gamma = nn.Parameter(torch.Tensor(1, channel_size, 1))
        self.beta = nn.Parameter(torch.Tensor(1, channel_size, 1))
        self.reset_parameters()

    def reset_parameters(self):
        self.gamma.data.fill_(1)
        self.beta.data.zero_()

    def forward(self, y):
        """y [M, N, K] -> gLN(y) (conv_tasnet.py:344-355)."""
        return _layer_norm_ncw(y, L.NORM_GLN, self.gamma, self.beta)
