"""CPU oracle for the Conv-TasNet hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The shipped path (``conv-tasnet_amd/``) runs the HIP kernels in
``libctn_hip.so`` and raises if that library is missing; it never routes
through this file.

What it is: a functional fp32 restatement (eager PyTorch on the CPU, autograd
for the backward pass) of the reference algorithm in
``jwr1995/Conv-TasNet`` (read-only at /root/reference).  Every function cites
the reference ``file:line`` it restates.  Parameters are passed as a dict keyed
exactly like the reference ``state_dict``, so the same weights
drive the oracle, the reference and the HIP build.

Pinning: ``tests/golden/make_golden.py`` imported the real reference in the
build container (with ``torch.Tensor.cuda`` shimmed to identity, because
``src/utils.py:40`` calls ``.cuda()`` unconditionally) and captured
input/output/gradient vectors into ``tests/golden/*.npz``.
``tests/test_oracle_golden.py`` checks this oracle against every one of them.
The reference itself ships no assertion-based tests, so those
captured vectors are the only pins.  SDRi (mir_eval) is not restated: parity
unpinned.
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass

import numpy as np
import torch
from scipy.signal import lfilter
import torch.nn.functional as F

# conv_tasnet.py:10 and pit_criterion.py:9 — both use 1e-8
EPS = 1e-8


@dataclass(frozen=True)
class Cfg:
    """Hyper-parameters of ``ConvTasNet.__init__`` (conv_tasnet.py:14-15)."""
    N: int
    L: int
    B: int
    H: int
    P: int
    X: int
    R: int
    C: int
    norm_type: str = "gLN"
    causal: bool = False
    mask_nonlinear: str = "relu"


# ----------------------------------------------------------------------------
# parameter naming / deterministic init
# ----------------------------------------------------------------------------
def block_prefix(r: int, x: int) -> str:
    """state_dict prefix of TemporalBlock (r, x): conv_tasnet.py:171-190."""
    return f"separator.network.2.{r}.{x}."


def param_shapes(cfg: Cfg) -> "list[tuple[str, tuple]]":
    """Parameter names and shapes in reference ``named_parameters()`` order.

    Order follows module registration: encoder (conv_tasnet.py:37,106),
    separator (:38,187-190 → cLN :167, bottleneck :169, blocks :171-183 with
    TemporalBlock.net = [conv1x1, prelu, norm, dsconv] :225 and
    DepthwiseSeparableConv.net = [dw, (chomp), prelu, norm, pw] :258-263,
    mask conv :185), decoder (:39,126).  BN (chose_norm :303) registers
    weight/bias; running stats are buffers and are not listed here.
    """
    N, L, B, H, P, C = cfg.N, cfg.L, cfg.B, cfg.H, cfg.P, cfg.C
    out = [("encoder.conv1d_U.weight", (N, 1, L)),
           ("separator.network.0.gamma", (1, N, 1)),
           ("separator.network.0.beta", (1, N, 1)),
           ("separator.network.1.weight", (B, N, 1))]

    def norm(prefix, ch):
        if cfg.norm_type in ("gLN", "cLN"):
            return [(prefix + "gamma", (1, ch, 1)), (prefix + "beta", (1, ch, 1))]
        return [(prefix + "weight", (ch,)), (prefix + "bias", (ch,))]

    off = 1 if cfg.causal else 0   # Chomp1d shifts the dsconv indices
    for r in range(cfg.R):
        for x in range(cfg.X):
            p = block_prefix(r, x)
            out += [(p + "net.0.weight", (H, B, 1)), (p + "net.1.weight", (1,))]
            out += norm(p + "net.2.", H)
            out += [(p + "net.3.net.0.weight", (H, 1, P)),
                    (p + f"net.3.net.{1 + off}.weight", (1,))]
            out += norm(p + f"net.3.net.{2 + off}.", H)
            out += [(p + f"net.3.net.{3 + off}.weight", (B, H, 1))]
    out += [("separator.network.3.weight", (C * N, B, 1)),
            ("decoder.basis_signals.weight", (L, N))]
    return out


def xavier_normal_std(shape) -> float:
    """torch.nn.init.xavier_normal_ std (gain 1) for a tensor of ``shape``."""
    if len(shape) == 2:
        fan_in, fan_out = shape[1], shape[0]
    else:
        rf = int(np.prod(shape[2:]))
        fan_in, fan_out = shape[1] * rf, shape[0] * rf
    return math.sqrt(2.0 / float(fan_in + fan_out))


def init_params(cfg: Cfg, seed: int) -> "dict[str, torch.Tensor]":
    """Deterministic init with the reference's *semantics* (conv_tasnet.py:41-43).

    Every parameter with dim > 1 — including the [1,C,1] gLN/cLN gamma/beta —
    is xavier-normal; PReLU alphas stay 0.25 (torch default); BN weight/bias
    1/0.  The random stream is numpy's PCG64 so that the HIP tests, the oracle
    and the golden generator reproduce the same weights on any machine.
    """
    rng = np.random.default_rng(seed)
    params = {}
    for name, shape in param_shapes(cfg):
        if len(shape) > 1:
            v = rng.standard_normal(size=shape) * xavier_normal_std(shape)
        elif shape == (1,):                    # PReLU alpha
            v = np.full(shape, 0.25)
        elif name.endswith(".bias"):           # BN bias
            v = np.zeros(shape)
        else:                                  # BN weight
            v = np.ones(shape)
        params[name] = torch.tensor(v, dtype=torch.float32)
    return params


# ----------------------------------------------------------------------------
# forward ops
# ----------------------------------------------------------------------------
def encoder(mixture, U):
    """conv_tasnet.py:108-117: ReLU(Conv1d(1, N, L, stride=L//2, bias=False))."""
    L = U.shape[-1]
    return F.relu(F.conv1d(mixture.unsqueeze(1), U, stride=L // 2))


def cln(y, gamma, beta):
    """conv_tasnet.py:319-329: per-frame stats over channels, biased var."""
    mu = y.mean(dim=1, keepdim=True)
    var = ((y - mu) ** 2).mean(dim=1, keepdim=True)
    return gamma * (y - mu) / torch.sqrt(var + EPS) + beta


def gln(y, gamma, beta):
    """conv_tasnet.py:344-355: per-utterance stats over [C, K] (two-pass)."""
    mu = y.mean(dim=(1, 2), keepdim=True)
    var = ((y - mu) ** 2).mean(dim=(1, 2), keepdim=True)
    return gamma * (y - mu) / torch.sqrt(var + EPS) + beta


def bn(y, weight, bias, training=True, running=None):
    """nn.BatchNorm1d(C) on [M,C,K] (chose_norm conv_tasnet.py:300-303)."""
    if training:
        return F.batch_norm(y, None, None, weight, bias, True, 0.0, 1e-5)
    rm, rv = running
    return F.batch_norm(y, rm, rv, weight, bias, False, 0.0, 1e-5)


# Test hook for BatchNorm running statistics: {norm prefix: (running_mean, running_var)}.
# When set, BN follows nn.BatchNorm1d with its buffers: training mode (BN_TRAINING)
# normalizes with batch statistics and updates the buffers in place (momentum 0.1,
# unbiased variance); eval mode normalizes with the buffers.  None: batch statistics.
BN_RUNNING = None
BN_TRAINING = True


def norm(cfg: Cfg, y, params, prefix):
    """chose_norm dispatch (conv_tasnet.py:292-303)."""
    if cfg.norm_type == "gLN":
        return gln(y, params[prefix + "gamma"], params[prefix + "beta"])
    if cfg.norm_type == "cLN":
        return cln(y, params[prefix + "gamma"], params[prefix + "beta"])
    if BN_RUNNING is not None:
        rm, rv = BN_RUNNING[prefix]
        return F.batch_norm(y, rm, rv, params[prefix + "weight"], params[prefix + "bias"], BN_TRAINING, 0.1, 1e-5)
    return bn(y, params[prefix + "weight"], params[prefix + "bias"])


def prelu(y, alpha):
    """nn.PReLU() with one shared alpha (conv_tasnet.py:218,253)."""
    return F.prelu(y, alpha)


def depthwise(y, w, dilation, causal):
    """conv_tasnet.py:176,247-250 + Chomp1d :289.

    Non-causal: symmetric pad (P-1)*d//2.  Causal: pad (P-1)*d both sides then
    drop the right (P-1)*d frames — restated literally.
    """
    P = w.shape[-1]
    pad = (P - 1) * dilation if causal else (P - 1) * dilation // 2
    out = F.conv1d(y, w, padding=pad, dilation=dilation, groups=y.shape[1])
    if causal:
        out = out[:, :, :-pad].contiguous()
    return out


def temporal_block(cfg: Cfg, x, params, r, xi):
    """TemporalBlock.forward (conv_tasnet.py:227-237) incl. DSConv :241-272."""
    p = block_prefix(r, xi)
    off = 1 if cfg.causal else 0
    h = F.conv1d(x, params[p + "net.0.weight"])
    h = prelu(h, params[p + "net.1.weight"])
    h = norm(cfg, h, params, p + "net.2.")
    h = depthwise(h, params[p + "net.3.net.0.weight"], 2 ** xi, cfg.causal)
    h = prelu(h, params[p + f"net.3.net.{1 + off}.weight"])
    h = norm(cfg, h, params, p + f"net.3.net.{2 + off}.")
    h = F.conv1d(h, params[p + f"net.3.net.{3 + off}.weight"])
    return h + x


def separator(cfg: Cfg, w, params):
    """TemporalConvNet.forward (conv_tasnet.py:192-209); first norm is always cLN (:167)."""
    M, N, K = w.shape
    y = cln(w, params["separator.network.0.gamma"], params["separator.network.0.beta"])
    y = F.conv1d(y, params["separator.network.1.weight"])
    for r in range(cfg.R):
        for xi in range(cfg.X):
            y = temporal_block(cfg, y, params, r, xi)
    score = F.conv1d(y, params["separator.network.3.weight"]).view(M, cfg.C, N, K)
    if cfg.mask_nonlinear == "softmax":
        return F.softmax(score, dim=1)
    if cfg.mask_nonlinear == "relu":
        return F.relu(score)
    raise ValueError("Unsupported mask non-linear function")


def overlap_and_add(frames, step):
    """utils.py:9-46 restated as a gather: out[k*step + j] += frames[k, j]."""
    *outer, K, L = frames.shape
    T = (K - 1) * step + L
    out = frames.new_zeros(*outer, T)
    for k0 in range(0, L, step):
        # every frame contributes columns [k0, k0+step) at offset k*step + k0
        seg = frames[..., :, k0:min(k0 + step, L)]            # [..., K, s]
        s = seg.shape[-1]
        idx = (torch.arange(K) * step + k0).unsqueeze(1) + torch.arange(s)
        out = out.index_add(-1, idx.reshape(-1), seg.reshape(*outer, K * s))
    return out


def decoder(w, mask, V, L):
    """Decoder.forward (conv_tasnet.py:128-142): (w ⊙ m)ᵀ·Vᵀ then OLA with step L//2."""
    src_w = (w.unsqueeze(1) * mask).transpose(2, 3)           # [M, C, K, N]
    frames = torch.matmul(src_w, V.t())                       # [M, C, K, L]
    return overlap_and_add(frames, L // 2)


def model_forward(cfg: Cfg, mixture, params):
    """ConvTasNet.forward (conv_tasnet.py:45-60) incl. the F.pad back to T."""
    w = encoder(mixture, params["encoder.conv1d_U.weight"])
    mask = separator(cfg, w, params)
    est = decoder(w, mask, params["decoder.basis_signals.weight"], cfg.L)
    return F.pad(est, (0, mixture.shape[-1] - est.shape[-1]))


# ----------------------------------------------------------------------------
# PIT SI-SNR loss (pit_criterion.py)
# ----------------------------------------------------------------------------
def get_mask(source, lengths):
    """pit_criterion.py:101-113."""
    Bsz, _, T = source.shape
    t = torch.arange(T).unsqueeze(0)
    return (t < lengths.view(-1, 1)).to(source.dtype).unsqueeze(1)


def si_snr_pairwise(source, est, lengths):
    """pit_criterion.py:36-62: the pairwise SI-SNR matrix snr[b, i, j] (estimate i against
    source j) and the masked estimate."""
    assert source.shape == est.shape
    Bsz, C, T = source.shape
    mask = get_mask(source, lengths)
    est = est * mask
    n = lengths.view(-1, 1, 1).to(source.dtype)
    zt = (source - source.sum(2, keepdim=True) / n) * mask
    ze = (est - est.sum(2, keepdim=True) / n) * mask
    dot = torch.einsum("bit,bjt->bij", ze, zt)
    e_t = (zt ** 2).sum(2) + EPS
    proj = dot.unsqueeze(-1) * zt.unsqueeze(1) / e_t.view(Bsz, 1, C, 1)
    noise = ze.unsqueeze(2) - proj
    ratio = (proj ** 2).sum(3) / ((noise ** 2).sum(3) + EPS)
    return 10 * torch.log10(ratio + EPS), est


def perm_rank(perm):
    """Lexicographic rank of a permutation of range(C) (the itertools.permutations order
    the reference indexes its table in, pit_criterion.py:66)."""
    C, r, used = len(perm), 0, set()
    for i, p in enumerate(perm):
        r += sum(1 for v in range(p) if v not in used) * math.factorial(C - 1 - i)
        used.add(p)
    return r


def si_snr_pit_assign(source, est, lengths):
    """The maximum of cal_si_snr_with_pit's permutation sums (pit_criterion.py:66-75) for any
    C as a linear assignment on the pairwise SI-SNR (scipy.optimize.linear_sum_assignment,
    maximize): equal to the reference's argmax over C! permutations except on exact ties,
    and usable where the reference's C!-row table is not (C > 10).  Returns (max_snr [B,1],
    perm [B,C] (estimate i -> source perm[i]), rank [B], est_masked)."""
    from scipy.optimize import linear_sum_assignment
    snr, est_m = si_snr_pairwise(source, est, lengths)
    Bsz, C, _ = snr.shape
    perms, ranks, vals = [], [], []
    for b in range(Bsz):
        rows, cols = linear_sum_assignment(snr[b].detach().double().numpy(), maximize=True)
        p = [int(c) for _, c in sorted(zip(rows, cols))]
        perms.append(p)
        ranks.append(perm_rank(p))
        vals.append(snr[b, torch.arange(C), torch.tensor(p)].sum())
    max_snr = torch.stack(vals).view(Bsz, 1) / C
    return max_snr, torch.tensor(perms), torch.tensor(ranks), est_m


def si_snr_pit(source, est, lengths):
    """cal_si_snr_with_pit (pit_criterion.py:27-76), returns (max_snr, perms, idx, est_masked).

    Note (:37-38): the reference masks ``estimate_source`` in place; here the
    masked tensor is returned instead so the caller can reproduce that.
    """
    assert source.shape == est.shape
    Bsz, C, T = source.shape
    mask = get_mask(source, lengths)
    est = est * mask
    n = lengths.view(-1, 1, 1).to(source.dtype)
    zt = (source - source.sum(2, keepdim=True) / n) * mask
    ze = (est - est.sum(2, keepdim=True) / n) * mask
    dot = torch.einsum("bit,bjt->bij", ze, zt)                # est i vs target j
    e_t = (zt ** 2).sum(2) + EPS                               # [B, C]
    proj = dot.unsqueeze(-1) * zt.unsqueeze(1) / e_t.view(Bsz, 1, C, 1)
    noise = ze.unsqueeze(2) - proj
    ratio = (proj ** 2).sum(3) / ((noise ** 2).sum(3) + EPS)
    snr = 10 * torch.log10(ratio + EPS)                        # [B, C, C]
    perms = torch.tensor(list(itertools.permutations(range(C))), dtype=torch.long)
    # snr_set[b, p] = sum_i snr[b, i, perms[p, i]] (pit_criterion.py:66-71), one gather
    snr_set = snr[:, torch.arange(C).view(1, C), perms].sum(2)
    idx = torch.argmax(snr_set, dim=1)
    max_snr = snr_set.max(dim=1, keepdim=True)[0] / C
    return max_snr, perms, idx, est


def reorder_source(source, perms, idx):
    """pit_criterion.py:79-98 — keeps the reference's perm-not-inverse quirk."""
    sel = perms[idx]                                           # [B, C]
    return torch.stack([source[b, sel[b]] for b in range(source.shape[0])])


def cal_loss(source, est, lengths):
    """pit_criterion.py:12-24 → (loss, max_snr, est_masked, reordered)."""
    max_snr, perms, idx, est_m = si_snr_pit(source, est, lengths)
    loss = 0 - torch.mean(max_snr)
    return loss, max_snr, est_m, reorder_source(est_m, perms, idx)


# ----------------------------------------------------------------------------
# evaluation metric (evaluate.py:108-144), numpy
# ----------------------------------------------------------------------------
def cal_sisnr(ref, out, eps=1e-8):
    """evaluate.py:128-144."""
    ref = ref - np.mean(ref)
    out = out - np.mean(out)
    proj = np.sum(ref * out) * ref / (np.sum(ref ** 2) + eps)
    noise = out - proj
    ratio = np.sum(proj ** 2) / (np.sum(noise ** 2) + eps)
    return 10 * np.log(ratio + eps) / np.log(10.0)


def cal_sisnri(src_ref, src_est, mix):
    """evaluate.py:108-125 generalised to C speakers (reference hard-codes C=2)."""
    C = src_ref.shape[0]
    return float(np.mean([cal_sisnr(src_ref[c], src_est[c]) - cal_sisnr(src_ref[c], mix)
                          for c in range(C)]))


# ----------------------------------------------------------------------------
# one training step (solver.py:178-186)
# ----------------------------------------------------------------------------
def train_step(cfg: Cfg, params, mixture, source, lengths, lr=1e-3, max_norm=5.0):
    """forward → cal_loss → backward → clip_grad_norm_(5) → Adam(lr) (solver.py:178-186)."""
    leaves = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    est = model_forward(cfg, mixture, leaves)
    loss = cal_loss(source, est, lengths)[0]
    loss.backward()
    plist = [leaves[n] for n, _ in param_shapes(cfg)]
    torch.nn.utils.clip_grad_norm_(plist, max_norm)
    opt = torch.optim.Adam(plist, lr=lr)
    opt.step()
    return float(loss.detach()), {n: leaves[n].detach().clone() for n, _ in param_shapes(cfg)}


def fwd_bwd(cfg: Cfg, params, mixture, source, lengths):
    """Forward + PIT loss + backward; returns (masked est, loss, max_snr, grads dict)."""
    leaves = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    est = model_forward(cfg, mixture, leaves)
    loss, max_snr, est_m, _ = cal_loss(source, est, lengths)
    loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in leaves.items()}
    return est_m.detach(), float(loss.detach()), max_snr.detach(), grads


# ----------------------------------------------------------------------------
# synthetic speech-like data
# ----------------------------------------------------------------------------
def synth_batch(M, C, T, seed):
    """AR(2)-filtered noise × slow envelope, unit RMS, ±2.5 dB gain; mixture = Σ sources."""
    rng = np.random.default_rng(seed)
    src = np.empty((M, C, T), dtype=np.float64)
    for m in range(M):
        for c in range(C):
            e = rng.standard_normal(T)
            r, th = rng.uniform(0.85, 0.97), rng.uniform(0.05, 0.6)
            y = lfilter([1.0], [1.0, -2 * r * math.cos(th), r * r], e)
            nk = max(2, T // 800)
            env = np.interp(np.arange(T), np.linspace(0, T - 1, nk),
                            np.abs(rng.standard_normal(nk)) + 0.1)
            y = y * env
            y /= np.sqrt(np.mean(y ** 2)) + 1e-12
            y *= 10 ** (rng.uniform(-2.5, 2.5) / 20)
            src[m, c] = y
    src = src.astype(np.float32)
    return torch.from_numpy(src.sum(1)), torch.from_numpy(src)
