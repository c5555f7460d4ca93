"""Drop-in for ``src/pit_criterion.py`` (PIT SI-SNR loss) on MI355X.

``cal_loss`` runs the batched HIP reduction kernels of ``libctn_hip.so``
(ctn_pit_forward / ctn_pit_backward): no per-utterance Python loop, fp64
sums, one element-wise backward pass.  Semantics kept from the reference:
``estimate_source`` is masked in place beyond each length and returned
(pit_criterion.py:37-38,24); max_snr is averaged over speakers (:75); loss is
-mean(max_snr) (:22); the reordered estimate uses perm, not its inverse (:91-97).
"""
from __future__ import annotations

from itertools import permutations

import torch

import ctn_lib as L
import ctn_ops as ops

EPS = 1e-8


def cal_loss(source, estimate_source, source_lengths):
    """pit_criterion.py:12-24 -> (loss, max_snr [B,1], estimate_source, reorder_estimate_source)."""
    loss, max_snr, est, best = ops.PITFn.apply(source, estimate_source, source_lengths)
    C = source.size(1)
    perms = source.new_tensor(list(permutations(range(C))), dtype=torch.long)
    reorder_estimate_source = reorder_source(est.detach(), perms, best)
    return loss, max_snr, est, reorder_estimate_source


def cal_si_snr_with_pit(source, estimate_source, source_lengths):
    """pit_criterion.py:27-76 -> (max_snr [B,1], perms [C!,C], max_snr_idx [B])."""
    _, max_snr, _, best = ops.PITFn.apply(source, estimate_source, source_lengths)
    C = source.size(1)
    perms = source.new_tensor(list(permutations(range(C))), dtype=torch.long)
    return max_snr, perms, best


def reorder_source(source, perms, max_snr_idx):
    """pit_criterion.py:79-98 (same indexing: reorder[b, c] = source[b, perm[c]])."""
    sel = torch.index_select(perms, dim=0, index=max_snr_idx)          # [B, C]
    return torch.gather(source, 1, sel.unsqueeze(-1).expand(-1, -1, source.size(-1)))


def get_mask(source, source_lengths):
    """pit_criterion.py:101-113 -> [B, 1, T]."""
    B, _, T = source.size()
    t = torch.arange(T, device=source.device).unsqueeze(0)
    return (t < source_lengths.to(source.device).view(-1, 1)).to(source.dtype).unsqueeze(1)
