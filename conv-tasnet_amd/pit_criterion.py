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
_PERMS = {}


def _perms(C, device):
    """range(C)'s permutations as a device tensor, built once per (C, device): a tensor
    made from a host list is a synchronous pageable copy, which in the training step
    stalled the host until the GPU had finished the forward pass."""
    if C > 10:   # 11! rows x C is 0.4 GB and grows C-fold: the reference's table stops being buildable
        raise L.CtnLibraryError(f"cal_si_snr_with_pit: the permutation table of C={C} speakers has {C}! "
                                "rows; cal_loss (assignment search on the device) supports C <= 16")
    key = (C, str(device))
    t = _PERMS.get(key)
    if t is None:
        t = torch.tensor(list(permutations(range(C))), dtype=torch.long).to(device)
        _PERMS[key] = t
    return t


def cal_loss(source, estimate_source, source_lengths):
    """pit_criterion.py:12-24 -> (loss, max_snr [B,1], estimate_source, reorder_estimate_source).
    The reordered estimate comes from the loss kernel pass itself (no index_select/gather)."""
    loss, max_snr, est, _, reorder_estimate_source = ops.PITFn.apply(source, estimate_source, source_lengths)
    return loss, max_snr, est, reorder_estimate_source


def cal_si_snr_with_pit(source, estimate_source, source_lengths):
    """pit_criterion.py:27-76 -> (max_snr [B,1], perms [C!,C], max_snr_idx [B])."""
    _, max_snr, _, best, _ = ops.PITFn.apply(source, estimate_source, source_lengths)
    return max_snr, _perms(source.size(1), source.device).clone(), best


def reorder_source(source, perms, max_snr_idx):
    """pit_criterion.py:79-98 (same indexing: reorder[b, c] = source[b, perm[c]])."""
    sel = torch.index_select(perms, dim=0, index=max_snr_idx)          # [B, C]
    return torch.gather(source, 1, sel.unsqueeze(-1).expand(-1, -1, source.size(-1)))


def get_mask(source, source_lengths):
    """pit_criterion.py:101-113 -> [B, 1, T]."""
    B, _, T = source.size()
    t = torch.arange(T, device=source.device).unsqueeze(0)
    return (t < source_lengths.to(source.device).view(-1, 1)).to(source.dtype).unsqueeze(1)
