#!/usr/bin/env python
"""Drop-in for ``src/evaluate.py``: SI-SNRi (and SDRi
when mir_eval is importable) of a trained model over a manifest directory.

Same flags and printout as the reference.  Differences, each deliberate:
* the forward runs on the HIP path (a ROCm device is required; the reference
  forces CUDA the same way, evaluate.py:44-46,57-61);
* SI-SNRi of all utterances of a minibatch is computed at once on the device
  in fp64 (``cal_SISNRi_batch``) for any number of speakers C (the reference
  loops over utterances in numpy and hard-codes C = 2, evaluate.py:73-84,117-124);
  ``cal_SISNR`` / ``cal_SISNRi`` keep the reference's numpy definitions
  (evaluate.py:108-144) and are what the batched version is tested against;
* ``--pit_fix 1`` pairs each target with the estimate its best permutation
  assigned to it; the reference's reorder_source uses the permutation itself,
  which mis-pairs 3-cycles for C >= 3 (pit_criterion.py:91-97).  Default 0 keeps
  the reference's pairing (identical for C = 2);
* SDRi uses mir_eval's bss_eval_sources (evaluate.py:10,90-105) when it is
  importable and otherwise ``bss_eval.bss_eval_sources``, a from-scratch
  restatement of the same BSS Eval v3 algorithm (mir_eval is not installed in
  this image, so SDRi parity is unpinned).
"""
import argparse

import numpy as np
import torch

from conv_tasnet import ConvTasNet
from data import AudioDataLoader, AudioDataset
from pit_criterion import cal_loss, cal_si_snr_with_pit
from utils import remove_pad

parser = argparse.ArgumentParser('Evaluate separation performance using Conv-TasNet')
parser.add_argument('--model_path', type=str, required=True,
                    help='Path to model file created by training')
parser.add_argument('--data_dir', type=str, required=True,
                    help='directory including mix.json, s1.json and s2.json')
parser.add_argument('--cal_sdr', type=int, default=0,
                    help='Whether calculate SDR, add this option because calculation of SDR is very slow')
parser.add_argument('--use_cuda', type=int, default=0,
                    help='Whether use GPU (the HIP path always runs on the GPU)')
parser.add_argument('--sample_rate', default=8000, type=int,
                    help='Sample rate')
parser.add_argument('--batch_size', default=1, type=int,
                    help='Batch size')
parser.add_argument('--num_workers', default=2, type=int,
                    help='DataLoader workers reading the wavs (the reference uses 2)')
parser.add_argument('--pit_fix', default=0, type=int,
                    help='1: pair targets with the inverse of the best permutation (C >= 3)')


def reorder_inverse(est, source, lengths):
    """Estimates reordered so that index c holds the estimate PIT assigned to target c."""
    _, perms, idx = cal_si_snr_with_pit(source, est.clone(), lengths)
    best = perms[idx]                                   # [B, C]: estimate i -> target best[b, i]
    inv = torch.empty_like(best)
    inv.scatter_(1, best, torch.arange(best.size(1), device=best.device).expand_as(best).contiguous())
    return torch.gather(est, 1, inv.unsqueeze(-1).expand(-1, -1, est.size(-1)))


class Evaluator:
    """Scores a trained model over one manifest directory (src/evaluate.py:33-90 behaviour:
    the same per-utterance printout and averages).  Minibatches are separated on the
    device, scored there in fp64 (SI-SNRi, cal_SISNRi_batch) and, with --cal_sdr, on the
    host (SDRi, cal_SDRi); ``records`` keeps one (SI-SNRi, SDRi or None) per utterance."""

    def __init__(self, args):
        self.args = args
        self.model = ConvTasNet.load_model(args.model_path)
        print(self.model)
        self.model.eval().cuda()
        dataset = AudioDataset(args.data_dir, args.batch_size, sample_rate=args.sample_rate, segment=-1)
        self.loader = AudioDataLoader(dataset, batch_size=1, num_workers=args.num_workers)
        self.records = []

    def _separate(self, mixture, lengths, source):
        """-> estimates paired with the targets (the reference's reorder, or --pit_fix)."""
        est = self.model(mixture)                                   # [B, C, T]
        _, _, est, paired = cal_loss(source, est, lengths)
        if self.args.pit_fix:
            paired = reorder_inverse(est, source, lengths)
        return paired

    def _score(self, mixture, lengths, source, paired):
        sisnri = cal_SISNRi_batch(source, paired, mixture, lengths).cpu().tolist()
        sdri = [None] * len(sisnri)
        if self.args.cal_sdr:
            mix_u, src_u, est_u = (remove_pad(t, lengths) for t in (mixture, source, paired))
            sdri = [cal_SDRi(src_u[b], est_u[b], mix_u[b]) for b in range(len(sisnri))]
        return list(zip(sisnri, sdri))

    @torch.no_grad()
    def run(self):
        for mixture, lengths, source in self.loader:
            mixture, lengths, source = mixture.cuda(), lengths.cuda(), source.cuda()
            for si, sd in self._score(mixture, lengths, source, self._separate(mixture, lengths, source)):
                self.records.append((si, sd))
                print("Utt", len(self.records))
                if sd is not None:
                    print("\tSDRi={0:.2f}".format(sd))
                print("\tSI-SNRi={0:.2f}".format(si))
        n = len(self.records)
        if self.args.cal_sdr:
            print("Average SDR improvement: {0:.2f}".format(sum(r[1] for r in self.records) / n))
        mean_sisnri = sum(r[0] for r in self.records) / n
        print("Average SISNR improvement: {0:.2f}".format(mean_sisnri))
        return mean_sisnri


def evaluate(args):
    """src/evaluate.py:33's entry point: score the model, return the mean SI-SNRi."""
    return Evaluator(args).run()


def cal_SDRi(src_ref, src_est, mix):
    """evaluate.py:90-105 (C speakers): mean over sources of SDR(est) - SDR(mixture)."""
    try:
        from mir_eval.separation import bss_eval_sources
    except ImportError:          # this image: the from-scratch BSS Eval v3 (parity unpinned)
        from bss_eval import bss_eval_sources
    src_anchor = np.stack([mix] * src_ref.shape[0], axis=0)
    sdr, sir, sar, popt = bss_eval_sources(src_ref, src_est)
    sdr0, sir0, sar0, popt0 = bss_eval_sources(src_ref, src_anchor)
    return float(np.mean(sdr - sdr0))


def cal_SISNRi(src_ref, src_est, mix):
    """evaluate.py:108-125 for C speakers: mean over c of SI-SNR(ref_c, est_c) - SI-SNR(ref_c, mix)
    (for C = 2 the same operations in the same order as the reference)."""
    acc = 0.0
    for c in range(src_ref.shape[0]):
        acc = acc + (cal_SISNR(src_ref[c], src_est[c]) - cal_SISNR(src_ref[c], mix))
    return acc / src_ref.shape[0]


def cal_SISNR(ref_sig, out_sig, eps=1e-8):
    """evaluate.py:128-144: scale-invariant SNR in dB of one signal pair (numpy)."""
    assert len(ref_sig) == len(out_sig)
    ref_sig = ref_sig - np.mean(ref_sig)
    out_sig = out_sig - np.mean(out_sig)
    ref_energy = np.sum(ref_sig ** 2) + eps
    proj = np.sum(ref_sig * out_sig) * ref_sig / ref_energy
    noise = out_sig - proj
    ratio = np.sum(proj ** 2) / (np.sum(noise ** 2) + eps)
    return 10 * np.log(ratio + eps) / np.log(10.0)


def _sisnr_rows(ref, out, mask, n, eps):
    """cal_SISNR over the last dim of fp64 tensors, restricted to mask (n valid samples)."""
    ref = (ref - (ref * mask).sum(-1, keepdim=True) / n.unsqueeze(-1)) * mask
    out = (out - (out * mask).sum(-1, keepdim=True) / n.unsqueeze(-1)) * mask
    ref_energy = (ref * ref).sum(-1, keepdim=True) + eps
    proj = (ref * out).sum(-1, keepdim=True) * ref / ref_energy
    noise = out - proj
    ratio = (proj * proj).sum(-1) / ((noise * noise).sum(-1) + eps)
    return 10 * torch.log(ratio + eps) / np.log(10.0)


def cal_SISNRi_batch(source, estimate, mixture, lengths, eps=1e-8):
    """SI-SNRi of every utterance of a padded batch at once (fp64, on the tensors' device):
    source/estimate [B, C, T], mixture [B, T], lengths [B] -> [B]; utterance b uses its first
    lengths[b] samples, as cal_SISNRi on remove_pad output (evaluate.py:67-84)."""
    B, C, T = source.shape
    dev = source.device
    lengths = lengths.to(dev)
    mask = (torch.arange(T, device=dev).unsqueeze(0) < lengths.unsqueeze(1)).double().unsqueeze(1).expand(B, C, T)
    n = lengths.double().unsqueeze(1).expand(B, C)
    s, e = source.double(), estimate.double()
    m = mixture.double().unsqueeze(1).expand(B, C, T)
    return (_sisnr_rows(s, e, mask, n, eps) - _sisnr_rows(s, m, mask, n, eps)).mean(1)


if __name__ == '__main__':
    args = parser.parse_args()
    print(args)
    evaluate(args)
