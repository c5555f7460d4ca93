#!/usr/bin/env python
"""Drop-in for ``src/separate.py``: separate every
mixture of a directory or manifest and write PCM_16 wavs.

For each input ``<dir>/<name>.wav`` the output directory receives
``<stem>.wav`` (the mixture, trimmed to its length) and ``<stem>_s<c>.wav``
(estimate c, 1-based).  ``<stem>`` reproduces the reference's
``os.path.basename(f).strip('.wav')``: str.strip removes any of the characters
``.``, ``w``, ``a``, ``v`` from BOTH ends, so ``"wave.wav"`` becomes ``"e"``
 — kept so existing scoring scripts find the
same files.  Same command-line flags as the reference.

The forward is the HIP path (``ConvTasNet`` on a ROCm device; the reference
also requires a GPU, separate.py:44-46,64-66), in inference mode; wavs are
written by audio_io (soundfile is not installed).  For frame-by-frame causal
models see ``streaming.StreamingSeparator``.
"""
import argparse
import os

import torch

from audio_io import write_wav
from conv_tasnet import ConvTasNet
from data import EvalDataLoader, EvalDataset
from utils import remove_pad

parser = argparse.ArgumentParser('Separate speech using Conv-TasNet')
parser.add_argument('--model_path', type=str, required=True,
                    help='Path to model file created by training')
parser.add_argument('--mix_dir', type=str, default=None,
                    help='Directory including mixture wav files')
parser.add_argument('--mix_json', type=str, default=None,
                    help='Json file including mixture wav files')
parser.add_argument('--out_dir', type=str, default='exp/result',
                    help='Directory putting separated wav files')
parser.add_argument('--use_cuda', type=int, default=0,
                    help='Whether use GPU to separate speech (the HIP path always runs on the GPU)')
parser.add_argument('--sample_rate', default=8000, type=int,
                    help='Sample rate')
parser.add_argument('--batch_size', default=1, type=int,
                    help='Batch size')


def output_stem(path: str) -> str:
    """Base name of the output files for mixture ``path`` (reference naming)."""
    return os.path.basename(path).strip('.wav')


class Separator:
    """A loaded model on the device plus the writer for its estimates."""

    def __init__(self, model_path: str, sample_rate: int, device=None):
        self.model = ConvTasNet.load_model(model_path)
        print(self.model)
        self.device = torch.device(device or "cuda")
        self.model.eval().to(self.device)
        self.sample_rate = sample_rate

    @torch.no_grad()
    def estimate(self, mixture: torch.Tensor, lengths: torch.Tensor):
        """Padded mixtures [B, T] -> (trimmed mixtures, trimmed estimates [C, T_b]) per utterance."""
        mixture, lengths = mixture.to(self.device), lengths.to(self.device)
        est = self.model(mixture)
        return remove_pad(mixture, lengths), remove_pad(est, lengths)

    def save(self, out_dir: str, name: str, mixture, estimates):
        stem = os.path.join(out_dir, output_stem(name))
        write_wav(stem + '.wav', mixture, self.sample_rate)
        for c, est in enumerate(estimates, start=1):
            write_wav('%s_s%d.wav' % (stem, c), est, self.sample_rate)

    def run(self, loader, out_dir: str):
        os.makedirs(out_dir, exist_ok=True)
        for mixture, lengths, names in loader:
            mixes, ests = self.estimate(mixture, lengths)
            for name, mix, est in zip(names, mixes, ests):
                self.save(out_dir, name, mix, est)


def separate(args):
    if args.mix_dir is None and args.mix_json is None:
        print("Must provide mix_dir or mix_json! When providing mix_dir, "
              "mix_json is ignored.")
    sep = Separator(args.model_path, args.sample_rate)
    dataset = EvalDataset(args.mix_dir, args.mix_json, batch_size=args.batch_size, sample_rate=args.sample_rate)
    sep.run(EvalDataLoader(dataset, batch_size=1), args.out_dir)


if __name__ == '__main__':
    args = parser.parse_args()
    print(args)
    separate(args)
