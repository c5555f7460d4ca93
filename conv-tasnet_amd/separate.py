#!/usr/bin/env python
"""Drop-in for ``src/separate.py``: separate every
mixture of a directory or manifest and write PCM_16 wavs
(``<name>.wav`` = the mixture, ``<name>_s<c>.wav`` = estimate c).

Same flags and output names as the reference, including its
``os.path.basename(f).strip('.wav')`` naming (strip removes any of the
characters ``.wav`` from both ends of the name).
The forward runs on the HIP path (a ROCm device is required; the reference
forces CUDA too, separate.py:44-46,64-66); wavs are written by audio_io
(soundfile is not installed).
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


def separate(args):
    if args.mix_dir is None and args.mix_json is None:
        print("Must provide mix_dir or mix_json! When providing mix_dir, "
              "mix_json is ignored.")

    model = ConvTasNet.load_model(args.model_path)
    print(model)
    model.eval()
    model.cuda()

    eval_dataset = EvalDataset(args.mix_dir, args.mix_json,
                               batch_size=args.batch_size,
                               sample_rate=args.sample_rate)
    eval_loader = EvalDataLoader(eval_dataset, batch_size=1)
    os.makedirs(args.out_dir, exist_ok=True)

    def write(inputs, filename, sr=args.sample_rate):
        write_wav(filename, inputs, sr)

    with torch.no_grad():
        for (i, data) in enumerate(eval_loader):
            mixture, mix_lengths, filenames = data
            mixture, mix_lengths = mixture.cuda(), mix_lengths.cuda()
            estimate_source = model(mixture)  # [B, C, T]
            flat_estimate = remove_pad(estimate_source, mix_lengths)
            mixture = remove_pad(mixture, mix_lengths)
            for b, filename in enumerate(filenames):
                filename = os.path.join(args.out_dir, os.path.basename(filename).strip('.wav'))
                write(mixture[b], filename + '.wav')
                C = flat_estimate[b].shape[0]
                for c in range(C):
                    write(flat_estimate[b][c], filename + '_s{}.wav'.format(c + 1))


if __name__ == '__main__':
    args = parser.parse_args()
    print(args)
    separate(args)
