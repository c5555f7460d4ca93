#!/usr/bin/env python
"""Drop-in for ``src/preprocess.py``: json manifests of
``[wav_path, #samples]`` per speaker directory (preprocess.py:12-34), read
without librosa (audio_io).

Same functions and flags.  Differences, each deliberate:
* ``#samples`` comes from the WAV header when the file is already at
  ``sample_rate`` (librosa.load decodes the whole file for it); otherwise it is
  the resampled length, as librosa's;
* files are listed in sorted order (the reference keeps ``os.listdir`` order,
  which is unspecified) so manifests are reproducible;
* ``preprocess`` handles ``mix`` plus every consecutive ``s1``, ``s2``, ``s3`` ...
  directory present (the reference hard-codes mix/s1/s2, preprocess.py:30).
"""
import argparse
import json
import os

from audio_io import read_wav, read_wav_info


def preprocess_one_dir(in_dir, out_dir, out_filename, sample_rate=8000):
    """preprocess.py:12-25: write out_dir/out_filename.json = [[path, #samples], ...]."""
    file_infos = []
    in_dir = os.path.abspath(in_dir)
    for wav_file in sorted(os.listdir(in_dir)):
        if not wav_file.endswith('.wav'):
            continue
        wav_path = os.path.join(in_dir, wav_file)
        n, rate, _ = read_wav_info(wav_path)
        if rate != sample_rate:
            n = len(read_wav(wav_path, sr=sample_rate)[0])
        file_infos.append((wav_path, n))
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, out_filename + '.json'), 'w') as f:
        json.dump(file_infos, f, indent=4)


def speaker_dirs(split_dir):
    """['mix', 's1', 's2', ...]: the mixture and every consecutive s{c} directory."""
    names, c = ['mix'], 1
    while os.path.isdir(os.path.join(split_dir, f's{c}')):
        names.append(f's{c}')
        c += 1
    return names


def preprocess(args):
    """preprocess.py:28-34 over tr/cv/tt."""
    for data_type in ['tr', 'cv', 'tt']:
        split = os.path.join(args.in_dir, data_type)
        for speaker in speaker_dirs(split):
            preprocess_one_dir(os.path.join(split, speaker), os.path.join(args.out_dir, data_type), speaker,
                               sample_rate=args.sample_rate)


if __name__ == "__main__":
    parser = argparse.ArgumentParser("WSJ0 data preprocessing")
    parser.add_argument('--in-dir', type=str, default=None,
                        help='Directory path of wsj0 including tr, cv and tt')
    parser.add_argument('--out-dir', type=str, default=None,
                        help='Directory path to put output files')
    parser.add_argument('--sample-rate', type=int, default=8000,
                        help='Sample rate of audio file')
    args = parser.parse_args()
    print(args)
    preprocess(args)
