"""Drop-in for ``src/data.py``: the reference's minibatch
construction, segmentation and padding, reading wav files without librosa.

Same classes and functions: ``AudioDataset`` (length-sorted buckets of
``segment``-second pieces, data.py:32-118), ``AudioDataLoader``
(data.py:121-128), ``_collate_fn`` (data.py:131-156), ``EvalDataset`` /
``EvalDataLoader`` / ``_collate_fn_eval`` (data.py:162-233),
``load_mixtures_and_sources``, ``load_mixtures`` and ``pad_list``
(data.py:237-299).  A minibatch entry is
``[mix_infos, s1_infos, ..., sC_infos, sample_rate, segment_len]`` — the
reference's layout for two speakers, generalized to the C speakers whose
``s{c}.json`` manifests exist (the reference hard-codes s1/s2, data.py:43-51,258).
As in the reference, a minibatch is ONE dataset item: the loaders run with
``batch_size=1`` and ``batch_size`` of the dataset counts segments
(SURVEY.md Appendix A item 12).

Distributed training: ``MinibatchSampler`` gives every rank an equal, disjoint
share of the minibatches (DDP needs the same number of steps on every rank);
the reference trains in one process (nn.DataParallel, train.py:121) and has none.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np
import torch
import torch.utils.data as data

from audio_io import read_wav
from preprocess import preprocess_one_dir


def _load_json(path):
    with open(path, 'r') as f:
        return json.load(f)


def speaker_names(json_dir):
    """['s1', 's2', ...]: every consecutive s{c}.json manifest in json_dir."""
    names, c = [], 1
    while os.path.exists(os.path.join(json_dir, f"s{c}.json")):
        names.append(f"s{c}")
        c += 1
    if not names:
        raise FileNotFoundError(f"{json_dir}: no s1.json speaker manifest")
    return names


def _sort(infos):
    """data.py:53-54: by #samples, longest first (stable: ties keep manifest order)."""
    return sorted(infos, key=lambda info: int(info[1]), reverse=True)


class AudioDataset(data.Dataset):

    def __init__(self, json_dir, batch_size, sample_rate=8000, segment=4.0, cv_maxlen=8.0):
        """data.py:34-112.  json_dir holds mix.json and s1.json, s2.json, ...; each
        manifest is a list of [wav_path, #samples].  segment < 0: whole utterances
        (cross validation), skipping minibatches whose longest one exceeds cv_maxlen s."""
        super(AudioDataset, self).__init__()
        mix_infos = _sort(_load_json(os.path.join(json_dir, 'mix.json')))
        spk_infos = [_sort(_load_json(os.path.join(json_dir, s + '.json'))) for s in speaker_names(json_dir)]
        self.num_spk = len(spk_infos)
        minibatch = []
        if segment >= 0.0:
            segment_len = int(segment * sample_rate)
            drop_utt, drop_len = 0, 0
            for _, sample in mix_infos:
                if sample < segment_len:
                    drop_utt += 1
                    drop_len += sample
            print("Drop {} utts({:.2f} h) which is short than {} samples".format(
                drop_utt, drop_len / sample_rate / 36000, segment_len))
            start = 0
            while True:
                num_segments, end = 0, start
                part_mix, part_spk = [], [[] for _ in spk_infos]
                while num_segments < batch_size and end < len(mix_infos):
                    utt_len = int(mix_infos[end][1])
                    if utt_len >= segment_len:              # shorter utterances are skipped
                        num_segments += math.ceil(utt_len / segment_len)
                        if num_segments > batch_size:
                            if start == end:                # alone over the budget: skip it
                                end += 1
                            break
                        part_mix.append(mix_infos[end])
                        for part, infos in zip(part_spk, spk_infos):
                            part.append(infos[end])
                    end += 1
                if len(part_mix) > 0:
                    minibatch.append([part_mix, *part_spk, sample_rate, segment_len])
                if end == len(mix_infos):
                    break
                start = end
        else:
            start = 0
            while start < len(mix_infos):
                end = min(len(mix_infos), start + batch_size)
                if int(mix_infos[start][1]) > cv_maxlen * sample_rate:   # OOM guard: skip long audio
                    start = end
                    continue
                minibatch.append([mix_infos[start:end], *[infos[start:end] for infos in spk_infos],
                                  sample_rate, segment])
                if end == len(mix_infos):
                    break
                start = end
        self.minibatch = minibatch

    def __getitem__(self, index):
        return self.minibatch[index]

    def __len__(self):
        return len(self.minibatch)


class AudioDataLoader(data.DataLoader):
    """data.py:121-128: batch_size stays 1 — one item is one whole minibatch."""

    def __init__(self, *args, **kwargs):
        kwargs.setdefault("collate_fn", _collate_fn)
        super(AudioDataLoader, self).__init__(*args, **kwargs)


class MinibatchSampler(torch.utils.data.Sampler):
    """Rank `rank` of `world` takes order[rank::world] of the minibatches; with
    shuffle the order is a permutation seeded by (seed + epoch), identical on all
    ranks (call set_epoch each epoch).

    drop_last=True (training): only the first world * (n // world) minibatches are
    used, so every rank runs the same number of DDP steps.  drop_last=False
    (validation): every minibatch is used, the low ranks taking the remainder, so
    the cross-validation loss that drives LR halving / early stopping sees the
    whole set (the solver all-reduces (sum, count) pairs, so unequal shards are
    fine there)."""

    def __init__(self, dataset, rank=0, world=1, shuffle=False, seed=0, drop_last=True):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world size {world}")
        self.n, self.rank, self.world = len(dataset), rank, world
        self.shuffle, self.seed, self.epoch = bool(shuffle), seed, 0
        self.drop_last = bool(drop_last)

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def _order(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            return torch.randperm(self.n, generator=g).tolist()
        return list(range(self.n))

    def __iter__(self):
        order = self._order()
        if self.drop_last:
            order = order[:(self.n // self.world) * self.world]
        return iter(order[self.rank::self.world])

    def __len__(self):
        if self.drop_last:
            return self.n // self.world
        return len(range(self.rank, self.n, self.world))


def _collate_fn(batch):
    """data.py:131-156 -> (mixtures_pad [B, T], ilens [B], sources_pad [B, C, T])."""
    assert len(batch) == 1
    mixtures, sources = load_mixtures_and_sources(batch[0])
    ilens = np.array([mix.shape[0] for mix in mixtures])
    pad_value = 0
    mixtures_pad = pad_list([torch.from_numpy(mix).float() for mix in mixtures], pad_value)
    ilens = torch.from_numpy(ilens)
    sources_pad = pad_list([torch.from_numpy(s).float() for s in sources], pad_value)
    sources_pad = sources_pad.permute((0, 2, 1)).contiguous()   # B x T x C -> B x C x T
    return mixtures_pad, ilens, sources_pad


class EvalDataset(data.Dataset):

    def __init__(self, mix_dir, mix_json, batch_size, sample_rate=8000):
        """data.py:164-193: mixtures only; mix_dir (a manifest is written into it) or mix_json."""
        super(EvalDataset, self).__init__()
        assert mix_dir is not None or mix_json is not None
        if mix_dir is not None:
            preprocess_one_dir(mix_dir, mix_dir, 'mix', sample_rate=sample_rate)
            mix_json = os.path.join(mix_dir, 'mix.json')
        mix_infos = _sort(_load_json(mix_json))
        minibatch = []
        start = 0
        while True:
            end = min(len(mix_infos), start + batch_size)
            minibatch.append([mix_infos[start:end], sample_rate])
            if end == len(mix_infos):
                break
            start = end
        self.minibatch = minibatch

    def __getitem__(self, index):
        return self.minibatch[index]

    def __len__(self):
        return len(self.minibatch)


class EvalDataLoader(data.DataLoader):
    """data.py:202-209."""

    def __init__(self, *args, **kwargs):
        kwargs.setdefault("collate_fn", _collate_fn_eval)
        super(EvalDataLoader, self).__init__(*args, **kwargs)


def _collate_fn_eval(batch):
    """data.py:212-233 -> (mixtures_pad [B, T], ilens [B], filenames)."""
    assert len(batch) == 1
    mixtures, filenames = load_mixtures(batch[0])
    ilens = np.array([mix.shape[0] for mix in mixtures])
    mixtures_pad = pad_list([torch.from_numpy(mix).float() for mix in mixtures], 0)
    ilens = torch.from_numpy(ilens)
    return mixtures_pad, ilens, filenames


# ------------------------------ utils ------------------------------------
def _read(path, sample_rate):
    return read_wav(path, sr=sample_rate)[0]


def load_mixtures_and_sources(batch):
    """data.py:237-271 -> (mixtures: B arrays [T], sources: B arrays [T, C]); with
    segment_len >= 0 every utterance is cut into segment_len pieces plus a last
    piece aligned to its end."""
    mixtures, sources = [], []
    mix_infos, spk_infos = batch[0], batch[1:-2]
    sample_rate, segment_len = batch[-2], batch[-1]
    for i, mix_info in enumerate(mix_infos):
        infos = [s[i] for s in spk_infos]
        assert all(mix_info[1] == info[1] for info in infos)
        mix = _read(mix_info[0], sample_rate)
        s = np.stack([_read(info[0], sample_rate) for info in infos], axis=1)   # T x C
        utt_len = mix.shape[-1]
        if segment_len >= 0:
            for j in range(0, utt_len - segment_len + 1, segment_len):
                mixtures.append(mix[j:j + segment_len])
                sources.append(s[j:j + segment_len])
            if utt_len % segment_len != 0:
                mixtures.append(mix[-segment_len:])
                sources.append(s[-segment_len:])
        else:
            mixtures.append(mix)
            sources.append(s)
    return mixtures, sources


def load_mixtures(batch):
    """data.py:274-290 -> (mixtures: B arrays [T], filenames)."""
    mixtures, filenames = [], []
    mix_infos, sample_rate = batch
    for mix_info in mix_infos:
        mixtures.append(_read(mix_info[0], sample_rate))
        filenames.append(mix_info[0])
    return mixtures, filenames


def pad_list(xs, pad_value):
    """data.py:293-299: stack along a new batch dim, padding dim 0 to the longest."""
    n_batch = len(xs)
    max_len = max(x.size(0) for x in xs)
    pad = xs[0].new(n_batch, max_len, *xs[0].size()[1:]).fill_(pad_value)
    for i in range(n_batch):
        pad[i, :xs[i].size(0)] = xs[i]
    return pad
