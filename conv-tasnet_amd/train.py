#!/usr/bin/env python
"""Drop-in for ``src/train.py``: the same flags and
defaults (train.py:15-98) and the same Solver loop, on the HIP path.

    python train.py --train_dir data/tr --valid_dir data/cv ...            # one GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...       # one process per GPU

Differences, each deliberate:
* multi-GPU is one process per GPU (DDP over RCCL, ``nccl`` backend) instead of
  nn.DataParallel (train.py:121): every rank trains its own share of the
  minibatches (data.MinibatchSampler) and DDP averages the gradients; on one
  GPU the model is wrapped in ``Single`` so ``.module`` works as the solver
  expects (solver.py:55,87,131);
* ``--optimizer adam`` is ctn_optim.Adam (torch.optim.Adam's update and
  state_dict, one launch per step); ``sgd`` is torch.optim.SGD;
* ``--shuffle`` reshuffles the minibatch order per epoch through the sampler
  (a DataLoader cannot take both a sampler and shuffle=True);
* ``--bf16 1`` trains with bf16 activations (fp32 parameters, statistics and
  optimizer state); the default 0 is fp32, the reference's arithmetic.
"""
import argparse
import os

import torch
import torch.distributed as dist

from conv_tasnet import ConvTasNet
from data import AudioDataLoader, AudioDataset, MinibatchSampler
from solver import Solver

parser = argparse.ArgumentParser(
    "Fully-Convolutional Time-domain Audio Separation Network (Conv-TasNet) "
    "with Permutation Invariant Training")
# Task related
parser.add_argument('--train_dir', type=str, default=None,
                    help='directory including mix.json, s1.json and s2.json')
parser.add_argument('--valid_dir', type=str, default=None,
                    help='directory including mix.json, s1.json and s2.json')
parser.add_argument('--sample_rate', default=8000, type=int,
                    help='Sample rate')
parser.add_argument('--segment', default=4, type=float,
                    help='Segment length (seconds)')
parser.add_argument('--cv_maxlen', default=8, type=float,
                    help='max audio length (seconds) in cv, to avoid OOM issue.')
# Network architecture
parser.add_argument('--N', default=256, type=int,
                    help='Number of filters in autoencoder')
parser.add_argument('--L', default=20, type=int,
                    help='Length of the filters in samples (40=5ms at 8kHZ)')
parser.add_argument('--B', default=256, type=int,
                    help='Number of channels in bottleneck 1 × 1-conv block')
parser.add_argument('--H', default=512, type=int,
                    help='Number of channels in convolutional blocks')
parser.add_argument('--P', default=3, type=int,
                    help='Kernel size in convolutional blocks')
parser.add_argument('--X', default=8, type=int,
                    help='Number of convolutional blocks in each repeat')
parser.add_argument('--R', default=4, type=int,
                    help='Number of repeats')
parser.add_argument('--C', default=2, type=int,
                    help='Number of speakers')
parser.add_argument('--norm_type', default='gLN', type=str,
                    choices=['gLN', 'cLN', 'BN'], help='Layer norm type')
parser.add_argument('--causal', type=int, default=0,
                    help='Causal (1) or noncausal(0) training')
parser.add_argument('--mask_nonlinear', default='relu', type=str,
                    choices=['relu', 'softmax'], help='non-linear to generate mask')
# Training config
parser.add_argument('--use_cuda', type=int, default=1,
                    help='Whether use GPU')
parser.add_argument('--epochs', default=30, type=int,
                    help='Number of maximum epochs')
parser.add_argument('--half_lr', dest='half_lr', default=0, type=int,
                    help='Halving learning rate when get small improvement')
parser.add_argument('--early_stop', dest='early_stop', default=0, type=int,
                    help='Early stop training when no improvement for 10 epochs')
parser.add_argument('--max_norm', default=5, type=float,
                    help='Gradient norm threshold to clip')
# minibatch
parser.add_argument('--shuffle', default=0, type=int,
                    help='reshuffle the data at every epoch')
parser.add_argument('--batch_size', default=128, type=int,
                    help='Batch size')
parser.add_argument('--num_workers', default=4, type=int,
                    help='Number of workers to generate minibatch')
# optimizer
parser.add_argument('--optimizer', default='adam', type=str,
                    choices=['sgd', 'adam'],
                    help='Optimizer (support sgd and adam now)')
parser.add_argument('--lr', default=1e-3, type=float,
                    help='Init learning rate')
parser.add_argument('--momentum', default=0.0, type=float,
                    help='Momentum for optimizer')
parser.add_argument('--l2', default=0.0, type=float,
                    help='weight decay (L2 penalty)')
# save and load model
parser.add_argument('--save_folder', default='exp/temp',
                    help='Location to save epoch models')
parser.add_argument('--checkpoint', dest='checkpoint', default=0, type=int,
                    help='Enables checkpoint saving of model')
parser.add_argument('--continue_from', default='',
                    help='Continue from checkpoint model')
parser.add_argument('--model_path', default='final.pth.tar',
                    help='Location to save best validation model')
# logging
parser.add_argument('--print_freq', default=10, type=int,
                    help='Frequency of printing training infomation')
parser.add_argument('--visdom', dest='visdom', type=int, default=0,
                    help='Turn on visdom graphing')
parser.add_argument('--visdom_epoch', dest='visdom_epoch', type=int, default=0,
                    help='Turn on visdom graphing each epoch')
parser.add_argument('--visdom_id', default='TasNet training',
                    help='Identifier for visdom run')
# MI355X path
parser.add_argument('--bf16', default=0, type=int,
                    help='1: bf16 activations (fp32 parameters, statistics and optimizer state)')


class Single(torch.nn.Module):
    """One-GPU stand-in for nn.DataParallel: exposes ``.module`` (solver.py:55)."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)


class FlatDP(Single):
    """One process per GPU: the gradients are averaged across ranks by one flat RCCL
    all-reduce after backward (ctn_dist.FlatGradAllReduce, run by the solver), which keeps
    the TemporalBlock gradient reductions deferred and batched; DistributedDataParallel's
    hooks need every gradient as it arrives (bench at world size 1: 2124 utt/s, DDP 1990, no exchange 2131)."""

    def __init__(self, module):
        super().__init__(module)
        import ctn_dist
        self.grad_sync = ctn_dist.FlatGradAllReduce(module.parameters())


def main(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    # data
    tr_dataset = AudioDataset(args.train_dir, args.batch_size,
                              sample_rate=args.sample_rate, segment=args.segment)
    cv_dataset = AudioDataset(args.valid_dir, batch_size=1,  # 1 -> use less GPU memory to do cv
                              sample_rate=args.sample_rate,
                              segment=-1, cv_maxlen=args.cv_maxlen)  # -1 -> use full audio
    tr_loader = AudioDataLoader(tr_dataset, batch_size=1,
                                sampler=MinibatchSampler(tr_dataset, rank, world, shuffle=args.shuffle),
                                num_workers=args.num_workers)
    cv_loader = AudioDataLoader(cv_dataset, batch_size=1,
                                sampler=MinibatchSampler(cv_dataset, rank, world, drop_last=False), num_workers=0)
    data = {'tr_loader': tr_loader, 'cv_loader': cv_loader}
    # model
    model = ConvTasNet(args.N, args.L, args.B, args.H, args.P, args.X, args.R,
                       args.C, norm_type=args.norm_type, causal=args.causal,
                       mask_nonlinear=args.mask_nonlinear)
    if args.bf16:
        model.act_dtype = torch.bfloat16
    if rank == 0:
        print(model)
    if args.use_cuda:
        model.cuda()
        if world == 1:
            model = Single(model)
        elif args.norm_type != 'BN':
            model = FlatDP(model)
        else:
            # BatchNorm: DDP also broadcasts rank 0's running statistics each forward.
            # Gradients as views into the RCCL buckets and a static graph: at world size 1
            # on one MI355X this took the DDP step from 21.8 to 18.8 ms (plain 18.3 ms)
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local], gradient_as_bucket_view=True,
                                                              static_graph=True)
    else:
        model = Single(model)
    # optimizer
    if args.optimizer == 'sgd':
        optimizer = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=args.momentum,
                                    weight_decay=args.l2)
    elif args.optimizer == 'adam':
        import ctn_optim
        optimizer = ctn_optim.Adam(model.parameters(), lr=args.lr, weight_decay=args.l2)
    else:
        print("Not support optimizer")
        return
    solver = Solver(data, model, optimizer, args)
    solver.train()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    args = parser.parse_args()
    print(args)
    main(args)
