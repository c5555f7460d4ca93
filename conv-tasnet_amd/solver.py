"""Drop-in for ``src/solver.py``: the epoch loop with
checkpoint / resume packages, learning-rate halving and early stopping.

The control rules are the reference's (solver.py:69-156): a checkpoint
``epoch%d.pth.tar`` after each training pass when ``checkpoint`` is set (written
before that epoch's losses are recorded, as in the reference), the LR of
``param_groups[0]`` halved once three consecutive validation losses failed to
improve on their predecessor, a stop after ten when ``early_stop`` is set, and
``model_path`` rewritten whenever the validation loss is the best so far.
Packages are ``ConvTasNet.serialize`` dicts, so reference checkpoints resume
here and the other way round.  The step is solver.py:172-188; with the
parameters on a ROCm device the clip is ``ctn_optim.clip_grad_norm_`` (one
launch pair over all tensors).

Differences, each deliberate:
* distributed (one process per GPU, DDP): every rank runs its share of the
  minibatches (data.MinibatchSampler), epoch losses are averaged over the ranks
  before any decision so all ranks halve and stop together, and only rank 0
  writes files;
* the reference's ``loss.item()`` after every step (a device sync per step) is
  replaced by a device-side fp64 running sum, read every ``print_freq`` steps
  and at the end of the epoch — the same values (fp32 losses summed in double,
  in order);
* cross validation runs under ``torch.no_grad()`` (the reference builds an
  unused graph);
* visdom plots are skipped with a message when visdom is not importable.
"""
import os
import time

import torch
import torch.distributed as dist

from pit_criterion import cal_loss


def _rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _unwrap(model):
    return model.module if hasattr(model, "module") else model


def _clip_fn(model):
    p = next(iter(model.parameters()), None)
    if p is not None and p.device.type == "cuda" and p.dtype == torch.float32:
        import ctn_optim
        return ctn_optim.clip_grad_norm_
    return torch.nn.utils.clip_grad_norm_


class Solver(object):

    def __init__(self, data, model, optimizer, args):
        self.tr_loader = data['tr_loader']
        self.cv_loader = data['cv_loader']
        self.model = model
        self.optimizer = optimizer

        # Training config
        self.use_cuda = args.use_cuda
        self.epochs = args.epochs
        self.half_lr = args.half_lr
        self.early_stop = args.early_stop
        self.max_norm = args.max_norm
        # save and load model
        self.save_folder = args.save_folder
        self.checkpoint = args.checkpoint
        self.continue_from = args.continue_from
        self.model_path = args.model_path
        # logging
        self.print_freq = args.print_freq
        self.tr_loss = torch.zeros(self.epochs)
        self.cv_loss = torch.zeros(self.epochs)
        self.visdom = args.visdom
        self.visdom_epoch = args.visdom_epoch
        self.visdom_id = args.visdom_id
        self.vis = None
        if self.visdom or self.visdom_epoch:
            try:
                from visdom import Visdom
                self.vis = Visdom(env=self.visdom_id)
            except ImportError:
                print("visdom is not installed: loss plots are skipped")
        self.vis_window = None
        self.rank, self.world = _rank_world()
        self._reset()

    def _reset(self):
        """solver.py:50-67."""
        if self.continue_from:
            print('Loading checkpoint model %s' % self.continue_from)
            package = torch.load(self.continue_from, map_location='cpu', weights_only=True)
            _unwrap(self.model).load_state_dict(package['state_dict'])
            self.optimizer.load_state_dict(package['optim_dict'])
            self.start_epoch = int(package.get('epoch', 1))
            self.tr_loss[:self.start_epoch] = package['tr_loss'][:self.start_epoch]
            self.cv_loss[:self.start_epoch] = package['cv_loss'][:self.start_epoch]
        else:
            self.start_epoch = 0
        os.makedirs(self.save_folder, exist_ok=True)
        self.prev_val_loss = float("inf")
        self.best_val_loss = float("inf")
        self.halving = False
        self.val_no_impv = 0

    def _save(self, file_path, epoch):
        if self.rank != 0:
            return
        m = _unwrap(self.model)
        torch.save(m.serialize(m, self.optimizer, epoch, tr_loss=self.tr_loss, cv_loss=self.cv_loss), file_path)

    def train(self):
        """solver.py:69-156."""
        for epoch in range(self.start_epoch, self.epochs):
            print("Training...")
            self.model.train()
            start = time.time()
            tr_avg_loss = self._run_one_epoch(epoch)
            print('-' * 85)
            print('Train Summary | End of Epoch {0} | Time {1:.2f}s | '
                  'Train Loss {2:.3f}'.format(epoch + 1, time.time() - start, tr_avg_loss))
            print('-' * 85)

            if self.checkpoint:
                file_path = os.path.join(self.save_folder, 'epoch%d.pth.tar' % (epoch + 1))
                self._save(file_path, epoch + 1)
                print('Saving checkpoint model to %s' % file_path)

            print('Cross validation...')
            self.model.eval()
            val_loss = self._run_one_epoch(epoch, cross_valid=True)
            print('-' * 85)
            print('Valid Summary | End of Epoch {0} | Time {1:.2f}s | '
                  'Valid Loss {2:.3f}'.format(epoch + 1, time.time() - start, val_loss))
            print('-' * 85)

            # learning-rate halving / early stop (against the PREVIOUS epoch's loss)
            if self.half_lr:
                if val_loss >= self.prev_val_loss:
                    self.val_no_impv += 1
                    if self.val_no_impv >= 3:
                        self.halving = True
                    if self.val_no_impv >= 10 and self.early_stop:
                        print("No imporvement for 10 epochs, early stopping.")
                        break
                else:
                    self.val_no_impv = 0
            if self.halving:
                optim_state = self.optimizer.state_dict()
                optim_state['param_groups'][0]['lr'] = optim_state['param_groups'][0]['lr'] / 2.0
                self.optimizer.load_state_dict(optim_state)
                print('Learning rate adjusted to: {lr:.6f}'.format(lr=optim_state['param_groups'][0]['lr']))
                self.halving = False
            self.prev_val_loss = val_loss

            self.tr_loss[epoch] = tr_avg_loss
            self.cv_loss[epoch] = val_loss
            if val_loss < self.best_val_loss:
                self.best_val_loss = val_loss
                file_path = os.path.join(self.save_folder, self.model_path)
                self._save(file_path, epoch + 1)
                print("Find better validated model, saving to %s" % file_path)

            if self.vis is not None and self.visdom and self.rank == 0:
                x_axis = torch.arange(1, epoch + 2)
                y_axis = torch.stack((self.tr_loss[0:epoch + 1], self.cv_loss[0:epoch + 1]), dim=1)
                opts = dict(title=self.visdom_id, ylabel='Loss', xlabel='Epoch', legend=['train loss', 'cv loss'])
                if self.vis_window is None:
                    self.vis_window = self.vis.line(X=x_axis, Y=y_axis, opts=opts)
                else:
                    self.vis.line(X=x_axis.unsqueeze(0).expand(y_axis.size(1), x_axis.size(0)).transpose(0, 1),
                                  Y=y_axis, win=self.vis_window, update='replace')

    def _run_one_epoch(self, epoch, cross_valid=False):
        """solver.py:158-210 -> mean loss of the epoch (over all ranks)."""
        start = time.time()
        data_loader = self.tr_loader if not cross_valid else self.cv_loader
        sampler = getattr(data_loader, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        clip = _clip_fn(self.model)
        dev = next(self.model.parameters()).device
        total_loss = torch.zeros((), dtype=torch.float64, device=dev)
        steps = 0
        for i, (data) in enumerate(data_loader):
            padded_mixture, mixture_lengths, padded_source = data
            if self.use_cuda:
                padded_mixture = padded_mixture.to(dev, non_blocking=True)
                mixture_lengths = mixture_lengths.to(dev, non_blocking=True)
                padded_source = padded_source.to(dev, non_blocking=True)
            if cross_valid:
                with torch.no_grad():
                    estimate_source = self.model(padded_mixture)
                    loss = cal_loss(padded_source, estimate_source, mixture_lengths)[0]
            else:
                estimate_source = self.model(padded_mixture)
                loss, max_snr, estimate_source, reorder_estimate_source = \
                    cal_loss(padded_source, estimate_source, mixture_lengths)
                self.optimizer.zero_grad()
                loss.backward()
                clip(self.model.parameters(), self.max_norm)
                self.optimizer.step()
            total_loss += loss.detach().double()
            steps = i + 1
            if i % self.print_freq == 0:
                print('Epoch {0} | Iter {1} | Average Loss {2:.3f} | '
                      'Current Loss {3:.6f} | {4:.1f} ms/batch'.format(
                          epoch + 1, i + 1, float(total_loss) / (i + 1),
                          loss.item(), 1000 * (time.time() - start) / (i + 1)), flush=True)
        stats = torch.tensor([float(total_loss), float(steps)], dtype=torch.float64)
        if self.world > 1:
            red = stats.to(dev) if dist.get_backend() == "nccl" else stats
            dist.all_reduce(red)
            stats = red.cpu()
        return float(stats[0] / stats[1]) if stats[1] > 0 else float("nan")
