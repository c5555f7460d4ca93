"""Drop-in for ``src/solver.py``: the epoch loop with
checkpoint / resume packages, learning-rate halving and early stopping.

Structure: ``PlateauSchedule`` owns the validation-plateau rules, ``Solver``
runs epochs as train pass -> optional checkpoint -> validation pass -> schedule
-> bookkeeping -> best-model package.  The decisions reproduce the reference's
(solver.py:69-156; pinned by scripted reference runs in tests/test_pipeline.py):

* ``epoch<n>.pth.tar`` is written after the training pass when ``checkpoint``
  is set, BEFORE that epoch's losses are recorded in the package;
* with ``half_lr``, a validation loss that does not beat the previous epoch's
  counts toward a plateau; from the third such epoch in a row the LR of
  ``param_groups[0]`` is halved (through the optimizer's state_dict), and with
  ``early_stop`` the tenth ends training before anything else of that epoch;
* ``model_path`` is rewritten whenever the validation loss is the best so far.

Packages are ``ConvTasNet.serialize`` dicts, so reference checkpoints resume
here and the other way round.  The step is solver.py:172-188; with fp32
parameters on a ROCm device the clip is ``ctn_optim.clip_grad_norm_``.

Deliberate differences:
* one process per GPU (DDP): each rank runs its share of minibatches
  (data.MinibatchSampler); the epoch loss is averaged over all ranks before any
  decision so every rank halves and stops together; only rank 0 writes files;
* the per-step ``loss.item()`` (a device sync per step) becomes a device-side
  fp64 running sum read at print time and at the end of the pass;
* validation runs under ``torch.no_grad()``;
* without visdom the loss plots are skipped with a message.
"""
import os
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

from pit_criterion import cal_loss

RULE = "-" * 85


@dataclass
class PlateauSchedule:
    """Validation-plateau bookkeeping of solver.py:104-123."""
    half_lr: bool
    early_stop: bool
    previous: float = float("inf")
    stalled: int = 0          # consecutive epochs without improving on the previous one
    pending_halve: bool = False

    def observe(self, val_loss: float) -> bool:
        """Record one validation loss; True means stop training now."""
        if not self.half_lr:
            return False
        if val_loss >= self.previous:   # (a NaN loss resets the count, as in the reference)
            self.stalled += 1
            self.pending_halve = self.pending_halve or self.stalled >= 3
            return self.early_stop and self.stalled >= 10
        self.stalled = 0
        return False

    def take_halve(self) -> bool:
        h, self.pending_halve = self.pending_halve, False
        return h


def _distributed():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _inner(model):
    """The ConvTasNet behind a DataParallel / DDP wrapper (or the model itself)."""
    return getattr(model, "module", model)


def _grad_clipper(model):
    p = next(iter(model.parameters()), None)
    if p is not None and p.device.type == "cuda" and p.dtype == torch.float32:
        import ctn_optim
        return ctn_optim.clip_grad_norm_
    return torch.nn.utils.clip_grad_norm_


class Solver(object):
    """Solver(data, model, optimizer, args).train() as in src/solver.py."""

    def __init__(self, data, model, optimizer, args):
        self.tr_loader, self.cv_loader = data['tr_loader'], data['cv_loader']
        self.model, self.optimizer = model, optimizer
        self.use_cuda = args.use_cuda
        self.epochs = args.epochs
        self.max_norm = args.max_norm
        self.save_folder, self.model_path = args.save_folder, args.model_path
        self.checkpoint, self.continue_from = args.checkpoint, args.continue_from
        self.print_freq = args.print_freq
        self.schedule = PlateauSchedule(bool(args.half_lr), bool(args.early_stop))
        self.tr_loss = torch.zeros(self.epochs)
        self.cv_loss = torch.zeros(self.epochs)
        self.rank, self.world = _distributed()
        self.visdom, self.visdom_epoch, self.visdom_id = args.visdom, args.visdom_epoch, args.visdom_id
        self.vis = self._open_visdom() if (self.visdom or self.visdom_epoch) else None
        self.vis_window = None
        self.best_val_loss = float("inf")
        self.start_epoch = self._resume() if self.continue_from else 0
        os.makedirs(self.save_folder, exist_ok=True)

    # -- setup ---------------------------------------------------------------
    def _open_visdom(self):
        try:
            from visdom import Visdom
        except ImportError:
            print("visdom is not installed: loss plots are skipped")
            return None
        return Visdom(env=self.visdom_id)

    def _resume(self) -> int:
        """solver.py:52-59: weights, optimizer state, epoch and the loss history."""
        print('Loading checkpoint model %s' % self.continue_from)
        pkg = torch.load(self.continue_from, map_location='cpu', weights_only=True)
        _inner(self.model).load_state_dict(pkg['state_dict'])
        self.optimizer.load_state_dict(pkg['optim_dict'])
        done = int(pkg.get('epoch', 1))
        self.tr_loss[:done] = pkg['tr_loss'][:done]
        self.cv_loss[:done] = pkg['cv_loss'][:done]
        return done

    # -- files ---------------------------------------------------------------
    def _write_package(self, name: str, epoch_done: int) -> str:
        path = os.path.join(self.save_folder, name)
        if self.rank == 0:
            m = _inner(self.model)
            torch.save(m.serialize(m, self.optimizer, epoch_done, tr_loss=self.tr_loss, cv_loss=self.cv_loss),
                       path)
        return path

    def _halve_lr(self):
        state = self.optimizer.state_dict()
        lr = state['param_groups'][0]['lr'] / 2.0
        state['param_groups'][0]['lr'] = lr
        self.optimizer.load_state_dict(state)
        print('Learning rate adjusted to: {lr:.6f}'.format(lr=lr))

    def _plot(self, epoch):
        if self.vis is None or not self.visdom or self.rank != 0:
            return
        xs = torch.arange(1, epoch + 2)
        ys = torch.stack((self.tr_loss[:epoch + 1], self.cv_loss[:epoch + 1]), dim=1)
        if self.vis_window is None:
            self.vis_window = self.vis.line(X=xs, Y=ys, opts=dict(title=self.visdom_id, ylabel='Loss',
                                                                  xlabel='Epoch',
                                                                  legend=['train loss', 'cv loss']))
        else:
            self.vis.line(X=xs.unsqueeze(0).expand(ys.size(1), xs.size(0)).t(), Y=ys, win=self.vis_window,
                          update='replace')

    @staticmethod
    def _summary(kind, epoch, start, loss):
        print(RULE)
        print('{0} Summary | End of Epoch {1} | Time {2:.2f}s | {3} Loss {4:.3f}'.format(
            kind, epoch + 1, time.time() - start, 'Train' if kind == 'Train' else 'Valid', loss))
        print(RULE)

    # -- epochs --------------------------------------------------------------
    def train(self):
        for epoch in range(self.start_epoch, self.epochs):
            start = time.time()
            print("Training...")
            self.model.train()
            tr_avg = self._run_one_epoch(epoch)
            self._summary('Train', epoch, start, tr_avg)
            if self.checkpoint:
                print('Saving checkpoint model to %s' % self._write_package('epoch%d.pth.tar' % (epoch + 1),
                                                                             epoch + 1))
            print('Cross validation...')
            self.model.eval()
            val = self._run_one_epoch(epoch, cross_valid=True)
            self._summary('Valid', epoch, start, val)

            if self.schedule.observe(val):
                print("No imporvement for 10 epochs, early stopping.")
                break
            if self.schedule.take_halve():
                self._halve_lr()
            self.schedule.previous = val

            self.tr_loss[epoch], self.cv_loss[epoch] = tr_avg, val
            if val < self.best_val_loss:
                self.best_val_loss = val
                print("Find better validated model, saving to %s" % self._write_package(self.model_path, epoch + 1))
            self._plot(epoch)

    def _batch_to_device(self, batch, dev):
        if not self.use_cuda:
            return batch
        return tuple(t.to(dev, non_blocking=True) for t in batch)

    def _run_one_epoch(self, epoch, cross_valid=False):
        """One pass over the train (or cv) loader -> mean loss over all ranks (solver.py:158-210)."""
        loader = self.cv_loader if cross_valid else self.tr_loader
        if hasattr(getattr(loader, "sampler", None), "set_epoch"):
            loader.sampler.set_epoch(epoch)
        clip = _grad_clipper(self.model)
        params = list(self.model.parameters())   # walked once per epoch, not per step
        dev = params[0].device
        running = torch.zeros((), dtype=torch.float64, device=dev)
        n, start = 0, time.time()
        for i, batch in enumerate(loader):
            mixture, lengths, source = self._batch_to_device(batch, dev)
            if cross_valid:
                # the unwrapped module: a DDP forward would broadcast buffers (BN running
                # stats), a collective that ranks without a cv minibatch never join
                with torch.no_grad():
                    loss = cal_loss(source, _inner(self.model)(mixture), lengths)[0]
            else:
                loss = cal_loss(source, self.model(mixture), lengths)[0]
                self.optimizer.zero_grad()
                loss.backward()
                if getattr(self.model, "grad_sync", None) is not None:   # train.FlatDP
                    self.model.grad_sync.sync()
                clip(params, self.max_norm)
                self.optimizer.step()
            running += loss.detach().double()
            n = i + 1
            if i % self.print_freq == 0:
                print('Epoch {0} | Iter {1} | Average Loss {2:.3f} | Current Loss {3:.6f} | {4:.1f} ms/batch'
                      .format(epoch + 1, n, float(running) / n, loss.item(), 1000 * (time.time() - start) / n),
                      flush=True)
        totals = torch.tensor([float(running), float(n)], dtype=torch.float64)
        if self.world > 1:
            buf = totals.to(dev) if dist.get_backend() == "nccl" else totals
            dist.all_reduce(buf)
            totals = buf.cpu()
        return float(totals[0] / totals[1]) if totals[1] > 0 else float("nan")
