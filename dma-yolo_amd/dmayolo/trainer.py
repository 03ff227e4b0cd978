"""The reference's batch loop (train.py:183-235, 343-463, 466-468) around the gfx950 model, loss and optimizer.

Trainer.step(imgs, targets) is one iteration of `for i, (imgs, targets, ...) in pbar` on a device batch:
  * warmup (ni <= nw, nw = max(round(warmup_epochs * nb), 1000)): accumulate and per-group lr / momentum
    interpolated exactly as train.py:408-422 (bias group from warmup_bias_lr, others from 0, to
    initial_lr * lf(epoch); momentum from warmup_momentum);
  * forward + ComputeLoss (or ComputeLoss_TAL) + backward seeded with GradScaler.upstream = loss scale * WORLD_SIZE
    (train.py:437-445: `loss *= WORLD_SIZE`, `scaler.scale(loss).backward()`), DDP all-reduce when `net` is
    DistributedDataParallel;
  * every `accumulate` iterations (ni - last_opt_step >= accumulate): scaler.step / update, zero_grad, EMA
    (train.py:448-454).
epoch_end() steps the LambdaLR scheduler (train.py:466-468).  Optimizer groups, weight-decay scaling
(hyp['weight_decay'] *= batch_size * accumulate / nbs, train.py:189-192), LambdaLR(one_cycle(1, lrf, epochs)) or
the linear lf (train.py:231-235) are built in __init__.  Host state only (ni, accumulate, lr values): no device
synchronisation anywhere in step().
"""
import math

import numpy as np
import torch

from .optim import build_optimizer, GradScaler
from .utils.torch_utils import ModelEMA, de_parallel


def one_cycle(y1=0.0, y2=1.0, steps=100):
    """utils/general.py:460-462: sinusoidal ramp from y1 to y2 over `steps`."""
    return lambda x: ((1 - math.cos(x * math.pi / steps)) / 2) * (y2 - y1) + y1


class Trainer:
    def __init__(self, model, hyp, batch_size, epochs=300, nb=100, adam=False, linear_lr=False, world_size=1,
                 rank=-1, net=None, compute_loss=None, ema=True, amp=True, nbs=64, start_epoch=0):
        """batch_size: the total batch size (train.py's opt.batch_size; each of `world_size` ranks holds
        batch_size // world_size images).  nb: batches per epoch.  hyp: the scaled hyp dict (model.hyp);
        its weight_decay is scaled here as train.py:189-192 does."""
        self.model = de_parallel(model)
        self.net = net if net is not None else model
        self.hyp = hyp
        self.nbs, self.batch_size, self.epochs, self.nb = nbs, batch_size, epochs, nb
        self.accumulate = max(round(nbs / batch_size), 1)
        hyp['weight_decay'] *= batch_size * self.accumulate / nbs
        self.optimizer = build_optimizer(self.model, 'adam' if adam else 'sgd', hyp['lr0'], hyp['momentum'],
                                         hyp['weight_decay'])
        if linear_lr:
            self.lf = lambda x: (1 - x / (epochs - 1)) * (1.0 - hyp['lrf']) + hyp['lrf']
        else:
            self.lf = one_cycle(1, hyp['lrf'], epochs)
        self.scheduler = torch.optim.lr_scheduler.LambdaLR(self.optimizer, lr_lambda=self.lf)
        self.scheduler.last_epoch = start_epoch - 1  # train.py:352
        self.epoch = start_epoch
        self.ema = ModelEMA(self.model) if (ema and rank in (-1, 0)) else None
        self.world = world_size if rank != -1 else 1
        dev = next(self.model.parameters()).device
        self.scaler = GradScaler(dev, enabled=amp and dev.type == 'cuda', world=self.world)
        if compute_loss is None:
            from .utils.loss import ComputeLoss
            compute_loss = ComputeLoss(self.model)
        self.compute_loss = compute_loss
        self.nw = max(round(hyp['warmup_epochs'] * nb), 1000)  # train.py:345
        self.last_opt_step = -1
        self.i = 0  # batch index within the epoch
        self.optimizer.zero_grad(set_to_none=True)

    @property
    def ni(self):
        return self.i + self.nb * self.epoch

    def warmup(self, ni):
        """train.py:408-422 for integrated batch ni (host-side writes into the param groups)."""
        if ni <= self.nw:
            xi = [0, self.nw]
            self.accumulate = max(1, np.interp(ni, xi, [1, self.nbs / self.batch_size]).round())
            h = self.hyp
            for j, x in enumerate(self.optimizer.param_groups):
                x['lr'] = np.interp(ni, xi, [h['warmup_bias_lr'] if j == 2 else 0.0, x['initial_lr'] * self.lf(self.epoch)])
                if 'momentum' in x:  # SGD only: Adam groups carry betas, untouched (as the reference)
                    x['momentum'] = np.interp(ni, xi, [h['warmup_momentum'], h['momentum']])

    def step(self, imgs, targets):
        """One batch iteration; returns (loss [1] before the WORLD_SIZE / loss-scale factors, items [3])."""
        ni = self.ni
        self.warmup(ni)
        pred = self.net(imgs)
        loss, items = self.compute_loss(pred, targets)
        loss.backward(self.scaler.upstream)
        if ni - self.last_opt_step >= self.accumulate:
            self.scaler.step(self.optimizer)
            self.scaler.update()
            self.optimizer.zero_grad(set_to_none=True)
            if self.ema is not None:
                self.ema.update(self.model)
            self.last_opt_step = ni
        self.i += 1
        return loss, items

    def epoch_end(self):
        """train.py:466-468: scheduler.step() (lr for the next epoch), batch counter reset."""
        self.scheduler.step()
        self.epoch += 1
        self.i = 0
