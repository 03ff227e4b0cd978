"""utils/torch_utils.py counterparts used on the hot path (initialize_weights, fuse_conv_and_bn,
ModelEMA, DDP helpers)."""
import math
from copy import deepcopy

import torch
import torch.nn as nn


def is_parallel(model):
    """utils/torch_utils.py:146-148 (+ the arena reducer, dmayolo.ddp.ArenaDDP)."""
    return type(model) in (nn.parallel.DataParallel, nn.parallel.DistributedDataParallel) or \
        type(model).__name__ == 'ArenaDDP'



def de_parallel(model):
    return model.module if is_parallel(model) else model


def initialize_weights(model):
    """utils/torch_utils.py:161-170: BN eps 1e-3, momentum 0.03 on exact-type BatchNorm2d."""
    for m in model.modules():
        t = type(m)
        if t is nn.BatchNorm2d:
            m.eps = 1e-3
            m.momentum = 0.03
        elif t in (nn.Hardswish, nn.LeakyReLU, nn.ReLU, nn.ReLU6, nn.SiLU):
            m.inplace = True


@torch.no_grad()
def fuse_conv_and_bn(conv, bn):
    """utils/torch_utils.py:198-218 (BN folded into the conv weight + bias)."""
    fused = nn.Conv2d(conv.in_channels, conv.out_channels, kernel_size=conv.kernel_size, stride=conv.stride,
                      padding=conv.padding, groups=conv.groups, bias=True).requires_grad_(False).to(conv.weight.device)
    w_conv = conv.weight.clone().view(conv.out_channels, -1)
    w_bn = torch.diag(bn.weight.div(torch.sqrt(bn.eps + bn.running_var)))
    fused.weight.copy_(torch.mm(w_bn, w_conv).view(fused.weight.shape))
    b_conv = torch.zeros(conv.weight.size(0), device=conv.weight.device) if conv.bias is None else conv.bias
    b_bn = bn.bias - bn.weight.mul(bn.running_mean).div(torch.sqrt(bn.running_var + bn.eps))
    fused.bias.copy_(torch.mm(w_bn, b_conv.reshape(-1, 1)).reshape(-1) + b_bn)
    return fused


class ModelEMA:
    """utils/torch_utils.py:309-343: EMA over the whole state_dict (params and float buffers).
    The update is one fused HIP kernel over a flat list of tensors (dmayolo.optim.ema_update)."""

    def __init__(self, model, decay=0.9999, updates=0):
        self.ema = deepcopy(de_parallel(model)).eval()
        self.updates = updates
        self.decay = lambda x: decay * (1 - math.exp(-x / 2000))
        for p in self.ema.parameters():
            p.requires_grad_(False)

    def update(self, model):
        from ..optim import ema_update
        with torch.no_grad():
            self.updates += 1
            d = self.decay(self.updates)
            m = de_parallel(model)
            if getattr(self, '_pairs_of', None) is not m:  # state_dict walks cost ~2 ms of host time per step
                msd = m.state_dict()
                pairs = [(v, msd[k].detach()) for k, v in self.ema.state_dict().items() if v.dtype.is_floating_point]
                self._pairs = ([a for a, _ in pairs], [b for _, b in pairs])
                self._pairs_of = m
            ema_update(self._pairs[0], self._pairs[1], d)
            from ..functional import PARAM_GEN
            PARAM_GEN[0] += 1  # EMA weights written in place by the kernel

    def update_attr(self, model, include=(), exclude=('process_group', 'reducer')):
        for k, v in model.__dict__.items():
            if (len(include) and k not in include) or k.startswith('_') or k in exclude:
                continue
            setattr(self.ema, k, v)
