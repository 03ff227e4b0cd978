"""utils/tal.py counterpart: ComputeLoss_TAL (TaskAlignedAssigner + CIoU + DFL + BCE) on gfx950.

ComputeLoss_TAL(model)(p, targets) -> (loss[1], items[3] = box, cls, dfl) as utils/tal.py:119-158,
p = TDetect training output (x, box [B, 64, A], cls [B, nc, A]).  One autograd Function runs the
assigner and the losses in csrc/tal.hip with no host synchronisation and keeps dL/dlogits from the
forward; backward scales it by the upstream gradient.  alpha / beta from $YA / $YB like the reference
(tal.py:92-93).
"""
import os

import torch

from ..functional import call, ptr, stream, dcode
from ..models.tdetect import level_arrays
from .torch_utils import de_parallel


class _TALLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cl, hw, targets, box, cls):
        dev = box.device
        B, _, A = box.shape
        t = targets.detach().to(device=dev, dtype=torch.float32).contiguous()
        nt = t.shape[0]
        cap = max(nt, 1)
        ws = torch.empty(call('dmy_tal_workspace_bytes', B, A, cap), dtype=torch.uint8, device=dev)
        no = 4 * 16 + cl.nc
        G = torch.empty((B, A, no), dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        items = torch.empty(3, dtype=torch.float32, device=dev)
        nl, H, W, S, keep = level_arrays(hw, cl.strides)
        sb, sc = box.stride(), cls.stride()
        call('dmy_tal_loss', dcode(box), ptr(box), sb[0], sb[1], sb[2], ptr(cls), sc[0], sc[1], sc[2], B, cl.nc, nl,
             H, W, S, ptr(t), nt, float(cl.alpha), float(cl.beta), float(cl.hyp['cls_pw']), ptr(ws), ptr(G),
             ptr(loss), ptr(items), stream())
        ctx.G, ctx.dtype = G, box.dtype
        ctx.mark_non_differentiable(items)
        return loss, items

    @staticmethod
    def backward(ctx, dloss, ditems):
        G = ctx.G
        g = torch.empty_like(G, dtype=ctx.dtype)
        call('dmy_loss_grad', 1 if ctx.dtype == torch.bfloat16 else 0, ptr(G), ptr(dloss.float().contiguous()), ptr(g),
             G.numel(), stream())
        ctx.G = None
        return None, None, None, g[..., :64].permute(0, 2, 1), g[..., 64:].permute(0, 2, 1)


class ComputeLoss_TAL:
    """utils/tal.py:81-158 (use_dfl=True)."""

    def __init__(self, model, use_dfl=True):
        assert use_dfl, 'the reference trains with DFL'
        m = de_parallel(model).model[-1]
        self.hyp = model.hyp if hasattr(model, 'hyp') else de_parallel(model).hyp
        self.stride, self.nc, self.nl = m.stride, m.nc, m.nl
        self.strides = getattr(m, 'stride_list', None) or [float(s) for s in m.stride.cpu()]
        self.alpha = float(os.getenv('YA', 0.5))
        self.beta = float(os.getenv('YB', 6.0))

    def __call__(self, p, targets, img=None, epoch=0):
        feats, pred_distri, pred_scores = p
        hw = [f.shape[2:] for f in feats]
        return _TALLossFn.apply(self, hw, targets, pred_distri, pred_scores)
