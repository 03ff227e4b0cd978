"""utils/loss.py counterpart: anchor-based YOLO loss with SIoU box regression on gfx950.

ComputeLoss(model)(p, targets) -> (loss[1], items[3]) exactly like utils/loss.py:135-218, with
sort_obj_iou forced on (loss.py:191-194) and the in-place gij clamp (loss.py:265-272).  One
autograd Function runs build_targets + per-target SIoU/BCE + dense objectness BCE in HIP kernels
and keeps dL/dp from the forward; backward scales it by the upstream gradient on device.
"""
import torch

from ..functional import call, ptr, stream, dcode
from .torch_utils import de_parallel


def smooth_BCE(eps=0.1):
    """utils/loss.py:13-15."""
    return 1.0 - 0.5 * eps, 0.5 * eps


def _targets_dev(targets, dev):
    return targets.detach().to(device=dev, dtype=torch.float32).contiguous()


def _build_level(targets, nt, anchors_i, na, H, W, anchor_t, dev):
    cap = max(5 * na * nt, 1)
    ii = torch.empty((6, cap), dtype=torch.int32, device=dev)   # b, a, gj, gi, tcls, count(at [5,0])
    tbox = torch.empty((cap, 4), dtype=torch.float32, device=dev)
    anch = torch.empty((cap, 2), dtype=torch.float32, device=dev)
    cnt = ii[5, :1]
    cnt.zero_()
    if nt:
        call('dmy_build_targets', ptr(targets), nt, ptr(anchors_i), na, H, W, float(anchor_t), ptr(ii[0]), ptr(ii[1]),
             ptr(ii[2]), ptr(ii[3]), ptr(ii[4]), ptr(tbox), ptr(anch), ptr(cnt), stream())
    return ii, tbox, anch, cnt, cap


class _YoloLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cl, targets, *p):
        dev = p[0].device
        t = _targets_dev(targets, dev)
        nt = t.shape[0]
        h = cl.hyp
        nl = len(p)
        PR = call('dmy_yolo_loss_part_rows')
        part = torch.zeros(nl * PR, dtype=torch.float32, device=dev)  # per-block partials, fixed-order reduction
        Gs = []
        bs = p[0].shape[0]
        for i, pi in enumerate(p):
            N, na, H, W, no = pi.shape
            assert pi.stride(4) == 1, 'channel dim must be contiguous'
            ii, tbox, anch, cnt, cap = _build_level(t, nt, cl.anchors[i], na, H, W, h['anchor_t'], dev)
            G = torch.zeros_like(pi, dtype=torch.float32)
            tobj = torch.zeros(N * na * H * W, dtype=torch.float32, device=dev)
            tgrad = torch.empty((cap, 4 + (cl.nc if cl.nc > 1 else 0)), dtype=torch.float32, device=dev)
            links = torch.empty(N * na * H * W + cap, dtype=torch.int32, device=dev)
            s = pi.stride()
            call('dmy_yolo_loss_level', dcode(pi), ptr(pi), s[0], s[1], s[2], s[3], N, na, H, W, no, cl.nc,
                 float(h['box']), float(h['obj']), float(h['cls']), float(h['cls_pw']), float(h['obj_pw']),
                 float(cl.cp), float(cl.cn), float(cl.balance[i]), float(bs), ptr(ii[0]), ptr(ii[1]), ptr(ii[2]),
                 ptr(ii[3]), ptr(ii[4]), ptr(tbox), ptr(anch), ptr(cnt), cap, ptr(G), ptr(tobj), ptr(part[PR * i:]),
                 ptr(tgrad), ptr(links), stream())
            Gs.append(G)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        items = torch.empty(3, dtype=torch.float32, device=dev)
        call('dmy_yolo_loss_finalize', ptr(part), nl, float(h['box']), float(h['obj']), float(h['cls']), float(bs),
             ptr(loss), ptr(items), stream())
        ctx.Gs = Gs
        ctx.dtypes = [pi.dtype for pi in p]
        ctx.mark_non_differentiable(items)
        return loss, items

    @staticmethod
    def backward(ctx, dloss, ditems):
        dloss = dloss.float().contiguous()
        grads = []
        for G, dt in zip(ctx.Gs, ctx.dtypes):
            dp = torch.empty_like(G, dtype=dt)
            call('dmy_loss_grad', 1 if dt == torch.bfloat16 else 0, ptr(G), ptr(dloss), ptr(dp), G.numel(), stream())
            grads.append(dp)
        ctx.Gs = None
        return (None, None, *grads)


class ComputeLoss:
    """utils/loss.py:135-218 (SIoU, anchor-based)."""

    def __init__(self, model, autobalance=False):
        assert not autobalance, 'autobalance is off in the reference training path'
        h = model.hyp
        if h.get('fl_gamma', 0.0) > 0:
            raise NotImplementedError('focal loss (fl_gamma > 0) is outside the DMA-YOLO hot path')
        self.cp, self.cn = smooth_BCE(eps=h.get('label_smoothing', 0.0))
        det = de_parallel(model).model[-1]
        self.balance = {3: [4.0, 1.0, 0.4]}.get(det.nl, [4.0, 1.0, 0.25, 0.06, 0.02])
        self.gr, self.hyp, self.autobalance = 1.0, h, False
        for k in ('na', 'nc', 'nl'):
            setattr(self, k, getattr(det, k))
        self.anchors = det.anchors.float().contiguous()

    def __call__(self, p, targets):
        return _YoloLossFn.apply(self, targets, *p)

    def build_targets(self, p, targets):
        """utils/loss.py:220-276 on device (the host sync here is for API compatibility only)."""
        dev = p[0].device
        t = _targets_dev(targets, dev)
        tcls, tbox, indices, anch = [], [], [], []
        for i, pi in enumerate(p):
            _, na, H, W, _ = pi.shape
            ii, tb, an, cnt, cap = _build_level(t, t.shape[0], self.anchors[i], na, H, W, self.hyp['anchor_t'], dev)
            n = int(cnt.item())
            iil = ii[:, :n].long()
            indices.append((iil[0], iil[1], iil[2], iil[3]))
            tcls.append(iil[4])
            tbox.append(tb[:n])
            anch.append(an[:n])
        return tcls, tbox, indices, anch
