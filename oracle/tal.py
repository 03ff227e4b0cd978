"""CPU fp32 restatement of the anchor-free TAL path (TEST INFRASTRUCTURE ONLY).

Follows models/detect_t.py:23-101 (TDetect head, DFL, make_anchors, dist2bbox),
utils/tal.py:81-221 (ComputeLoss_TAL, BboxLoss, bbox2dist, CIoU) and
utils/tal_assign.py:54-189 (TaskAlignedAssigner).  Pinned by tests/golden/tal_*.npz, generated
from the reference in this container by tools/gen_golden.py.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

REG_MAX = 16


def anchor_grid(shapes, strides, offset=0.5):
    """make_anchors (detect_t.py:62-74): per level, cell centres in grid units, row-major (y, x)."""
    pts, st = [], []
    for (h, w), s in zip(shapes, strides):
        ys, xs = torch.meshgrid(torch.arange(h, dtype=torch.float32) + offset,
                                torch.arange(w, dtype=torch.float32) + offset, indexing='ij')
        pts.append(torch.stack((xs.reshape(-1), ys.reshape(-1)), 1))
        st.append(torch.full((h * w, 1), float(s)))
    return torch.cat(pts), torch.cat(st)


def ltrb_to_xyxy(d, pts):
    """dist2bbox(xywh=False) (tal.py:206-215): d [..., 4] (l, t, r, b) around pts [..., 2]."""
    return torch.cat((pts - d[..., :2], pts + d[..., 2:]), -1)


def xyxy_to_ltrb(pts, box, reg_max):
    """bbox2dist (tal.py:218-221): clamp to [0, reg_max - 0.01]."""
    return torch.cat((pts - box[..., :2], box[..., 2:] - pts), -1).clamp(0, reg_max - 0.01)


def dfl_expectation(logits):
    """bbox_decode (tal.py:113-117): softmax over REG_MAX bins per side, expectation with 0..15."""
    p = logits.view(*logits.shape[:-1], 4, REG_MAX).softmax(-1)
    return (p * torch.arange(REG_MAX, dtype=logits.dtype)).sum(-1)


def ciou_xyxy(b1, b2, eps=1e-7):
    """bbox_iou(xywh=False, CIoU=True) (tal.py:24-62 == tal_assign.py:6-40); alpha is a constant
    (computed under no_grad in the reference).  Broadcasts over leading dims; returns [...]."""
    ax1, ay1, ax2, ay2 = b1.unbind(-1)
    bx1, by1, bx2, by2 = b2.unbind(-1)
    w1, h1 = ax2 - ax1, ay2 - ay1 + eps
    w2, h2 = bx2 - bx1, by2 - by1 + eps
    inter = (torch.minimum(ax2, bx2) - torch.maximum(ax1, bx1)).clamp(0) * \
            (torch.minimum(ay2, by2) - torch.maximum(ay1, by1)).clamp(0)
    union = w1 * h1 + w2 * h2 - inter + eps
    iou = inter / union
    cw = torch.maximum(ax2, bx2) - torch.minimum(ax1, bx1)
    ch = torch.maximum(ay2, by2) - torch.minimum(ay1, by1)
    c2 = cw ** 2 + ch ** 2 + eps
    rho2 = ((bx1 + bx2 - ax1 - ax2) ** 2 + (by1 + by2 - ay1 - ay2) ** 2) / 4
    v = (4 / math.pi ** 2) * (torch.atan(w2 / h2) - torch.atan(w1 / h1)) ** 2
    with torch.no_grad():
        alpha = v / (v - iou + (1 + eps))
    return iou - (rho2 / c2 + v * alpha)


def pad_targets(targets, bs, scale):
    """ComputeLoss_TAL.preprocess (tal.py:96-111): [nt, 6] (img, cls, xywh normalised) ->
    [bs, nmax, 5] (cls, xyxy pixels), zero rows as padding."""
    if targets.shape[0] == 0:
        return torch.zeros(bs, 0, 5)
    img = targets[:, 0].long()
    nmax = int(torch.bincount(img, minlength=bs).max())
    out = torch.zeros(bs, nmax, 5)
    for b in range(bs):
        rows = targets[img == b, 1:]
        out[b, :rows.shape[0]] = rows
    xywh = out[..., 1:5] * scale
    out[..., 1:5] = torch.cat((xywh[..., :2] - xywh[..., 2:] / 2, xywh[..., :2] + xywh[..., 2:] / 2), -1)
    return out


@torch.no_grad()
def tal_assign(scores, pboxes, pts, labels, gboxes, gmask, topk=10, nc=80, alpha=0.5, beta=6.0, eps=1e-9):
    """TaskAlignedAssigner.forward (tal_assign.py:83-189).
    scores [B, A, nc] (sigmoid), pboxes [B, A, 4] xyxy px, pts [A, 2] px, labels [B, n, 1], gboxes [B, n, 4],
    gmask [B, n, 1] -> (target_labels [B, A], target_boxes [B, A, 4], target_scores [B, A, nc], fg [B, A])."""
    B, A = scores.shape[:2]
    n = gboxes.shape[1]
    if n == 0:
        return (torch.full((B, A), nc), torch.zeros(B, A, 4), torch.zeros(B, A, nc), torch.zeros(B, A, dtype=torch.bool))
    lab = labels.long().squeeze(-1)                                              # [B, n]
    cls_score = torch.gather(scores.transpose(1, 2), 1, lab[:, :, None].expand(B, n, A))  # [B, n, A]
    ov = ciou_xyxy(gboxes[:, :, None, :], pboxes[:, None, :, :]).clamp(0)       # [B, n, A]
    metric = cls_score.pow(alpha) * ov.pow(beta)
    # anchor centre strictly inside the gt box (select_candidates_in_gts)
    d = torch.cat((pts[None, None] - gboxes[:, :, None, :2], gboxes[:, :, None, 2:] - pts[None, None]), -1)
    inside = (d.amin(-1) > eps).float()
    # top-k per gt over the in-box metric; k-th picks of padded gts point at anchor 0; duplicates dropped
    _, idx = torch.topk(metric * inside, topk, dim=-1)
    idx = torch.where(gmask.bool().expand(B, n, topk), idx, torch.zeros_like(idx))
    cnt = torch.zeros(B, n, A).scatter_add_(2, idx, torch.ones_like(idx, dtype=torch.float32))
    sel = torch.where(cnt > 1, torch.zeros_like(cnt), cnt)
    pos = sel * inside * gmask                                                   # mask_pos [B, n, A]
    # one gt per anchor: anchors claimed by several gts go to the gt of largest overlap
    fgc = pos.sum(1)                                                             # [B, A]
    if float(fgc.max()) > 1:
        best = F.one_hot(ov.argmax(1), n).permute(0, 2, 1).float()
        pos = torch.where((fgc > 1)[:, None, :].expand(B, n, A), best, pos)
        fgc = pos.sum(1)
    gi = pos.argmax(1)                                                           # [B, A]
    t_lab = torch.gather(lab, 1, gi)
    t_box = torch.gather(gboxes, 1, gi[..., None].expand(B, A, 4))
    t_sc = F.one_hot(t_lab, nc) * (fgc > 0)[..., None]
    m = metric * pos
    norm = (m * (ov * pos).amax(-1, keepdim=True) / (m.amax(-1, keepdim=True) + eps)).amax(1)  # [B, A]
    return t_lab, t_box, t_sc * norm[..., None], fgc > 0


def compute_loss_tal(feats, pred_distri, pred_scores, targets, strides, hyp, nc, alpha=0.5, beta=6.0):
    """ComputeLoss_TAL.__call__ (tal.py:119-158).  feats: list of [B, no, H, W] (for shapes);
    pred_distri [B, 64, A], pred_scores [B, nc, A] (TDetect training outputs).  -> (loss[1], items[3])."""
    B = pred_scores.shape[0]
    ps = pred_scores.permute(0, 2, 1)
    pd = pred_distri.permute(0, 2, 1)
    shapes = [f.shape[2:] for f in feats]
    pts, st = anchor_grid(shapes, strides)
    img = torch.tensor(feats[0].shape[2:], dtype=torch.float32) * float(strides[0])     # (h, w) px
    tg = pad_targets(targets, B, img[[1, 0, 1, 0]])
    glab, gbox = tg[..., :1], tg[..., 1:]
    gmask = (gbox.sum(-1, keepdim=True) > 0).float()
    pbox = ltrb_to_xyxy(dfl_expectation(pd), pts)                               # grid units
    _, t_box, t_sc, fg = tal_assign(ps.detach().sigmoid(), (pbox.detach() * st), pts * st, glab, gbox, gmask,
                                    nc=nc, alpha=alpha, beta=beta)
    t_box = t_box / st
    tss = t_sc.sum()
    pw = torch.tensor([hyp['cls_pw']])
    lcls = F.binary_cross_entropy_with_logits(ps, t_sc, pos_weight=pw, reduction='none').sum() / tss
    lbox = torch.zeros(())
    ldfl = torch.zeros(())
    if fg.sum():
        w = t_sc.sum(-1)[fg][:, None]
        lbox = ((1.0 - ciou_xyxy(pbox[fg], t_box[fg])[:, None]) * w).sum() / tss
        tl = xyxy_to_ltrb(pts, t_box, REG_MAX - 1)[fg]                           # [F, 4]
        logit = pd[fg].reshape(-1, REG_MAX)
        lo = tl.long()
        wl = (lo + 1) - tl
        ce_l = F.cross_entropy(logit, lo.reshape(-1), reduction='none').view(lo.shape)
        ce_r = F.cross_entropy(logit, (lo + 1).reshape(-1), reduction='none').view(lo.shape)
        ldfl = ((ce_l * wl + ce_r * (1 - wl)).mean(-1, keepdim=True) * w).sum() / tss
    items = torch.stack((lbox * 7.5, lcls * 0.5, ldfl * 1.5))
    return items.sum() * B, items.detach()


class DFL(nn.Module):
    """models/detect_t.py:92-101: fixed 1x1 conv holding the bin values 0..c1-1 (a state_dict entry)."""

    def __init__(self, c1=REG_MAX):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        self.conv.weight.data[:] = torch.arange(c1, dtype=torch.float32).view(1, c1, 1, 1)


class TDetect(nn.Module):
    """models/detect_t.py:23-59 with oracle Conv (oracle.nn.Conv)."""

    def __init__(self, nc=80, ch=(), inplace=True):
        super().__init__()
        from .nn import Conv
        self.nc, self.reg_max, self.nl = nc, REG_MAX, len(ch)
        self.no = nc + REG_MAX * 4
        self.stride = torch.zeros(self.nl)
        c2, c3 = max(ch[0] // 4, 16), max(ch[0], self.no - 4)
        self.cv2 = nn.ModuleList(nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 4 * REG_MAX, 1))
                                 for x in ch)
        self.cv3 = nn.ModuleList(nn.Sequential(Conv(x, c3, 3), Conv(c3, c3, 3), nn.Conv2d(c3, nc, 1)) for x in ch)
        self.dfl = DFL(REG_MAX)

    def forward(self, xs):
        xs = [torch.cat((self.cv2[i](x), self.cv3[i](x)), 1) for i, x in enumerate(xs)]
        B = xs[0].shape[0]
        flat = torch.cat([x.reshape(B, self.no, -1) for x in xs], 2)
        box, cls = flat.split((REG_MAX * 4, self.nc), 1)
        if self.training:
            return xs, box, cls
        pts, st = anchor_grid([x.shape[2:] for x in xs], self.stride)
        d = dfl_expectation(box.permute(0, 2, 1))                                # [B, A, 4]
        xyxy = ltrb_to_xyxy(d, pts)
        xywh = torch.cat(((xyxy[..., :2] + xyxy[..., 2:]) / 2, xyxy[..., 2:] - xyxy[..., :2]), -1) * st
        return torch.cat((xywh.permute(0, 2, 1), cls.sigmoid()), 1), (xs, box, cls)

    def bias_init(self):
        """detect_t.py:53-59."""
        for a, b, s in zip(self.cv2, self.cv3, self.stride):
            a[-1].bias.data[:] = 1.0
            b[-1].bias.data[:self.nc] = math.log(5 / self.nc / (640 / s) ** 2)


def space_to_depth(x):
    """models/common.py:1451-1458."""
    return torch.cat([x[..., ::2, ::2], x[..., 1::2, ::2], x[..., ::2, 1::2], x[..., 1::2, 1::2]], 1)
