"""CPU fp32 restatement of utils/loss.ComputeLoss + utils/metrics.bbox_iou(SIoU) (TEST INFRASTRUCTURE ONLY)."""
import math

import torch
import torch.nn.functional as F


def siou(b1, b2, eps=1e-7):
    """SIoU of xywh boxes b1 [M,4] vs b2 [M,4] -> [M].  utils/metrics.py:192-235 (x1y1x2y2=False, SIoU=True)."""
    p1x, p2x = b1[:, 0] - b1[:, 2] / 2, b1[:, 0] + b1[:, 2] / 2
    p1y, p2y = b1[:, 1] - b1[:, 3] / 2, b1[:, 1] + b1[:, 3] / 2
    q1x, q2x = b2[:, 0] - b2[:, 2] / 2, b2[:, 0] + b2[:, 2] / 2
    q1y, q2y = b2[:, 1] - b2[:, 3] / 2, b2[:, 1] + b2[:, 3] / 2
    iw = (torch.minimum(p2x, q2x) - torch.maximum(p1x, q1x)).clamp(0)
    ih = (torch.minimum(p2y, q2y) - torch.maximum(p1y, q1y)).clamp(0)
    inter = iw * ih
    w1, h1 = p2x - p1x, p2y - p1y + eps
    w2, h2 = q2x - q1x, q2y - q1y + eps
    iou = inter / (w1 * h1 + w2 * h2 - inter + eps)
    cw = torch.maximum(p2x, q2x) - torch.minimum(p1x, q1x)
    chh = torch.maximum(p2y, q2y) - torch.minimum(p1y, q1y)
    dx = (q1x + q2x - p1x - p2x) * 0.5
    dy = (q1y + q2y - p1y - p2y) * 0.5
    sig = (dx ** 2 + dy ** 2) ** 0.5
    sa1, sa2 = dx.abs() / sig, dy.abs() / sig
    sa = torch.where(sa1 > math.sqrt(2) / 2, sa2, sa1)
    ang = torch.cos(torch.arcsin(sa) * 2 - math.pi / 2)
    gam = ang - 2
    dist = 2 - torch.exp(gam * (dx / cw) ** 2) - torch.exp(gam * (dy / chh) ** 2)
    ow = (w1 - w2).abs() / torch.maximum(w1, w2)
    oh = (h1 - h2).abs() / torch.maximum(h1, h2)
    shape = (1 - torch.exp(-ow)) ** 4 + (1 - torch.exp(-oh)) ** 4
    return iou - 0.5 * (dist + shape)


_OFF = torch.tensor([[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1]], dtype=torch.float32) * 0.5


def build_targets(shapes, targets, anchors, anchor_t):
    """utils/loss.py:220-276.  shapes: list of p[i].shape; anchors [nl,na,2] (grid units).

    Candidate order: offset-major, then anchor, then target (the reference's repeat/mask order).
    gij is clamped IN PLACE before tbox is built.
    """
    nl, na = anchors.shape[:2]
    nt = targets.shape[0]
    out = []
    for i in range(nl):
        _, _, H, W, _ = shapes[i]
        gain = torch.tensor([1, 1, W, H, W, H], dtype=torch.float32)
        res = dict(b=[], a=[], gj=[], gi=[], tbox=[], anch=[], tcls=[])
        if nt:
            t = targets * gain                                                      # [nt,6]
            rows = []
            for o in range(5):
                for a in range(na):
                    r = t[:, 4:6] / anchors[i, a]
                    ok = torch.maximum(r, 1 / r).max(1)[0] < anchor_t
                    gxy = t[:, 2:4]
                    gxi = torch.tensor([W, H], dtype=torch.float32) - gxy
                    if o == 0:
                        sel = ok
                    elif o in (1, 2):
                        v = gxy[:, o - 1]
                        sel = ok & (v % 1 < 0.5) & (v > 1)
                    else:
                        v = gxi[:, o - 3]
                        sel = ok & (v % 1 < 0.5) & (v > 1)
                    idx = torch.nonzero(sel).view(-1)
                    for j in idx.tolist():
                        rows.append((o, a, j))
            for (o, a, j) in rows:
                tt = t[j]
                gxy = tt[2:4]
                gij = (gxy - _OFF[o]).long()
                gi = int(gij[0].clamp(0, W - 1))
                gj = int(gij[1].clamp(0, H - 1))
                res['b'].append(int(tt[0]))
                res['tcls'].append(int(tt[1]))
                res['a'].append(a)
                res['gj'].append(gj)
                res['gi'].append(gi)
                res['tbox'].append(torch.stack([gxy[0] - gi, gxy[1] - gj, tt[4], tt[5]]))
                res['anch'].append(anchors[i, a])
        for k in ('b', 'a', 'gj', 'gi', 'tcls'):
            res[k] = torch.tensor(res[k], dtype=torch.int64)
        res['tbox'] = torch.stack(res['tbox']) if res['tbox'] else torch.zeros(0, 4)
        res['anch'] = torch.stack(res['anch']) if res['anch'] else torch.zeros(0, 2)
        out.append(res)
    return out


def bce_logits(x, t, pw):
    """BCEWithLogitsLoss(pos_weight=pw), mean reduction."""
    return F.binary_cross_entropy_with_logits(x, t, pos_weight=torch.tensor([pw], dtype=x.dtype))


def compute_loss(p, targets, anchors, hyp, nc):
    """utils/loss.py:167-218 with sort_obj_iou forced on: returns (loss[1], items[3])."""
    nl = len(p)
    balance = {3: [4.0, 1.0, 0.4]}.get(nl, [4.0, 1.0, 0.25, 0.06, 0.02])
    tg = build_targets([x.shape for x in p], targets, anchors, hyp['anchor_t'])
    lbox, lobj, lcls = torch.zeros(1), torch.zeros(1), torch.zeros(1)
    for i, pi in enumerate(p):
        r = tg[i]
        tobj = torch.zeros(pi.shape[:4], dtype=pi.dtype)
        n = r['b'].numel()
        if n:
            ps = pi[r['b'], r['a'], r['gj'], r['gi']]
            pxy = ps[:, :2].sigmoid() * 2 - 0.5
            pwh = (ps[:, 2:4].sigmoid() * 2) ** 2 * r['anch']
            iou = siou(torch.cat([pxy, pwh], 1), r['tbox'])
            lbox = lbox + (1.0 - iou).mean()
            s = iou.detach().clamp(0)
            # sorted ascending + last-write-wins => each cell keeps its max IoU
            flat = ((r['b'] * pi.shape[1] + r['a']) * pi.shape[2] + r['gj']) * pi.shape[3] + r['gi']
            tv = tobj.view(-1)
            tv.scatter_reduce_(0, flat, s, reduce='amax', include_self=True)
            if nc > 1:
                t = torch.zeros_like(ps[:, 5:])
                t[torch.arange(n), r['tcls']] = 1.0
                lcls = lcls + bce_logits(ps[:, 5:], t, hyp['cls_pw'])
        lobj = lobj + bce_logits(pi[..., 4], tobj, hyp['obj_pw']) * balance[i]
    lbox = lbox * hyp['box']
    lobj = lobj * hyp['obj']
    lcls = lcls * hyp['cls']
    bs = p[0].shape[0]
    return (lbox + lobj + lcls) * bs, torch.cat([lbox, lobj, lcls]).detach()
