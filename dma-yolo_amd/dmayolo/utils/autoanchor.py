"""utils/autoanchor.py counterparts: check_anchor_order (models/yolo.py uses it at build), check_anchors and
kmean_anchors (utils/autoanchor.py:26-162), which train.py:318 runs at train start unless --noautoanchor.

Host-side numpy / scipy / torch-CPU code (once per run, not on the GPU hot path).  The dataset argument of the
reference is replaced by what the functions read from it: `shapes` [n_img, 2] (w, h) and `labels`, a list of
[n_i, 5] (cls, x, y, w, h normalised) arrays (utils/datasets.py:376-656's LoadImagesAndLabels.shapes / .labels).
Config 5 (`anchors: 4` in models/yolov5l-xs-tr-cbam-spp-bifpn.yaml:7) builds with the placeholder anchors
range(8) per level -- grid-unit widths 0..1.75, one of them zero -- and relies on exactly this recomputation.
"""
import random

import numpy as np
import torch


def _ratio_metric(k, wh):
    """utils/autoanchor.py:35-37 / 86-90: per (label, anchor) min(r, 1/r) over w and h, and its best anchor"""
    r = wh[:, None] / k[None]
    x = torch.min(r, 1 / r).min(2)[0]
    return x, x.max(1)[0]


def label_wh(shapes, labels, img_size, scale=None):
    """[sum n_i, 2] label widths / heights in pixels at img_size (autoanchor.py:31-33, 114-115)"""
    shapes = img_size * np.asarray(shapes, dtype=np.float64) / np.asarray(shapes, dtype=np.float64).max(1, keepdims=True)
    if scale is not None:
        shapes = shapes * scale
    return np.concatenate([np.asarray(l)[:, 3:5] * s for s, l in zip(shapes, labels)])


def kmean_anchors(shapes, labels, n=9, img_size=640, thr=4.0, gen=1000, verbose=False):
    """utils/autoanchor.py:64-162: whitened scipy kmeans on the label wh (> 2 px), then `gen` generations of
    multiplicative mutation keeping the best anchor_fitness.  Draws from numpy's global RNG (kmeans init and the
    mutations) and Python's `random`, as the reference does; seed both for a reproducible result."""
    from scipy.cluster.vq import kmeans
    thr = 1 / thr
    wh0 = label_wh(shapes, labels, img_size)
    wh = wh0[(wh0 >= 2.0).any(1)]  # filter > 2 pixels
    s = wh.std(0)  # sigmas for whitening
    k, _ = kmeans(wh / s, n, iter=30)
    assert len(k) == n, f'kmeans requested {n} points but returned only {len(k)}'
    k *= s
    wht = torch.tensor(wh, dtype=torch.float32)

    def anchor_fitness(kk):
        _, best = _ratio_metric(torch.tensor(kk, dtype=torch.float32), wht)
        return (best * (best > thr).float()).mean()

    k = k[np.argsort(k.prod(1))]
    npr = np.random
    f, sh, mp, s = anchor_fitness(k), k.shape, 0.9, 0.1  # fitness, generations, mutation prob, sigma
    for _ in range(gen):
        v = np.ones(sh)
        while (v == 1).all():  # mutate until a change occurs (prevent duplicates)
            v = ((npr.random(sh) < mp) * random.random() * npr.randn(*sh) * s + 1).clip(0.3, 3.0)
        kg = (k.copy() * v).clip(min=2.0)
        fg = anchor_fitness(kg)
        if fg > f:
            f, k = fg, kg.copy()
    k = k[np.argsort(k.prod(1))]  # print_results sorts small to large (autoanchor.py:97, 162)
    if verbose:
        x, best = _ratio_metric(torch.tensor(k, dtype=torch.float32), torch.tensor(wh0, dtype=torch.float32))
        print(f'autoanchor: thr={thr:.2f}: {float((best > thr).float().mean()):.4f} best possible recall, '
              f'{float((x > thr).float().mean()) * n:.2f} anchors past thr')
    return k


def check_anchors(shapes, labels, model, thr=4.0, imgsz=640, gen=1000):
    """utils/autoanchor.py:26-60: best possible recall of the model's anchors on the (0.9-1.1 randomly scaled)
    labels; below 0.98 run kmean_anchors and keep the result if its recall is higher (anchors stored / stride in
    Detect.anchors, then check_anchor_order).  Returns (bpr_before, bpr_after)."""
    from ..models.yolo import check_anchor_order
    m = model.module.model[-1] if hasattr(model, 'module') else model.model[-1]
    scale = np.random.uniform(0.9, 1.1, size=(np.asarray(shapes).shape[0], 1))  # augment scale
    wh = torch.tensor(label_wh(shapes, labels, imgsz, scale)).float()

    def metric(k):
        r = wh[:, None] / k[None]
        x = torch.min(r, 1 / r).min(2)[0]
        best = x.max(1)[0]
        return (best > 1 / thr).float().mean(), (x > 1 / thr).float().sum(1).mean()

    stride = m.stride.to(m.anchors.device).view(-1, 1, 1)
    anchors = m.anchors.clone() * stride
    bpr, _ = metric(anchors.cpu().view(-1, 2))
    new_bpr = bpr
    if bpr < 0.98:
        na = m.anchors.numel() // 2
        k = kmean_anchors(shapes, labels, n=na, img_size=imgsz, thr=thr, gen=gen)
        new_bpr = metric(torch.tensor(k, dtype=torch.float32))[0]
        if new_bpr > bpr:
            a = torch.tensor(k, device=m.anchors.device).type_as(m.anchors)
            with torch.no_grad():
                m.anchors[:] = a.clone().view_as(m.anchors) / stride
            check_anchor_order(m)
    return float(bpr), float(new_bpr)
