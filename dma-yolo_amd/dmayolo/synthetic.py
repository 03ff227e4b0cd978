"""Synthetic VisDrone-shaped batches: uint8 images + [nt, 6] normalised targets, and
the hyperparameters the reference trains DMA-YOLO with (data/hyps/hyp.VisDrone.yaml:1-28) scaled
as train.py:331-333 does."""
import math
import os

import torch

CONFIGS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'configs')

# data/hyps/hyp.VisDrone.yaml (loss-relevant keys)
HYP_VISDRONE = dict(lr0=0.0032, lrf=0.12, momentum=0.843, weight_decay=0.00036, warmup_epochs=2.0, warmup_momentum=0.5,
                    warmup_bias_lr=0.05, box=0.07, cls=0.18, cls_pw=0.631, obj=0.15, obj_pw=0.911, anchor_t=3.0,
                    fl_gamma=0.0, label_smoothing=0.0, hsv_h=0.4, hsv_s=0.3, hsv_v=0.5, degrees=0.2, translate=0.0,
                    scale=0.4, shear=0.0, perspective=0.0, flipud=0.0, fliplr=0.5, mosaic=1.0, mixup=0.2,
                    copy_paste=0.0)
# data/hyps/hyp.scratch.yaml
HYP_SCRATCH = dict(lr0=0.01, lrf=0.1, momentum=0.937, weight_decay=0.0005, warmup_epochs=3.0, warmup_momentum=0.8,
                   warmup_bias_lr=0.1, box=0.05, cls=0.5, cls_pw=1.0, obj=1.0, obj_pw=1.0, anchor_t=4.0, fl_gamma=0.0,
                   label_smoothing=0.0, hsv_h=0.015, hsv_s=0.7, hsv_v=0.4, degrees=0.0, translate=0.1, scale=0.5,
                   shear=0.0, perspective=0.0, flipud=0.0, fliplr=0.5, mosaic=1.0, mixup=0.0, copy_paste=0.0)


def scaled_hyp(hyp, nc, imgsz, nl=3):
    """train.py:330-335."""
    h = dict(hyp)
    h['box'] *= 3 / nl
    h['cls'] *= nc / 80 * 3 / nl
    h['obj'] *= (imgsz / 640) ** 2 * 3 / nl
    return h


def images(n, size, seed=1, device='cpu'):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (n, 3, size, size), generator=g, dtype=torch.uint8).to(device)


def targets(n, nc, per_image=50, seed=1, device='cpu'):
    """class ~ U[0,nc), centre ~ U(0.05,0.95), wh ~ log-uniform(0.005, 0.1) of the image side."""
    g = torch.Generator().manual_seed(seed + 7)
    nt = n * per_image
    b = torch.arange(n).repeat_interleave(per_image).float()
    c = torch.randint(0, nc, (nt,), generator=g).float()
    xy = torch.rand(nt, 2, generator=g) * 0.9 + 0.05
    wh = torch.exp(torch.rand(nt, 2, generator=g) * (math.log(0.1) - math.log(0.005)) + math.log(0.005))
    return torch.cat([b[:, None], c[:, None], xy, wh], 1).to(device)


def clustered_predictions(n_img, A, nc, n_clusters=200, per=10, seed=2, device='cpu'):
    """Detect-shaped predictions with a controlled number of above-threshold boxes (NMS load)."""
    g = torch.Generator().manual_seed(seed)
    p = torch.zeros(n_img, A, nc + 5)
    p[..., :2] = torch.rand(n_img, A, 2, generator=g) * 640
    p[..., 2:4] = torch.rand(n_img, A, 2, generator=g) * 40 + 2
    p[..., 4] = torch.rand(n_img, A, generator=g) * 0.2
    p[..., 5:] = torch.rand(n_img, A, nc, generator=g)
    for b in range(n_img):
        idx = torch.randperm(A, generator=g)[:n_clusters * per]
        cen = torch.rand(n_clusters, 2, generator=g) * 640
        wh = torch.rand(n_clusters, 2, generator=g) * 60 + 10
        for ci in range(n_clusters):
            ii = idx[ci * per:(ci + 1) * per]
            p[b, ii, :2] = cen[ci] + torch.randn(per, 2, generator=g) * 3
            p[b, ii, 2:4] = wh[ci] * (1 + 0.1 * torch.randn(per, 2, generator=g))
            p[b, ii, 4] = torch.rand(per, generator=g) * 0.7 + 0.3
    return p.to(device)
