"""Validation loop: the statistics part of the reference's val.run (val.py:196-311) on the gfx950 path.

Per batch: model eval forward (Detect decode) -> non_max_suppression(conf 0.001, iou 0.6, multi_label)
-> labels to pixel xyxy -> process_batch for every image of the batch in ONE kernel launch
(utils/metrics.process_batch_multi) -> (correct, conf, pcls, tcls) stats.  At the end ap_per_class
gives P, R, mAP@0.5 and mAP@0.5:0.95 exactly as val.py:283-291.

Batches are what dmayolo.data.create_dataloader yields (datasets.py:624-629's collate: uint8 images at the
network size [N, 3, H, W], normalised targets [nt, 6] (img, cls, x, y, w, h), paths, shapes), or
(img, targets[, shapes]) tensors; `shapes` (per-image (h0, w0), ((ratio), (pad))) drive scale_coords.
Out of scope (control plane): plots, COCO-JSON, confusion matrix, txt saving.
"""
import numpy as np
import torch

from .utils.general import non_max_suppression, scale_coords, xywh2xyxy
from .utils.metrics import ap_per_class, process_batch_multi


def batch_stats(out, targets, img_hw, iouv, shapes=None, single_cls=False):
    """val.py:236-270 for one batch: NMS outputs `out` (list of [k, 6]), targets [nt, 6] with PIXEL xywh ->
    list of (correct [k, T] bool, conf [k], pcls [k], tcls list) numpy tuples; every image's matching in one
    process_batch launch."""
    device, niou = iouv.device, iouv.numel()
    height, width = img_hw
    stats, dets, labs, tcls_all, keep = [], [], [], [], []
    for si, pred in enumerate(out):
        labels = targets[targets[:, 0] == si, 1:]
        nl = len(labels)
        tcls = labels[:, 0].tolist() if nl else []
        if len(pred) == 0:
            if nl:
                stats.append((np.zeros((0, niou), dtype=bool), np.zeros(0, np.float32), np.zeros(0, np.float32), tcls))
            continue
        if single_cls:
            pred[:, 5] = 0
        predn = pred.clone()
        shape0 = shapes[si][0] if shapes is not None else (height, width)
        ratio_pad = shapes[si][1] if shapes is not None else None
        scale_coords((height, width), predn[:, :4], shape0, ratio_pad)
        if nl:
            tbox = xywh2xyxy(labels[:, 1:5])
            scale_coords((height, width), tbox, shape0, ratio_pad)
            labelsn = torch.cat((labels[:, 0:1], tbox), 1)
        else:
            labelsn = torch.zeros((0, 5), device=device)
        dets.append(predn)
        labs.append(labelsn)
        tcls_all.append(tcls)
        keep.append(pred)
    if dets:
        for correct, pred, tcls in zip(process_batch_multi(dets, labs, iouv), keep, tcls_all):
            stats.append((correct.cpu().numpy(), pred[:, 4].float().cpu().numpy(), pred[:, 5].float().cpu().numpy(),
                          tcls))
    return stats


def summarize(stats, nc):
    """val.py:283-291: stats list -> (mp, mr, map50, map, maps [nc], nt [nc])."""
    mp = mr = map50 = map_ = 0.0
    stats = [np.concatenate([np.asarray(s) for s in x], 0) for x in zip(*stats)]
    ap = None
    ap_class = np.zeros(0, dtype=np.int32)
    if len(stats) and stats[0].any():
        p, r, ap, f1, ap_class = ap_per_class(*stats)
        ap50, ap = ap[:, 0], ap.mean(1)
        mp, mr, map50, map_ = p.mean(), r.mean(), ap50.mean(), ap.mean()
        nt = np.bincount(stats[3].astype(np.int64), minlength=nc)
    else:
        nt = np.zeros(nc, dtype=np.int64)
    maps = np.zeros(nc) + map_
    for i, c in enumerate(ap_class):
        maps[c] = ap[i]
    return mp, mr, map50, map_, maps, nt


@torch.no_grad()
def run(model, batches, nc, conf_thres=0.001, iou_thres=0.6, max_det=300, single_cls=False, compute_loss=None):
    """Returns ((mp, mr, map50, map, *loss), maps [nc], seen, nt [nc]) like val.py:303-311."""
    device = next(model.parameters()).device
    was_training = model.training
    model.eval()
    iouv = torch.linspace(0.5, 0.95, 10, device=device)  # val.py:163
    seen = nbatches = 0
    loss = torch.zeros(3, device=device)
    stats = []
    for batch in batches:
        img, targets = batch[0], batch[1]
        shapes = batch[3] if len(batch) > 3 else (batch[2] if len(batch) > 2 else None)  # (img, t, paths, shapes)
        img = img.to(device, non_blocking=True)
        targets = targets.to(device).float()
        nb, _, height, width = img.shape
        out, train_out = model(img)
        if compute_loss:
            loss += compute_loss([x.float() for x in train_out], targets)[1]
        targets[:, 2:] *= torch.tensor([width, height, width, height], device=device, dtype=torch.float32)
        out = non_max_suppression(out, conf_thres, iou_thres, multi_label=True, agnostic=single_cls, max_det=max_det)
        nbatches += 1
        seen += len(out)
        stats += batch_stats(out, targets, (height, width), iouv, shapes, single_cls)
    mp, mr, map50, map_, maps, nt = summarize(stats, nc)
    model.train(was_training)
    loss_items = (loss.cpu() / max(nbatches, 1)).tolist()
    return (mp, mr, map50, map_, *loss_items), maps, seen, nt
