"""Validation metrics: detection/label matching on the GPU (csrc/metrics.hip)
and the per-class AP integration on the host, as the reference does it.

  process_batch        val.py:62-83 (+ box_iou utils/metrics.py:254-276)  -> dmy_process_batch (HIP)
  process_batch_multi  the same for a whole batch of images in one launch
  ap_per_class         utils/metrics.py:21-87   (numpy on the host, like the reference: a few thousand
  compute_ap           utils/metrics.py:90-116   scalars per validation run, not a device workload)
  fitness              utils/metrics.py:15-18
"""
import numpy as np
import torch

from .._lib import call, ptr, stream

_trapz = getattr(np, 'trapezoid', None) or np.trapz  # numpy 2 renamed trapz (same rule)


def process_batch_multi(detections, labels, iouv):
    """detections: list of [n_i, 6] (x1, y1, x2, y2, conf, cls); labels: list of [m_i, 5] (cls, x1, y1, x2, y2),
    all fp32 on one GPU.  Returns the list of correct [n_i, len(iouv)] bool tensors (val.py:62-83 per image)."""
    assert len(detections) == len(labels)
    dev = iouv.device
    if dev.type != 'cuda':
        raise RuntimeError('process_batch runs on the gfx950 kernel: tensors must be on a GPU')
    T = iouv.numel()
    nd = [int(d.shape[0]) for d in detections]
    nl = [int(l.shape[0]) for l in labels]
    ND = sum(nd)
    if ND == 0:
        return [torch.zeros(0, T, dtype=torch.bool, device=dev) for _ in detections]
    det = torch.cat([d[:, :6].float() for d in detections]).contiguous()
    lab = (torch.cat([l[:, :5].float() for l in labels]) if sum(nl) else torch.zeros(0, 5, device=dev)).contiguous()
    offs = torch.tensor(np.concatenate([[0], np.cumsum(nd), [0], np.cumsum(nl)]).astype(np.int32)).to(dev)
    doff, loff = offs[:len(nd) + 1], offs[len(nd) + 1:]
    iv = iouv.float().contiguous()
    ws_lab = torch.empty(ND, dtype=torch.int32, device=dev)
    ws_iou = torch.empty(ND, dtype=torch.float32, device=dev)
    ws_win = torch.empty(ND, dtype=torch.int32, device=dev)
    correct = torch.empty((ND, T), dtype=torch.uint8, device=dev)
    call('dmy_process_batch', ptr(det), ptr(doff), ptr(lab), ptr(loff), len(nd), ptr(iv), T, ptr(ws_lab), ptr(ws_iou),
         ptr(ws_win), ptr(correct), stream())
    return list(correct.bool().split(nd))


def process_batch(detections, labels, iouv):
    """val.py:62-83: correct [N, len(iouv)] for one image (detections [N, 6], labels [M, 5], xyxy)."""
    return process_batch_multi([detections], [labels], iouv)[0]


def compute_ap(recall, precision):
    """utils/metrics.py:90-116 (101-point COCO interpolation of the precision envelope)."""
    mrec = np.concatenate(([0.0], recall, [1.0]))
    mpre = np.concatenate(([1.0], precision, [0.0]))
    mpre = np.flip(np.maximum.accumulate(np.flip(mpre)))
    x = np.linspace(0, 1, 101)
    return _trapz(np.interp(x, mrec, mpre), x), mpre, mrec


def ap_per_class(tp, conf, pred_cls, target_cls):
    """utils/metrics.py:21-87 without the plots: (p, r, ap [nc, T], f1, unique classes).  p / r / f1 are taken at
    the confidence that maximises the class-mean F1 on the 1000-point grid, as the reference."""
    i = np.argsort(-conf)
    tp, conf, pred_cls = tp[i], conf[i], pred_cls[i]
    unique_classes = np.unique(target_cls)
    nc = unique_classes.shape[0]
    px = np.linspace(0, 1, 1000)
    ap, p, r = np.zeros((nc, tp.shape[1])), np.zeros((nc, 1000)), np.zeros((nc, 1000))
    for ci, c in enumerate(unique_classes):
        i = pred_cls == c
        n_l = (target_cls == c).sum()
        n_p = i.sum()
        if n_p == 0 or n_l == 0:
            continue
        fpc = (1 - tp[i]).cumsum(0)
        tpc = tp[i].cumsum(0)
        recall = tpc / (n_l + 1e-16)
        r[ci] = np.interp(-px, -conf[i], recall[:, 0], left=0)
        precision = tpc / (tpc + fpc)
        p[ci] = np.interp(-px, -conf[i], precision[:, 0], left=1)
        for j in range(tp.shape[1]):
            ap[ci, j], _, _ = compute_ap(recall[:, j], precision[:, j])
    f1 = 2 * p * r / (p + r + 1e-16)
    i = f1.mean(0).argmax()
    return p[:, i], r[:, i], ap, f1[:, i], unique_classes.astype('int32')


def fitness(x):
    """utils/metrics.py:15-18: 0.1 mAP@0.5 + 0.9 mAP@0.5:0.95."""
    w = [0.0, 0.0, 0.1, 0.9]
    return (x[:, :4] * w).sum(1)
