"""CPU restatement of the validation matching (TEST INFRASTRUCTURE ONLY: imported by tests/ only).

  box_iou        utils/metrics.py:254-276   pinned by tests/golden/box_iou.npz (reference output)
  process_batch  val.py:62-83               parity unpinned against the reference itself: no reference test
                 or fixture covers it and the reference was not imported to capture one;
                 pinned by hand-derived known answers in tests/test_oracle_metrics.py instead.
"""
import numpy as np
import torch


def box_iou(box1, box2):
    """utils/metrics.py:254-276: [N, 4] x [M, 4] xyxy -> [N, M], no eps."""
    area1 = (box1[:, 2] - box1[:, 0]) * (box1[:, 3] - box1[:, 1])
    area2 = (box2[:, 2] - box2[:, 0]) * (box2[:, 3] - box2[:, 1])
    lt = torch.max(box1[:, None, :2], box2[:, :2])
    rb = torch.min(box1[:, None, 2:], box2[:, 2:])
    inter = (rb - lt).clamp(0).prod(2)
    return inter / (area1[:, None] + area2 - inter)


def process_batch(detections, labels, iouv):
    """val.py:62-83.  detections [N, 6] (x1 y1 x2 y2 conf cls), labels [M, 5] (cls x1 y1 x2 y2) -> bool [N, T].
    Candidate (label, detection) pairs with IoU >= iouv[0] and equal class, in torch.where (row-major) order;
    highest IoU per detection (IoU sorted descending with numpy's default argsort, reversed), then per label the
    surviving pair with the smallest detection index (val.py:77-79: the second unique runs on rows ordered by
    detection, the IoU re-sort at val.py:78 is commented out).  Exact IoU ties (duplicate label boxes) are
    ordered by a STABLE argsort here: numpy's default argsort is stable only for small inputs (insertion
    sort) and leaves ties unspecified otherwise, so the restatement fixes the small-input behaviour."""
    correct = torch.zeros(detections.shape[0], iouv.shape[0], dtype=torch.bool)
    iou = box_iou(labels[:, 1:], detections[:, :4])
    li, di = torch.where((iou >= iouv[0]) & (labels[:, 0:1] == detections[:, 5]))
    if li.shape[0] == 0:
        return correct
    m = torch.cat((torch.stack((li, di), 1), iou[li, di][:, None]), 1).numpy()
    if m.shape[0] > 1:
        m = m[m[:, 2].argsort(kind='stable')[::-1]]  # exact ties: later where-index first (see docstring)
        m = m[np.unique(m[:, 1], return_index=True)[1]]
        m = m[np.unique(m[:, 0], return_index=True)[1]]
    m = torch.tensor(m)
    correct[m[:, 1].long()] = m[:, 2:3] >= iouv
    return correct
