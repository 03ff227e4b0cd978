"""Validation-matching oracle (oracle/metrics.py) on CPU: box_iou against the reference's own output
(tests/golden/box_iou.npz), process_batch against hand-derived known answers (val.py:62-83), and the
product's host-side AP integration (dmayolo/utils/metrics.ap_per_class, utils/metrics.py:21-116)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.metrics import box_iou, process_batch  # noqa: E402
from golden_util import Fixture  # noqa: E402

IOUV = torch.linspace(0.5, 0.95, 10)


def _box(cx, cy, w, h):
    return [cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2]


def _shifted(iou_target, side=64.0):
    """a side x side box and a same-size box shifted in x so that IoU = (s - d) / (s + d) = iou_target"""
    d = side * (1 - iou_target) / (1 + iou_target)
    return [0.0, 0.0, side, side], [d, 0.0, side + d, side]


def test_box_iou_matches_reference_golden():
    fx = Fixture('box_iou')
    got = box_iou(fx.t('a'), fx.t('b'))
    torch.testing.assert_close(got, fx.t('iou'), rtol=0, atol=0)


def test_process_batch_smallest_detection_wins_a_label():
    # label 0 overlapped by d0 (IoU ~0.62) and d1 (IoU ~0.93): the reference keeps d0 (val.py:79, re-sort
    # commented out at :78) -- the higher-IoU d1 is a false positive
    lb, d0 = _shifted(0.62)
    _, d1 = _shifted(0.93)
    det = torch.tensor([d0 + [0.9, 2.0], d1 + [0.8, 2.0]])
    lab = torch.tensor([[2.0] + lb])
    c = process_batch(det, lab, IOUV)
    assert c[1].sum() == 0
    iou0 = float(box_iou(lab[:, 1:], det[:1, :4])[0, 0])
    assert torch.equal(c[0], iou0 >= IOUV)
    assert c[0, :3].all() and not c[0, 3:].any()


def test_process_batch_detection_takes_its_best_label_and_classes_must_match():
    a, d = _shifted(0.75)
    b = [a[0] + 30, a[1], a[2] + 30, a[3]]  # second label further away from d
    det = torch.tensor([d + [0.9, 1.0], d + [0.5, 3.0]])  # d1 has a class no label has
    lab = torch.tensor([[1.0] + b, [1.0] + a])
    c = process_batch(det, lab, IOUV)
    iou = box_iou(lab[:, 1:], det[:, :4])
    assert float(iou[1, 0]) > float(iou[0, 0])
    assert torch.equal(c[0], iou[1, 0] >= IOUV)
    assert not c[1].any()


def test_process_batch_empty_and_below_threshold():
    lb, d = _shifted(0.3)
    det = torch.tensor([d + [0.9, 0.0]])
    assert not process_batch(det, torch.tensor([[0.0] + lb]), IOUV).any()
    assert process_batch(det, torch.zeros(0, 5), IOUV).shape == (1, 10)
    assert process_batch(torch.zeros(0, 6), torch.tensor([[0.0] + lb]), IOUV).shape == (0, 10)


def test_ap_per_class_known_answers():
    from dmayolo.utils.metrics import ap_per_class, compute_ap
    # every prediction a TP at all IoU levels, one per label -> P = R = 1 and AP 0.995: the appended sentinel
    # (recall 1, precision 0) makes np.interp return 0 at x = 1, so the last 1/100 trapezoid is half
    # (utils/metrics.py:102-111; YOLOv5's well-known 0.995 ceiling)
    tp = np.ones((5, 10), dtype=bool)
    p, r, ap, f1, cls = ap_per_class(tp, np.linspace(0.9, 0.5, 5), np.zeros(5), np.zeros(5))
    assert np.allclose(ap, 0.995) and np.allclose(p, 1.0) and np.allclose(r, 1.0)
    # no TP -> AP 0
    p, r, ap, f1, cls = ap_per_class(np.zeros((3, 10), dtype=bool), np.array([0.9, 0.8, 0.7]), np.ones(3),
                                     np.ones(4))
    assert np.allclose(ap, 0.0)
    # half recall at precision 1: the 101-point envelope integrates to 0.5 (+1/101 trapezoid edge)
    ap, mpre, mrec = compute_ap(np.array([0.25, 0.5]), np.array([1.0, 1.0]))
    x = np.linspace(0, 1, 101)
    want = np.trapezoid(np.interp(x, [0, 0.25, 0.5, 1.0], [1, 1, 1, 0]), x)
    assert abs(ap - want) < 1e-12
