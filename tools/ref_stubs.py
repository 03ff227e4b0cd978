"""In-container-only import shim for the read-only reference at /root/reference.

Used ONLY by tools/gen_golden.py to capture golden vectors.
Never imported by the product, the tests or anything that runs on the GPU box.

Stubs provided (the reference's missing optional deps, none on the hot path's arithmetic
except torchvision.ops.nms, which is restated from torchvision's documented CPU algorithm):
  cv2 (constants only), torchvision.ops.nms, seaborn (empty), utils.plots (no-op; the real
  module fetches a font over the network at import time).
"""
import sys
import types

import torch

REF = '/root/reference'


def _nms(boxes, scores, iou_thres):
    # torchvision CPU semantics: stable descending score order, suppress IoU > thr, no +1 in areas
    order = torch.sort(scores, stable=True, descending=True)[1]
    x1, y1, x2, y2 = boxes.unbind(1)
    areas = (x2 - x1) * (y2 - y1)
    sup = torch.zeros(len(scores), dtype=torch.bool)
    keep = []
    for _i in range(len(order)):
        i = order[_i]
        if sup[i]:
            continue
        keep.append(i)
        j = order[_i + 1:]
        inter = (torch.minimum(x2[i], x2[j]) - torch.maximum(x1[i], x1[j])).clamp(min=0) * \
                (torch.minimum(y2[i], y2[j]) - torch.maximum(y1[i], y1[j])).clamp(min=0)
        sup[j[inter / (areas[i] + areas[j] - inter) > iou_thres]] = True
    return torch.stack(keep) if keep else torch.zeros(0, dtype=torch.long)


def install():
    if 'models.yolo' in sys.modules:
        return sys.modules['models.yolo']
    cv2 = types.ModuleType('cv2')
    cv2.setNumThreads = lambda n: None
    cv2.INTER_AREA = 3
    cv2.INTER_LINEAR = 1
    sys.modules['cv2'] = cv2
    tv = types.ModuleType('torchvision')
    ops = types.ModuleType('torchvision.ops')
    ops.nms = _nms
    tv.ops = ops
    tv.__version__ = '0.0'
    sys.modules['torchvision'] = tv
    sys.modules['torchvision.ops'] = ops
    sys.modules['seaborn'] = types.ModuleType('seaborn')
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import utils  # noqa: reference package
    pl = types.ModuleType('utils.plots')

    class _Colors:
        def __call__(self, i, bgr=False):
            return (0, 0, 0)
    pl.colors = _Colors()
    for _n in ('Annotator', 'feature_visualization', 'output_to_target', 'plot_images', 'plot_labels',
               'plot_evolve', 'plot_results', 'plot_val_study', 'plot_lr_scheduler'):
        setattr(pl, _n, lambda *a, **k: None)
    sys.modules['utils.plots'] = pl
    utils.plots = pl
    import models.yolo as Y
    from models.common import CoorAttention
    Y.CA = CoorAttention  # bind the undefined YAML token CA to CoorAttention
    return Y
