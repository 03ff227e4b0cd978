"""Config-5 anchors (models/yolov5l-xs-tr-cbam-spp-bifpn.yaml, `anchors: 4` placeholder) as train.py:318's
check_anchors would set them at train start: kmean_anchors (utils/autoanchor.py:64-162, dmayolo.utils.autoanchor)
on the synthetic UAVDT-shaped label set of bench.py (50 targets / image, 1,000 images at 1920 x 1920)
with numpy / random seeded 0, anchor_t 3.0 (hyp.VisDrone.yaml:14), 1,000 generations.

python tools/gen_c5_anchors.py   ->  tests/golden/c5_anchors.json  (16 anchors in pixels, small to large, + BPRs)
"""
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]


def synthetic_labels(n_img=1000, nc=3, per=50, seed=0):
    from dmayolo.synthetic import targets
    t = targets(n_img, nc, per_image=per, seed=seed).numpy()
    labels = [t[t[:, 0] == i][:, 1:] for i in range(n_img)]
    shapes = np.full((n_img, 2), 1920.0)
    return shapes, labels


def main():
    import torch
    from dmayolo.utils.autoanchor import kmean_anchors, _ratio_metric, label_wh
    shapes, labels = synthetic_labels()
    np.random.seed(0)
    random.seed(0)
    k = kmean_anchors(shapes, labels, n=16, img_size=1920, thr=3.0, gen=1000)
    wh = torch.tensor(label_wh(shapes, labels, 1920), dtype=torch.float32)
    # `anchors: 4` -> [list(range(8))] * nl in pixels (models/yolo.py:432-436), the same 4 tiny anchors per level
    ph = torch.tensor([[float(a), float(b)] for _ in range(4) for a, b in zip(range(0, 8, 2), range(1, 8, 2))])
    bpr = lambda kk: float((_ratio_metric(kk, wh)[1] > 1 / 3.0).float().mean())  # noqa: E731
    out = dict(anchors=[[round(float(a), 4), round(float(b), 4)] for a, b in k],
               bpr=bpr(torch.tensor(k, dtype=torch.float32)), bpr_placeholder=bpr(ph),
               source='tools/gen_c5_anchors.py: kmean_anchors(n=16, img_size=1920, thr=3.0, gen=1000), seeds 0, '
                      '1000 synthetic images x 50 targets (dmayolo.synthetic.targets, nc=3, seed 0)')
    path = os.path.join(ROOT, 'tests', 'golden', 'c5_anchors.json')
    with open(path, 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
