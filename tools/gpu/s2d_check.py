"""Stem weight-grad error vs the reference golden with the s2d stem on / off (model_c5 fp32)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'dma-yolo_amd')]
from golden_util import Fixture  # noqa: E402
from test_gpu_model import _model  # noqa: E402

for name in sys.argv[1:] or ['model_c5', 'model_dma', 'model_v5s']:
    fx = Fixture(name)
    for s2d in [bool(int(c)) for c in os.environ.get('ORDER', '10')]:
        m = _model(fx)
        m.s2d_stem = s2d
        x = fx.t('in.0').cuda()
        m.train()
        outs = m(x)
        loss = sum((o.float() * g.cuda()).sum() for o, g in zip(outs, fx.seq('gup')))
        loss.backward()
        params = dict(m.named_parameters())
        worst = []
        for k, g in fx.group('gp').items():
            d = (params[k].grad.cpu() - g).abs()
            worst.append((float(d.max() / max(1.0, float(g.abs().max()))), k, float(g.abs().max())))
        worst.sort(reverse=True)
        print(name, 'x', tuple(x.shape), x.dtype, 's2d', s2d, 'worst rel-to-max errors:', worst[:4], flush=True)
