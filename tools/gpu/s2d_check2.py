"""s2d vs strided stem on the model_c5 fixture input: layer-0 forward + grads in both orders."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'dma-yolo_amd')]
from golden_util import Fixture  # noqa: E402
from test_gpu_model import _model  # noqa: E402

fx = Fixture('model_c5')
x = fx.t('in.0').cuda()
print('input range', float(x.min()), float(x.max()), x.shape, x.is_contiguous(), flush=True)
res = {}
for s2d in (False, True, False, True):
    m = _model(fx)
    m.s2d_stem = s2d
    m.train()
    xi = m.to_input(x)
    y0 = m.model[0](xi)
    g = torch.randn(y0.shape, generator=torch.Generator().manual_seed(3)).cuda()
    (y0.float() * g).sum().backward()
    r = (y0.detach().float().clone(), m.model[0].conv.weight.grad.clone(), m.model[0].bn.weight.grad.clone())
    if s2d in res:
        print('repeat', s2d, [float((a - b).abs().max()) for a, b in zip(r, res[s2d])])
    res[s2d] = r
a, b = res[True], res[False]
print('s2d vs strided', [float((p - q).abs().max() / max(1e-6, float(q.abs().max()))) for p, q in zip(a, b)])
d = (a[0] - b[0]).abs()
idx = (d == d.max()).nonzero()[:5]
print('worst y0 idx', idx.tolist(), flush=True)
