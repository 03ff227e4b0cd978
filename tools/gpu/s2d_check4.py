"""model_c5 train step, s2d stem on vs off in one process: y0 / dy0 / every parameter gradient."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'dma-yolo_amd')]
from golden_util import Fixture  # noqa: E402
from test_gpu_model import _model  # noqa: E402

fx = Fixture(os.environ.get('FX', 'model_c5'))
x = fx.t('in.0').cuda()
R = {}
for s2d in (False, True):
    m = _model(fx)
    m.s2d_stem = s2d
    m.train()
    keep = {}

    def hook(mod, inp, out, keep=keep):
        keep['y0'] = out.detach().clone()
        out.register_hook(lambda g: keep.__setitem__('dy0', g.detach().clone()))

    m.model[0].register_forward_hook(hook)
    outs = m(x)
    loss = sum((o.float() * g.cuda()).sum() for o, g in zip(outs, fx.seq('gup')))
    loss.backward()
    keep['grads'] = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    keep['outs'] = [o.detach().float().clone() for o in outs]
    R[s2d] = keep
a, b = R[True], R[False]
rel = lambda p, q: float((p - q).abs().max() / max(1e-9, float(q.abs().max())))
print('y0', rel(a['y0'], b['y0']), 'dy0', rel(a['dy0'], b['dy0']), 'outs', [rel(p, q) for p, q in zip(a['outs'], b['outs'])])
d = sorted(((rel(a['grads'][k], b['grads'][k]), k) for k in b['grads']), reverse=True)
print('grad diffs top', d[:8])
print('missing', set(b['grads']) ^ set(a['grads']))
gp = fx.group('gp')
print('vs golden (s2d on)', sorted(((rel(a['grads'][k].cpu(), g), k) for k, g in gp.items()), reverse=True)[:5])
print('vs golden (s2d off)', sorted(((rel(b['grads'][k].cpu(), g), k) for k, g in gp.items()), reverse=True)[:5])
