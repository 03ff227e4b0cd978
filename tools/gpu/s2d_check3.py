"""Does any later kernel overwrite the stem's output / saved tensors in the full model_c5 train step?"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'dma-yolo_amd')]
from golden_util import Fixture  # noqa: E402
from test_gpu_model import _model  # noqa: E402

fx = Fixture('model_c5')
x = fx.t('in.0').cuda()
for s2d in (False, True):
    m = _model(fx)
    m.s2d_stem = s2d
    m.train()
    keep = {}

    def hook(mod, inp, out, keep=keep):
        keep['in'] = (inp[0], inp[0].detach().clone())
        keep['out'] = (out, out.detach().clone())

    h0 = m.model[0].register_forward_hook(hook)
    h1 = m.model[1].register_forward_hook(lambda mod, inp, out: keep.__setitem__('out1', (out, out.detach().clone())))
    outs = m(x)
    torch.cuda.synchronize()
    print(s2d, 'after fwd changed:', {k: float((a.detach() - b).abs().max()) for k, (a, b) in keep.items()}, flush=True)
    loss = sum((o.float() * g.cuda()).sum() for o, g in zip(outs, fx.seq('gup')))
    loss.backward()
    torch.cuda.synchronize()
    print(s2d, 'after bwd changed:', {k: float((a.detach() - b).abs().max()) for k, (a, b) in keep.items()}, flush=True)
    print(s2d, 'ptrs', {k: (hex(a.data_ptr()), a.untyped_storage().nbytes()) for k, (a, b) in keep.items()}, flush=True)
    h0.remove()
    h1.remove()
