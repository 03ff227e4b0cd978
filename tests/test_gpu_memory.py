"""GPU: device memory stays flat across training steps.

Round 4's deferred-BN path for SCConv's k3 (functional.ConvBNActFn with conv_bn_act(defer=True), reference layer
models/common.py:1309-1316) made the Function's ctx hold its own output z through the BnLink, a cycle through the C++
autograd node that Python's GC cannot break: every SCConv's pre-BN output leaked, ~4 GiB per DMA-YOLO-l step at bs32
@1536.  These tests run Trainer steps (forward, ComputeLoss, backward, GradScaler + SGD, EMA; train.py:433-454) and
require torch.cuda.memory_allocated() to be the same after every step from the second on (the first allocates the
optimizer momenta, the EMA copy and the caches)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
CFG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'dma-yolo_amd', 'dmayolo', 'configs')


def _allocated_per_step(yaml, img, bs, steps):
    from dmayolo.models.yolo import Model
    from dmayolo.trainer import Trainer
    from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, yaml), nc=10, act_dtype=torch.bfloat16).cuda().train()
    m.hyp = scaled_hyp(HYP_VISDRONE, 10, img)
    x = images(bs, img, seed=1, device='cuda')
    t = targets(bs, 10, seed=1, device='cuda')
    tr = Trainer(m, dict(m.hyp), 64, nb=100)
    tr.i = 500
    mem = []
    for _ in range(steps):
        loss, _ = tr.step(x, t)
        del loss
        torch.cuda.synchronize()
        mem.append(torch.cuda.memory_allocated())
    return mem


@pytest.mark.parametrize('yaml,img,bs', [('yolov5l-ca-sppfcspc-bifpn-scconv.yaml', 256, 4),
                                         ('yolov5s.yaml', 320, 8),
                                         ('yolov5l-xs-tr-cbam-spp-bifpn.yaml', 256, 2)])
def test_memory_flat_across_train_steps(yaml, img, bs):
    mem = _allocated_per_step(yaml, img, bs, 12)
    grow = [b - a for a, b in zip(mem[1:], mem[2:])]
    # one SCConv z at this size is >= 64 ch * 128^2 px * 4 img * 2 B = 8 MiB: a leak of it per step cannot hide
    # under a 1 MiB bound
    assert max(abs(g) for g in grow) <= (1 << 20), (yaml, [round(v / 2 ** 20, 1) for v in mem])


def test_deferred_bn_path_is_taken_and_does_not_leak():
    """The SCConv gate really takes k3's deferred BN (z carries _dmy_affine) -- so the flat-memory test above
    covers the path that leaked -- and after a forward + backward + del no tensor from it survives."""
    import gc
    import dmayolo.functional as Fn
    from dmayolo.models.common import SCConv
    assert Fn.DEFER_AFFINE[0]
    torch.manual_seed(0)
    mod = SCConv(64, 128, 2).cuda().train()
    x = torch.randn(4, 64, 96, 96, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    seen = []
    orig = Fn.SCGateFn.forward

    def spy(ctx, xx, u3, g, sink=None):
        seen.append(getattr(u3, '_dmy_affine', None) is not None)
        return orig(ctx, xx, u3, g, sink)

    Fn.SCGateFn.forward = staticmethod(spy)
    try:
        before = None
        for i in range(4):
            y = mod(x)
            y.float().sum().backward()
            del y
            x.grad = None
            for p in mod.parameters():
                p.grad = None
            gc.collect()
            torch.cuda.synchronize()
            if i == 1:
                before = torch.cuda.memory_allocated()
        after = torch.cuda.memory_allocated()
    finally:
        Fn.SCGateFn.forward = orig
    assert seen and all(seen)
    assert after == before, (before, after)
