"""GPU: one SCConv block (models/common.py:1279-1316, k4(k3(x) * sigmoid(x + up(k2(x))))) at the DMA-YOLO-l bench
shapes, product (bf16 storage, HIP kernels) against a plain-torch fp32 restatement of the same block on the same
bf16-rounded input and weights, for an upstream gradient with a per-channel mean (as a Detect-loss gradient has).

A single SCConv has no argmax routing, so unlike the whole-model single-step comparison its gradients are not chaotic
at random init: bf16 storage noise gives relative L2 errors of a few 1e-3 .. 1e-2 and NO norm bias.  Checked per
parameter: relative L2 <= 5e-2 (a BN bias gradient, sum of du over up to 1.18 M pixels that cancels to a small
fraction of its terms: <= 0.1; measured 6.6e-2 for k3's at 768^2 bs2, 1e-2 at 384^2) and |norm ratio - 1| <= 1e-2 --
a dropped partial row, a wrong BN count or a mis-scaled gate gradient is a norm error of several percent.  Measured
(round 4): every weight, dx and y within 5.3e-3 relative and 1e-3 in norm at all three shapes.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_scconv(m, x, r):
    """the reference forward in fp32 torch ops (training-mode BN with batch statistics)"""
    def bn(z, b):
        return F.batch_norm(z, None, None, b.weight.float(), b.bias.float(), True, 0.0, b.eps)

    def conv(z, c):
        return F.conv2d(z, c.weight.float(), None, c.stride, c.padding)
    g = bn(conv(F.avg_pool2d(x, r, r), m.k2[1]), m.k2[2])
    u3 = bn(conv(x, m.k3[0]), m.k3[1])
    gate = torch.sigmoid(x + F.interpolate(g, size=x.shape[2:], mode='nearest'))
    return bn(conv(u3 * gate, m.k4[0]), m.k4[1])


# (N, c1, H, W, c2): DMA-YOLO-l @1536 bs2 model.1 / model.3, and model.1 at the trajectory test's 384 bs4
SHAPES = [(2, 64, 768, 768, 128), (2, 128, 384, 384, 256), (4, 64, 192, 192, 128)]


@pytest.mark.parametrize('N,C,H,W,C2', SHAPES)
def test_scconv_block_grads_vs_fp32(N, C, H, W, C2):
    import copy
    from dmayolo.models.common import SCConv
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.manual_seed(N + C + H)
    m = SCConv(C, C2, 2)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.eps, mod.momentum = 1e-3, 0.03  # yolo.initialize_weights
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.2, 0.2)
        if isinstance(mod, torch.nn.Conv2d):
            mod.weight.data = mod.weight.data.bfloat16().float()
    ref = copy.deepcopy(m).cuda()
    m = m.cuda()
    x0 = torch.randn(N, C, H, W, device='cuda').bfloat16()
    x = x0.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = m(x)
    OH, OW = y.shape[2:]
    gup = (torch.randn(N, C2, OH, OW, device='cuda') + torch.linspace(-0.5, 0.5, C2, device='cuda').view(1, -1, 1, 1))
    (y.float() * gup).sum().backward()
    xr = x0.float().requires_grad_(True)
    yr = _ref_scconv(ref, xr, 4)
    (yr * gup).sum().backward()
    torch.cuda.synchronize()
    rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm())  # noqa: E731
    nr = lambda a, b: float(a.double().norm() / b.double().norm()) - 1  # noqa: E731
    rows = [('y', rel(y.float(), yr), nr(y.float(), yr)), ('dx', rel(x.grad.float(), xr.grad), nr(x.grad.float(), xr.grad))]
    pr = dict(ref.named_parameters())
    for k, p in m.named_parameters():
        rows.append((k, rel(p.grad, pr[k].grad), nr(p.grad, pr[k].grad)))
    print(f'SCConv {C}->{C2} @{H}x{W} bs{N}: ' + ', '.join(f'{k} rel {e:.2e} norm {n:+.2e}' for k, e, n in rows))
    bad = [(k, e, n) for k, e, n in rows if e > (0.1 if k.endswith('1.bias') or k.endswith('2.bias') else 5e-2)
           or abs(n) > 1e-2]
    assert not bad, bad
