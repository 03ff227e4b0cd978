"""GPU parity of the anchor-free TAL path (csrc/tal.hip) against golden vectors from the reference:
ComputeLoss_TAL loss / items / gradients, the TDetect head (train outputs, grads, inference decode),
space_to_depth, and a bf16 CASPD_ODRTA (P2-P5 TDetect) training step."""
import os

import pytest
import torch

from golden_util import Fixture, load_sd
from gpu_util import rel_err

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Det:
    def __init__(self, nc, strides):
        self.nc, self.nl = nc, len(strides)
        self.stride = torch.tensor(strides, dtype=torch.float32)
        self.stride_list = list(strides)


class _Model:
    def __init__(self, det, hyp):
        self.model = [det]
        self.hyp = hyp


@pytest.mark.parametrize('tag', ['a', 'b'])
def test_tal_loss_vs_reference_golden(tag):
    from dmayolo.utils.tal import ComputeLoss_TAL
    fx = Fixture(f'tal_loss_{tag}')
    meta = fx.meta
    cl = ComputeLoss_TAL(_Model(_Det(meta['nc'], meta['strides']), meta['hyp']))
    feats = [torch.zeros(2, meta['nc'] + 64, h, w, device='cuda') for h, w in meta['shapes']]
    pd = fx.t('pdist').cuda().requires_grad_(True)
    pc = fx.t('pcls').cuda().requires_grad_(True)
    loss, items = cl((feats, pd, pc), fx.t('targets'))
    loss.backward()
    torch.testing.assert_close(items.cpu(), fx.t('items'), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(loss.cpu().reshape(-1), fx.t('loss').reshape(-1), rtol=1e-4, atol=1e-5)
    for got, key in ((pd.grad, 'g_pdist'), (pc.grad, 'g_pcls')):
        ref = fx.t(key)
        torch.testing.assert_close(got.cpu(), ref, rtol=1e-3, atol=1e-5 * float(ref.abs().max()))


def test_tal_loss_channel_major_and_anchor_major_agree():
    """The loss reads box / cls through strides: [B, C, A] tensors and the TDetect anchor-major views
    of one [B, A, 64 + nc] buffer give the same loss and gradients."""
    from dmayolo.utils.tal import ComputeLoss_TAL
    fx = Fixture('tal_loss_a')
    meta = fx.meta
    cl = ComputeLoss_TAL(_Model(_Det(meta['nc'], meta['strides']), meta['hyp']))
    feats = [torch.zeros(2, meta['nc'] + 64, h, w, device='cuda') for h, w in meta['shapes']]
    pd0, pc0 = fx.t('pdist').cuda(), fx.t('pcls').cuda()
    flat = torch.cat((pd0, pc0), 1).permute(0, 2, 1).contiguous().requires_grad_(True)
    l1, i1 = cl((feats, flat[..., :64].permute(0, 2, 1), flat[..., 64:].permute(0, 2, 1)), fx.t('targets'))
    l1.backward()
    pd, pc = pd0.clone().requires_grad_(True), pc0.clone().requires_grad_(True)
    l2, i2 = cl((feats, pd, pc), fx.t('targets'))
    l2.backward()
    torch.testing.assert_close(i1, i2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(flat.grad[..., :64].permute(0, 2, 1), pd.grad, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(flat.grad[..., 64:].permute(0, 2, 1), pc.grad, rtol=1e-5, atol=1e-7)


def test_tdetect_vs_reference_golden():
    from dmayolo.models.tdetect import TDetect
    from oracle.nn import bn_defaults
    fx = Fixture('tdetect')
    meta = fx.meta
    det = bn_defaults(TDetect(meta['args'][0], meta['args'][1]))
    det.stride = torch.tensor(meta['stride'])
    det.stride_list = list(meta['stride'])
    load_sd(det, fx.group('sd'))
    det = det.cuda().train()
    xs = [x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True) for x in fx.seq('in')]
    lvl, box, cls = det(list(xs))
    outs = list(lvl) + [box, cls]
    for o, r in zip(outs, fx.seq('out')):
        torch.testing.assert_close(o.float().cpu(), r, rtol=2e-4, atol=2e-4)
    sum((o.float() * g.cuda()).sum() for o, g in zip(outs, fx.seq('gup'))).backward()
    for x, r in zip(xs, fx.seq('gin')):
        torch.testing.assert_close(x.grad.float().cpu(), r, rtol=1e-3, atol=1e-3 * max(1.0, float(r.abs().max())))
    gp = fx.group('gp')
    for k, p in det.named_parameters():
        if k in gp:
            torch.testing.assert_close(p.grad.cpu(), gp[k], rtol=1e-3, atol=1e-3 * max(1.0, float(gp[k].abs().max())))
    load_sd(det, {k: v.cuda() for k, v in fx.group('sd').items()})
    det.eval()
    with torch.no_grad():
        y, _ = det([x.detach() for x in fx.seq('in')] if False else [x.cuda() for x in fx.seq('in')])
    torch.testing.assert_close(y.cpu(), fx.t('eout.0'), rtol=2e-4, atol=2e-3)


def test_space_to_depth_vs_reference_golden():
    from dmayolo.functional import SpaceToDepthFn
    fx = Fixture('space_to_depth')
    x = fx.t('in.0').cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = SpaceToDepthFn.apply(x)
    assert torch.equal(y.cpu(), fx.t('out.0'))
    g = torch.randn(y.shape, device='cuda')
    y.backward(g)
    ref = torch.zeros(x.shape)
    C = x.shape[1]
    gc = g.cpu()
    ref[..., ::2, ::2] = gc[:, :C]
    ref[..., 1::2, ::2] = gc[:, C:2 * C]
    ref[..., ::2, 1::2] = gc[:, 2 * C:3 * C]
    ref[..., 1::2, 1::2] = gc[:, 3 * C:]
    assert torch.equal(x.grad.cpu(), ref)


def test_caspd_tal_train_step_bf16():
    """A reduced-width CASPD_ODRTA (space_to_depth, C3CA, P2-P5 TDetect) trains one bf16 step with
    ComputeLoss_TAL: finite loss, every parameter that the reference optimises gets a finite gradient."""
    import yaml
    from dmayolo.models.yolo import Model
    from dmayolo.utils.tal import ComputeLoss_TAL
    from dmayolo.synthetic import HYP_VISDRONE, images, targets
    d = yaml.safe_load(open(os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs', 'CASPD_ODRTA.yaml')))
    d['width_multiple'], d['depth_multiple'] = 0.125, 0.33
    torch.manual_seed(0)
    m = Model(d, nc=10, act_dtype=torch.bfloat16).cuda()
    m.hyp = dict(HYP_VISDRONE)
    cl = ComputeLoss_TAL(m)
    x = images(2, 128, device='cuda')
    t = targets(2, 10, per_image=8)
    loss, items = cl(m(x), t)
    loss.backward()
    assert torch.isfinite(loss).all() and torch.isfinite(items).all(), items
    bad = [k for k, p in m.named_parameters() if p.requires_grad and (p.grad is None or not torch.isfinite(p.grad).all())]
    assert not bad, bad[:5]
