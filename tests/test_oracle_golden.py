"""Pin the CPU oracle to the reference: oracle vs golden vectors captured from the reference (CPU only)."""
import pytest
import torch

from golden_util import Fixture, golden_names, load_sd
from oracle import nn as onn
from oracle import loss as oloss
from oracle import general as ogen

MODS = {
    'Conv': onn.Conv, 'Bottleneck': onn.Bottleneck, 'C3': onn.C3, 'SCConv': onn.SCConv,
    'CoorAttention': onn.CoorAttention, 'C3CA': onn.C3CA, 'SPPF': onn.SPPF, 'SPPFCSPC': onn.SPPFCSPC,
    'Upsample': torch.nn.Upsample, 'AdConcat2': onn.AdConcat2, 'AdConcat3': onn.AdConcat3, 'Concat': onn.Concat,
    'SwinTransformerLayer': lambda c, h, ws, sh: onn.SwinTransformerLayer(c, h, ws, sh), 'C3STR': onn.C3STR,
    'SPP': lambda c1, c2, k: onn.SPP(c1, c2, tuple(k)), 'CBAM': onn.CBAM, 'C3TR': onn.C3TR,
}

MODULE_CASES = [n for n in golden_names('') if n.split('_')[0] in (
    'conv', 'bottleneck', 'c3', 'scconv', 'ca', 'c3ca', 'sppf', 'sppfcspc', 'upsample', 'adconcat2',
    'adconcat3', 'concat', 'swin', 'c3str', 'spp', 'cbam', 'c3tr') and n != 'conv_fuse']


def run_module_case(name, build=None, device='cpu', dtype=torch.float32):
    """Train-mode fwd+bwd and eval fwd of module `build(meta)` against fixture `name`."""
    fx = Fixture(name)
    meta = fx.meta
    mod = (build or (lambda m: MODS[m['module']](*m['args'])))(meta)
    onn.bn_defaults(mod)
    for m in mod.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0  # the fixtures were captured with dropout off (tools/gen_golden.py randomize_bn)
    load_sd(mod, fx.group('sd'))
    mod = mod.to(device)
    ins = [x.to(device, dtype).requires_grad_(True) for x in fx.seq('in')]
    mod.train()
    listin = meta['module'] in ('AdConcat2', 'AdConcat3', 'Concat')
    out = mod(ins if listin else ins[0])
    outs = list(out) if isinstance(out, (list, tuple)) else [out]
    gups = [g.to(device, dtype) for g in fx.seq('gup')]
    loss = sum((o.float() * g.float()).sum() for o, g in zip(outs, gups))
    loss.backward()
    res = dict(out=[o.detach().float().cpu() for o in outs], gin=[x.grad.float().cpu() for x in ins],
               gp={k: p.grad.float().cpu() for k, p in mod.named_parameters() if p.grad is not None},
               buf={k: v.float().cpu().clone() for k, v in mod.state_dict().items() if 'running' in k})
    mod.load_state_dict({k: v for k, v in mod.state_dict().items()})
    load_sd(mod, fx.group('sd'))
    mod.eval()
    with torch.no_grad():
        eo = mod([x.detach() for x in ins] if listin else ins[0].detach())
    res['eout'] = [o.float().cpu() for o in (eo if isinstance(eo, (list, tuple)) else [eo])]
    return fx, res


def check_module_case(fx, res, rtol, atol, grad_tol=None):
    gt = grad_tol or (rtol, atol)
    for a, b in zip(res['out'], fx.seq('out')):
        torch.testing.assert_close(a, b, rtol=rtol, atol=atol)
    for a, b in zip(res['gin'], fx.seq('gin')):
        torch.testing.assert_close(a, b, rtol=gt[0], atol=gt[1] * max(1.0, float(b.abs().max())))
    gp = fx.group('gp')
    assert set(gp) == set(res['gp']), (set(gp) ^ set(res['gp']))
    for k, b in gp.items():
        torch.testing.assert_close(res['gp'][k], b, rtol=gt[0], atol=gt[1] * max(1.0, float(b.abs().max())),
                                   msg=lambda m: f'{k}: {m}')
    for k, b in fx.group('sd_after').items():
        if 'running' in k:
            torch.testing.assert_close(res['buf'][k], b, rtol=rtol, atol=atol)
    for a, b in zip(res['eout'], fx.seq('eout')):
        torch.testing.assert_close(a, b, rtol=rtol, atol=atol)


@pytest.mark.parametrize('name', MODULE_CASES)
def test_oracle_module(name):
    fx, res = run_module_case(name)
    check_module_case(fx, res, rtol=1e-4, atol=1e-5)


def test_oracle_swin_mask():
    for name in golden_names('swinmask'):
        fx = Fixture(name)
        H, W = fx.meta['H'], fx.meta['W']
        m = onn.swin_mask(-(-H // 8) * 8, -(-W // 8) * 8, 8, 4)
        torch.testing.assert_close(m, fx.t('mask'))


def test_oracle_conv_fuse():
    fx = Fixture('conv_fuse')
    m = onn.bn_defaults(onn.Conv(16, 32, 3, 1))
    load_sd(m, fx.group('sd'))
    m.eval()
    s = m.bn.weight / torch.sqrt(m.bn.running_var + m.bn.eps)
    w = m.conv.weight * s[:, None, None, None]
    b = m.bn.bias - m.bn.running_mean * s
    torch.testing.assert_close(w, fx.t('fw'), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(b, fx.t('fb'), rtol=1e-6, atol=1e-7)
    y = torch.nn.functional.silu(torch.nn.functional.conv2d(fx.t('in.0'), w, b, 1, 1))
    torch.testing.assert_close(y, fx.t('eout.0'), rtol=1e-5, atol=1e-5)


def test_oracle_detect():
    fx = Fixture('detect')
    meta = fx.meta
    d = onn.Detect(meta['nc'], meta['anchors'], meta['ch'])
    d.stride = torch.tensor(meta['stride'], dtype=torch.float32)
    load_sd(d, fx.group('sd'))
    d.train()
    outs = d(fx.seq('in'))
    for a, b in zip(outs, fx.seq('out')):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    d.eval()
    with torch.no_grad():
        z, _ = d(fx.seq('in'))
    torch.testing.assert_close(z, fx.t('eout.0'), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize('hyp', ['VisDrone', 'scratch'])
def test_oracle_loss(hyp):
    fx = Fixture(f'loss_{hyp}')
    meta = fx.meta
    p = [fx.t(f'p.{i}') for i in range(3)]
    anchors = fx.t('anchors')
    tg = oloss.build_targets([x.shape for x in p], fx.t('targets'), anchors, meta['hyp']['anchor_t'])
    for i in range(3):
        for k in ('b', 'a', 'gj', 'gi'):
            assert torch.equal(tg[i][k], fx.t(f'{k}.{i}').long()), (i, k)
        assert torch.equal(tg[i]['tcls'], fx.t(f'tcls.{i}').long())
        torch.testing.assert_close(tg[i]['tbox'], fx.t(f'tbox.{i}'))
        torch.testing.assert_close(tg[i]['anch'], fx.t(f'anch.{i}'))
    pp = [x.clone().requires_grad_(True) for x in p]
    loss, items = oloss.compute_loss(pp, fx.t('targets'), anchors, meta['hyp'], meta['nc'])
    loss.backward()
    torch.testing.assert_close(loss, fx.t('loss'), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(items, fx.t('items'), rtol=1e-5, atol=1e-6)
    for i in range(3):
        torch.testing.assert_close(pp[i].grad, fx.t(f'gp.{i}'), rtol=1e-4, atol=1e-7)


def test_oracle_siou():
    fx = Fixture('siou')
    b1 = fx.t('b1').requires_grad_(True)
    iou = oloss.siou(b1, fx.t('b2'))
    iou.sum().backward()
    torch.testing.assert_close(iou, fx.t('iou'), rtol=1e-5, atol=1e-6, equal_nan=True)
    torch.testing.assert_close(b1.grad, fx.t('g'), rtol=1e-4, atol=1e-5, equal_nan=True)


@pytest.mark.parametrize('name', golden_names('nms_'))
def test_oracle_nms(name):
    fx = Fixture(name)
    out = ogen.non_max_suppression(fx.t('pred'), **fx.meta)
    ref = fx.seq('out')
    assert len(out) == len(ref)
    for a, b in zip(out, ref):
        assert a.shape == b.shape, (a.shape, b.shape)
        assert torch.equal(a, b)


@pytest.mark.parametrize('name', ['model_v5s', 'model_dma', 'model_c5'])
def test_oracle_model(name):
    fx = Fixture(name)
    meta = fx.meta
    m = onn.bn_defaults(onn.Model(meta['yaml'], nc=meta['nc']))
    sd = fx.group('sd')
    load_sd(m, sd)
    for mod in m.modules():
        if isinstance(mod, onn.SwinTransformerLayer):
            mod.drop_prob = 0.0
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    x = fx.t('in.0').requires_grad_(False)
    m.train()
    outs = m(x)
    gups = fx.seq('gup')
    loss = sum((o * g).sum() for o, g in zip(outs, gups))
    loss.backward()
    for a, b in zip(outs, fx.seq('out')):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)
    for k, g in fx.group('gp').items():
        got = dict(m.named_parameters())[k].grad
        torch.testing.assert_close(got, g, rtol=1e-3, atol=1e-4 * max(1.0, float(g.abs().max())))
    load_sd(m, sd)
    m.eval()
    with torch.no_grad():
        z, _ = m(x)
    torch.testing.assert_close(z, fx.t('eout.0'), rtol=1e-3, atol=1e-3)
