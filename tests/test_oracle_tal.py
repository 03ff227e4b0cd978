"""CPU: the TAL oracle (oracle/tal.py) against golden vectors captured from the reference
(TaskAlignedAssigner, ComputeLoss_TAL and its gradients, TDetect, space_to_depth, CASPD_ODRTA)."""
import pytest
import torch

from golden_util import Fixture, load_sd
from oracle import tal as OT
from oracle import nn as onn


@pytest.mark.parametrize('tag', ['a', 'b'])
def test_oracle_tal_assign(tag):
    fx = Fixture(f'tal_assign_{tag}')
    tl, tb, ts, fg = OT.tal_assign(fx.t('scores'), fx.t('pboxes'), fx.t('pts'), fx.t('labels'), fx.t('gboxes'),
                                   fx.t('gmask'), nc=fx.meta['nc'])
    assert torch.equal(fg, fx.t('fg'))
    m = fx.t('fg')
    assert torch.equal(tl[m], fx.t('t_lab')[m])
    torch.testing.assert_close(tb[m], fx.t('t_box')[m])
    torch.testing.assert_close(ts, fx.t('t_sc'), rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize('tag', ['a', 'b'])
def test_oracle_tal_loss_and_grads(tag):
    fx = Fixture(f'tal_loss_{tag}')
    meta = fx.meta
    feats = [torch.zeros(2, meta['nc'] + 64, h, w) for h, w in meta['shapes']]
    pd = fx.t('pdist').requires_grad_(True)
    pc = fx.t('pcls').requires_grad_(True)
    loss, items = OT.compute_loss_tal(feats, pd, pc, fx.t('targets'), meta['strides'], meta['hyp'], meta['nc'])
    loss.backward()
    torch.testing.assert_close(items, fx.t('items'), rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(loss.reshape(-1), fx.t('loss').reshape(-1), rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(pd.grad, fx.t('g_pdist'), rtol=1e-4, atol=1e-6 * float(fx.t('g_pdist').abs().max()))
    torch.testing.assert_close(pc.grad, fx.t('g_pcls'), rtol=1e-4, atol=1e-6 * float(fx.t('g_pcls').abs().max()))


def test_oracle_tdetect():
    fx = Fixture('tdetect')
    meta = fx.meta
    det = OT.TDetect(meta['args'][0], meta['args'][1])
    onn.bn_defaults(det)
    det.stride = torch.tensor(meta['stride'])
    load_sd(det, fx.group('sd'))
    xs = [x.clone().requires_grad_(True) for x in fx.seq('in')]
    det.train()
    lvl, box, cls = det(list(xs))
    outs = list(lvl) + [box, cls]
    for o, r in zip(outs, fx.seq('out')):
        torch.testing.assert_close(o, r, rtol=1e-4, atol=1e-4)
    sum((o * g).sum() for o, g in zip(outs, fx.seq('gup'))).backward()
    for x, r in zip(xs, fx.seq('gin')):
        torch.testing.assert_close(x.grad, r, rtol=1e-3, atol=1e-3)
    load_sd(det, fx.group('sd'))
    det.eval()
    with torch.no_grad():
        y, _ = det(fx.seq('in'))
    torch.testing.assert_close(y, fx.t('eout.0'), rtol=1e-4, atol=1e-4)


def test_oracle_space_to_depth():
    fx = Fixture('space_to_depth')
    torch.testing.assert_close(OT.space_to_depth(fx.t('in.0')), fx.t('out.0'), rtol=0, atol=0)
