"""GPU parity of whole models (product Model/parse_model) against golden vectors captured from
the reference: train-mode outputs, parameter gradients, eval-mode decoded predictions."""
import pytest
import torch

from golden_util import Fixture, load_sd

pytestmark = pytest.mark.gpu


def _model(fx, dtype=torch.float32):
    from dmayolo.models.yolo import Model
    m = Model(fx.meta['yaml'], nc=fx.meta['nc'], act_dtype=dtype)
    load_sd(m, fx.group('sd'))
    for mod in m.modules():
        if type(mod).__name__ == 'SwinTransformerLayer':
            mod.drop_path = torch.nn.Identity()
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    return m.cuda()


@pytest.mark.parametrize('name', ['model_v5s', 'model_dma', 'model_c5'])
def test_model_train_eval_fp32(name):
    fx = Fixture(name)
    m = _model(fx)
    x = fx.t('in.0').cuda()
    m.train()
    outs = m(x)
    gups = [g.cuda() for g in fx.seq('gup')]
    loss = sum((o.float() * g).sum() for o, g in zip(outs, gups))
    loss.backward()
    for a, b in zip(outs, fx.seq('out')):
        torch.testing.assert_close(a.float().cpu(), b, rtol=1e-3, atol=1e-3)
    params = dict(m.named_parameters())
    for k, g in fx.group('gp').items():
        torch.testing.assert_close(params[k].grad.cpu(), g, rtol=2e-3, atol=2e-3 * max(1.0, float(g.abs().max())))
    gn = fx.t('gnorm')
    names = [str(s) for s in fx.z['pnames']]
    got = torch.tensor([float(params[k].grad.norm()) if params[k].grad is not None else 0.0 for k in names],
                       dtype=torch.float64)
    torch.testing.assert_close(got, gn, rtol=5e-3, atol=1e-5)  # zero-grad biases before BN: noise in the reference
    load_sd(m, fx.group('sd'))
    m.eval()
    with torch.no_grad():
        z, _ = m(x)
    torch.testing.assert_close(z.cpu(), fx.t('eout.0'), rtol=1e-3, atol=2e-3)


def test_model_bf16_close_to_fp32():
    fx = Fixture('model_v5s')
    m32, m16 = _model(fx), _model(fx, torch.bfloat16)
    x = fx.t('in.0').cuda()
    m32.eval()
    m16.eval()
    with torch.no_grad():
        z32, _ = m32(x)
        z16, _ = m16(x)
    err = (z16 - z32).abs().max() / z32.abs().max()
    assert float(err) < 2e-2, float(err)
