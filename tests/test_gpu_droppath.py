"""GPU: DropPath's product paths (models/swin.py DropPath -> Fn.SampleScaleFn -> dmy_sample_scale, and DropPath.add ->
Fn.DropPathAddFn -> dmy_droppath_add, the form the Swin layers use), which the
model goldens bypass (they set drop_path = Identity to be deterministic).  Reference semantics, models/common.py
drop_path: keep = 1 - p; mask = floor(keep + rand(N, 1, ...)); out = x / keep * mask -- one uniform draw per sample
from torch's generator, so the same seed gives the same mask here.  Forward and backward are compared with that
formula on the same draw (fp32: to one rounding, x * (1/keep) vs x / keep; bf16: the same within bf16 rounding)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('shape', [(8, 64, 12, 10), (6, 49, 96)])
def test_drop_path_matches_reference_formula(dtype, shape):
    from dmayolo.models.swin import DropPath
    p = 0.375
    g = torch.Generator().manual_seed(5)
    x = torch.randn(*shape, generator=g).to(dtype).cuda()
    if x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    dy = torch.randn(*shape, generator=g).to(dtype).cuda()
    m = DropPath(p).train()
    torch.cuda.manual_seed(123)
    y = m(x)
    y.backward(dy)
    torch.cuda.manual_seed(123)
    keep = 1 - p
    mask = (keep + torch.rand((shape[0],) + (1,) * (len(shape) - 1), dtype=torch.float32, device='cuda')).floor_()
    ref = x.detach().float().div(keep) * mask
    dref = dy.float().div(keep) * mask
    tol = dict(rtol=1e-6, atol=0) if dtype == torch.float32 else dict(rtol=8e-3, atol=0)
    torch.testing.assert_close(y.float(), ref, **tol)
    torch.testing.assert_close(x.grad.float(), dref, **tol)
    kept = mask.flatten()
    assert 0 < int(kept.sum()) < shape[0], 'the seed should drop some samples and keep others'
    assert torch.all(y.float().flatten(1)[kept == 0] == 0)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('shape', [(8, 64, 12, 10), (6, 49, 96), (5, 40, 7, 9)])
def test_drop_path_add_matches_reference_formula(dtype, shape):
    """DropPath.add (functional.DropPathAddFn, one dmy_droppath_add pass): x + DropPath(f) on the same torch draw as
    the reference formula; dx = dy, df = dy * mask / keep.  (5, 40, 7, 9): a sample size that is no multiple of 8 (the
    scalar path)"""
    from dmayolo.models.swin import DropPath
    p = 0.375
    g = torch.Generator().manual_seed(6)
    mk = lambda: torch.randn(*shape, generator=g).to(dtype).cuda()  # noqa: E731
    x, f, dy = mk(), mk(), mk()
    if x.dim() == 4:
        x, f = (t.contiguous(memory_format=torch.channels_last) for t in (x, f))
    x.requires_grad_(True)
    f.requires_grad_(True)
    m = DropPath(p).train()
    torch.cuda.manual_seed(321)
    y = m.add(x, f)
    y.backward(dy)
    torch.cuda.manual_seed(321)
    keep = 1 - p
    mask = (keep + torch.rand((shape[0],) + (1,) * (len(shape) - 1), dtype=torch.float32, device='cuda')).floor_()
    ref = x.detach().float() + f.detach().float() * (mask / keep)
    tol = dict(rtol=1e-6, atol=1e-6) if dtype == torch.float32 else dict(rtol=8e-3, atol=1e-2)
    torch.testing.assert_close(y.float(), ref, **tol)
    torch.testing.assert_close(x.grad.float(), dy.float(), rtol=0, atol=0)
    torch.testing.assert_close(f.grad.float(), dy.float() * (mask / keep), **tol)
    assert 0 < int(mask.sum()) < shape[0], 'the seed should drop some samples and keep others'


def test_drop_path_identity_in_eval_and_at_zero():
    from dmayolo.models.swin import DropPath
    x = torch.randn(4, 8, 5, 5, device='cuda')
    assert DropPath(0.5).eval()(x) is x
    assert DropPath(0.0).train()(x) is x


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_c3str_active_droppath_inplace_concat_matches_copy(dtype):
    """with DropPath active (train mode) the last Swin layer cannot write into the C3STR concat slice, so
    C3.forward's in-place mode (DMY_INPLACE_CAT=2) mixes a producer that returns its own tensor (Swin) with one that
    wrote in place (cv2).  Forward, input gradient and every parameter gradient must equal the copying concat
    (DMY_INPLACE_CAT=0) on the same DropPath draws (same CUDA seed), bit for bit: the kernels and their operands are
    the same, only where the concat's halves come from differs."""
    import copy
    from dmayolo.models import common as P
    from dmayolo.models.swin import DropPath
    torch.manual_seed(0)
    base = P.C3STR(64, 64, n=2)
    for layer in base.m.tr:
        layer.drop_path = DropPath(0.4)
    base = base.cuda().train()
    g = torch.Generator().manual_seed(7)
    x0 = torch.randn(4, 64, 16, 16, generator=g).to(dtype).cuda().contiguous(memory_format=torch.channels_last)
    gup = torch.randn(4, 64, 16, 16, generator=g).to(dtype).cuda().contiguous(memory_format=torch.channels_last)
    import dmayolo.functional as Fn
    res = []
    old = P._INPLACE_CAT
    Fn.set_deterministic(True)  # split-K weight-grads reduced in split order: the two runs sum identically
    try:
        for mode in (0, 2):
            P._INPLACE_CAT = mode
            m = copy.deepcopy(base)
            x = x0.clone().requires_grad_(True)
            torch.cuda.manual_seed(321)
            y = m(x)
            y.backward(gup)
            res.append((y.detach().float(), x.grad.float(), {k: p.grad.clone() for k, p in m.named_parameters()
                                                             if p.grad is not None}))
    finally:
        P._INPLACE_CAT = old
        Fn.set_deterministic(False)
    (y0, gx0, gp0), (y2, gx2, gp2) = res
    torch.cuda.manual_seed(321)
    drops = [float((0.6 + torch.rand(4, device='cuda')).floor_().sum()) for _ in range(4)]
    assert any(d < 4 for d in drops), 'the seed should drop at least one sample in some layer'
    assert torch.equal(y0, y2)
    assert torch.equal(gx0, gx2)
    assert set(gp0) == set(gp2) and len(gp0) > 10
    diff = [k for k in gp0 if not torch.equal(gp0[k], gp2[k])]
    assert not diff, diff
