"""GPU: DropPath's product path (models/swin.py DropPath -> Fn.SampleScaleFn -> dmy_sample_scale), which the
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


def test_drop_path_identity_in_eval_and_at_zero():
    from dmayolo.models.swin import DropPath
    x = torch.randn(4, 8, 5, 5, device='cuda')
    assert DropPath(0.5).eval()(x) is x
    assert DropPath(0.0).train()(x) is x
