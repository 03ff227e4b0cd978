"""GPU: deterministic mode (functional.set_deterministic; SURVEY §5 "run-twice bitwise checks").

With the split-K weight-gradients reduced in split order through a workspace (dmy_conv_wgrad_det) and the loss's
order-fixed partial sums / per-cell gradient combine (always on), one full training step -- forward, ComputeLoss,
backward, GradScaler + SGD, EMA -- run twice from the same state gives bit-identical loss, gradients, parameters,
BN running statistics and EMA weights, in fp32 and in bf16 storage.  Models: yolov5n (Conv / C3 / SPPF / Detect) at a
size where the weight-gradients use several splits, so the workspace path is exercised."""
import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
CFG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'dma-yolo_amd', 'dmayolo', 'configs')


@pytest.fixture
def deterministic():
    import dmayolo.functional as Fn
    Fn.set_deterministic(True)
    yield
    Fn.set_deterministic(False)


def _state(m, ema):
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    sd.update({'ema.' + k: v.detach().clone() for k, v in ema.ema.state_dict().items()})
    return sd


@pytest.mark.parametrize('topology', ['yolov5n', 'dma'])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_train_step_run_twice_bitwise(deterministic, dtype, topology):
    from dmayolo.models.yolo import Model
    from dmayolo.trainer import Trainer
    from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp
    from golden_util import Fixture
    torch.manual_seed(0)
    cfg = os.path.join(CFG, 'yolov5n.yaml') if topology == 'yolov5n' else Fixture('model_dma').meta['yaml']
    base = Model(cfg, nc=10, act_dtype=dtype)
    for mod in base.modules():
        if type(mod).__name__ == 'SwinTransformerLayer':
            mod.drop_path = torch.nn.Identity()  # the DropPath draw is the RNG's, not a reduction order
    base = base.cuda().train()
    base.hyp = scaled_hyp(HYP_VISDRONE, 10, 256)
    x = images(8, 256, seed=1, device='cuda')
    t = targets(8, 10, seed=1, device='cuda')
    runs = []
    for _ in range(2):
        m = copy.deepcopy(base)
        tr = Trainer(m, dict(m.hyp), 64, nb=100)  # nominal batch 64: accumulate 1, an optimizer step every call
        tr.i = 500  # mid-warmup: every group has a non-zero lr
        for _ in range(2):  # two optimizer steps: the second one's forward already sees the first's updates
            loss, items = tr.step(x, t)
        torch.cuda.synchronize()
        runs.append((loss.detach().clone(), items.clone(), _state(m, tr.ema)))
    (l0, i0, s0), (l1, i1, s1) = runs
    assert torch.equal(l0, l1) and torch.equal(i0, i1), (l0, l1)
    diff = [k for k in s0 if not torch.equal(s0[k], s1[k])]
    assert not diff, diff[:10]


def test_wgrad_det_matches_atomic_sums(deterministic):
    """The workspace path computes the same sums as the atomic path (to fp32 reordering) and is bit-stable."""
    from dmayolo.functional import call, ptr, stream
    torch.manual_seed(0)
    N, H, W, C, K = 8, 64, 64, 64, 128
    x = torch.randn(N, H, W, C, device='cuda').bfloat16()
    dy = torch.randn(N, H, W, K, device='cuda').bfloat16()
    args = (1, ptr(x), ptr(dy))
    geo = (N, H, W, C, C, K, 3, 3, 1, 1, H, W, K)
    ne = call('dmy_conv_wgrad_ws_elems', *args, *geo, 0)
    assert ne > 0  # several splits at this size
    outs = []
    for _ in range(2):
        dw = torch.empty(K * 9 * C, device='cuda')
        ws = torch.empty(ne, device='cuda')
        call('dmy_conv_wgrad_det', *args, ptr(dw), *geo, 0, ptr(ws), ne, stream())
        outs.append(dw)
    dwa = torch.empty(K * 9 * C, device='cuda')
    call('dmy_conv_wgrad_ex', *args, ptr(dwa), *geo, 0, stream())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    torch.testing.assert_close(outs[0], dwa, rtol=1e-4, atol=1e-3)
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).float(), (K, C, 3, 3), dy.permute(0, 3, 1, 2).float(),
                                      padding=1)
    torch.testing.assert_close(outs[0].view(K, 3, 3, C).permute(0, 3, 1, 2), ref, rtol=1e-3, atol=1e-2)
