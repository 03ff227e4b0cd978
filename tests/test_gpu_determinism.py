"""GPU: deterministic mode (functional.set_deterministic; SURVEY §5 "run-twice bitwise checks").

With the split-K weight-gradients reduced in split order through a workspace (dmy_conv_wgrad_det) and the loss's
order-fixed partial sums / per-cell gradient combine (always on), one full training step -- forward, ComputeLoss,
backward, GradScaler + SGD, EMA -- run twice from the same state gives bit-identical loss, gradients, parameters,
BN running statistics and EMA weights, in fp32 and in bf16 storage.  Models: yolov5n (Conv / C3 / SPPF / Detect) at a
size where the weight-gradients use several splits, so the workspace path is exercised; the DMA-YOLO-l topology (Swin
LayerNorm / bias-table gradients in fixed order) and the config-5 topology (CBAM channel-attention gradient folded
per image in wave order, C3TR attention).  The TAL loss (anchor-free head) sums its terms through per-block partials
folded in block order: run twice on a multi-block problem it is bit-identical too."""
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


@pytest.mark.parametrize('topology', ['yolov5n', 'dma', 'c5'])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_train_step_run_twice_bitwise(deterministic, dtype, topology):
    from dmayolo.models.yolo import Model
    from dmayolo.trainer import Trainer
    from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp
    from golden_util import Fixture
    torch.manual_seed(0)
    cfg = os.path.join(CFG, 'yolov5n.yaml') if topology == 'yolov5n' else Fixture(f'model_{topology}').meta['yaml']
    base = Model(cfg, nc=10, act_dtype=dtype)
    for mod in base.modules():
        if type(mod).__name__ == 'SwinTransformerLayer':
            mod.drop_path = torch.nn.Identity()  # the DropPath draw is the RNG's, not a reduction order
        if type(mod).__name__ == 'TransformerLayer':
            mod.dropout.p = 0.0  # C3TR's dropout mask: the same (the device generator advances between runs)
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


def test_tal_loss_run_twice_bitwise():
    """ComputeLoss_TAL on 8 images @640 (67,200 anchors: hundreds of loss blocks): loss, items and the gradients of
    both head outputs are bit-identical between two calls."""
    from dmayolo.utils.tal import ComputeLoss_TAL
    from golden_util import Fixture
    fx = Fixture('tal_loss_a')
    meta = fx.meta

    class _Det:
        nc, nl = meta['nc'], 3
        stride = torch.tensor([8., 16., 32.])
        stride_list = [8., 16., 32.]

    class _M:
        model = [_Det()]
        hyp = meta['hyp']

    cl = ComputeLoss_TAL(_M())
    g = torch.Generator().manual_seed(3)
    B, shapes = 8, [(80, 80), (40, 40), (20, 20)]
    A = sum(h * w for h, w in shapes)
    feats = [torch.zeros(B, meta['nc'] + 64, h, w, device='cuda') for h, w in shapes]
    pd0 = torch.randn(B, 64, A, generator=g).cuda()
    pc0 = torch.randn(B, meta['nc'], A, generator=g).cuda() - 4
    nt = 200
    t = torch.cat((torch.randint(0, B, (nt, 1), generator=g).float(),
                   torch.randint(0, meta['nc'], (nt, 1), generator=g).float(),
                   torch.rand(nt, 2, generator=g) * 0.8 + 0.1, torch.rand(nt, 2, generator=g) * 0.2 + 0.02), 1)
    outs = []
    for _ in range(2):
        pd, pc = pd0.clone().requires_grad_(True), pc0.clone().requires_grad_(True)
        loss, items = cl((feats, pd, pc), t)
        loss.backward()
        torch.cuda.synchronize()
        outs.append((loss.detach(), items, pd.grad, pc.grad))
    assert float(outs[0][0]) > 0
    for a, b in zip(*outs):
        assert torch.equal(a, b)
