"""GPU: the fused 1x1 Conv-BN-act backward (bwd1x1.hip, dmy_conv1x1_bwd_bn) against the three-pass path it replaces
(dmy_bn_bwd_apply -> dmy_conv_dgrad -> dmy_conv_wgrad_ex) and a float64 reference of the same bf16 operands.

The fused kernel computes dz with dmy_bn_bwd_apply's expression in registers and never stores it, so the reference
dz is the apply kernel's own output; dx = bf16(dz Wt) (+ the stored dx, accumulate) and dw = dz^T x are then checked
in float64.  Shapes: every (K, C) pair the kernel is built for, ragged pixel counts (partial last tile, fewer tiles
than CUs), strided dy / x / dx (channel slices of concat buffers), accumulate on and off; then whole modules (a 1x1
Conv, a C3 block whose cv1 / cv2 feed GradSinks) with the fused path on and off."""
import pytest
import torch

pytestmark = pytest.mark.gpu

PAIRS = [(64, 64), (128, 64), (64, 128), (128, 128), (128, 256), (128, 512), (256, 128), (256, 256), (64, 256)]


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _coefs(K, g):
    scale = torch.rand(K, generator=g) * 2 + 0.1
    shift = torch.randn(K, generator=g)
    mean = torch.randn(K, generator=g) * 0.5
    invstd = torch.rand(K, generator=g) * 2 + 0.2
    ca = torch.rand(K, generator=g) + 0.5
    cb = torch.randn(K, generator=g) * 0.1
    cc = torch.randn(K, generator=g) * 0.1
    return [t.float().cuda() for t in (scale, shift, mean, invstd, ca, cb, cc)]


@pytest.mark.parametrize('K,C', PAIRS)
@pytest.mark.parametrize('M,strided,acc', [(4099, False, 0), (64 * 256 * 3 + 17, True, 1), (96, True, 0),
                                           (20000, False, 1)])
def test_bwd1x1_matches_apply_then_gemms(K, C, M, strided, acc):
    from dmayolo.functional import call, ptr, stream
    g = torch.Generator().manual_seed(K * 7 + C + M)
    dps, xps, bps = (K + 64, C + 192, C + 64) if strided else (K, C, C)
    dyb = (torch.randn(M, dps, generator=g) * 0.1).bfloat16().cuda()
    xb = torch.randn(M, xps, generator=g).bfloat16().cuda()
    z = (torch.randn(M, K, generator=g) * 2 + 0.3).bfloat16().cuda()
    w = torch.randn(K, C, generator=g) / C ** 0.5
    wt = w.t().contiguous().bfloat16().cuda()  # the IHWO copy of a 1x1: [C][K]
    old = torch.randn(M, bps, generator=g).bfloat16().cuda()
    dxb = old.clone()
    scale, shift, mean, invstd, ca, cb, cc = _coefs(K, g)
    act = 1  # SiLU
    assert call('dmy_conv1x1_bwd_bn_ok', M, K, C, dps, xps, bps, ptr(dyb), ptr(z), ptr(xb), ptr(dxb)) == 1
    dw = torch.zeros(K, C, device='cuda')
    rc = call('dmy_conv1x1_bwd_bn', ptr(dyb), dps, ptr(z), ptr(xb), xps, ptr(wt), ptr(scale), ptr(shift), ptr(mean),
              ptr(invstd), act, ptr(ca), ptr(cb), ptr(cc), ptr(dxb), bps, acc, ptr(dw), None, 0, M, K, C, stream())
    assert rc == 0
    # deterministic mode (workspace partials summed in block order): the same sums, bit-identical run to run
    ne = call('dmy_conv1x1_bwd_bn_ws_elems', M, K, C)
    dets = []
    for _ in range(2):
        dwd, dxd = torch.zeros(K, C, device='cuda'), old.clone()
        ws = torch.full((ne,), float('nan'), device='cuda')
        call('dmy_conv1x1_bwd_bn', ptr(dyb), dps, ptr(z), ptr(xb), xps, ptr(wt), ptr(scale), ptr(shift), ptr(mean),
             ptr(invstd), act, ptr(ca), ptr(cb), ptr(cc), ptr(dxd), bps, acc, ptr(dwd), ptr(ws), ne, M, K, C, stream())
        dets.append((dwd, dxd))
    assert torch.equal(dets[0][0], dets[1][0]) and torch.equal(dets[0][1], dets[1][1])
    # reference: the apply kernel's dz, then float64 GEMMs of the same bf16 operands
    dz = torch.empty(M, K, dtype=torch.bfloat16, device='cuda')
    assert call('dmy_bn_bwd_apply', 1, ptr(z), K, ptr(dyb), dps, ptr(scale), ptr(shift), ptr(mean), ptr(invstd), act,
                ptr(ca), ptr(cb), ptr(cc), ptr(dz), K, M, K, stream()) == 0
    torch.cuda.synchronize()
    x = xb[:, :C].double()
    dx_ref = (dz.double() @ wt.double().t()).bfloat16()
    if acc:
        dx_ref = (dx_ref.float() + old[:, :C].float()).bfloat16()
    dw_ref = dz.double().t() @ x
    dx = dxb[:, :C]
    # dx: fp32 sums in another order, then one bf16 rounding (and one more after the accumulate add)
    assert _rel(dx, dx_ref) < (3e-3 if acc else 2e-3), _rel(dx, dx_ref)
    assert (dx.float() - dx_ref.float()).abs().max() <= 2e-2 * dx_ref.float().abs().max()
    assert _rel(dw, dw_ref) < 1e-5, _rel(dw, dw_ref)
    assert _rel(dets[0][0], dw_ref) < 1e-5 and torch.equal(dets[0][1], dxb)
    # the slice bounds of the strided dx buffer are untouched
    if bps > C:
        assert torch.equal(dxb[:, C:], old[:, C:])


def test_bwd1x1_unsupported_shapes_launch_nothing():
    from dmayolo.functional import call, ptr, stream
    t = torch.zeros(64, 96, dtype=torch.bfloat16, device='cuda')
    assert call('dmy_conv1x1_bwd_bn_ok', 64, 96, 64, 96, 64, 64, ptr(t), ptr(t), ptr(t), ptr(t)) == 0  # K = 96
    assert call('dmy_conv1x1_bwd_bn_ok', 64, 512, 512, 512, 512, 512, ptr(t), ptr(t), ptr(t), ptr(t)) == 0
    assert call('dmy_conv1x1_bwd_bn_ok', 64, 256, 512, 256, 512, 512, ptr(t), ptr(t), ptr(t), ptr(t)) == 0
    assert call('dmy_conv1x1_bwd_bn_ok', 64, 512, 128, 512, 128, 128, ptr(t), ptr(t), ptr(t), ptr(t)) == 0
    assert call('dmy_conv1x1_bwd_bn_ok', 64, 64, 64, 68, 64, 64, ptr(t), ptr(t), ptr(t), ptr(t)) == 0  # dps % 8
    with pytest.raises(RuntimeError, match='hipError -1'):
        call('dmy_conv1x1_bwd_bn', ptr(t), 64, ptr(t), ptr(t), 64, ptr(t), None, None, None, None, 1, None, None, None,
             ptr(t), 64, 0, None, None, 0, 64, 96, 64, stream())


def _module_grads(mod, x, gup, fused):
    from dmayolo import functional as fn
    prev = fn.BWD1X1[0]
    fn.BWD1X1[0] = fused
    try:
        mod.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        y = mod(xi)
        (y.float() * gup).sum().backward()
        torch.cuda.synchronize()
        return xi.grad.float().clone(), {k: p.grad.clone() for k, p in mod.named_parameters() if p.grad is not None}
    finally:
        fn.BWD1X1[0] = prev


@pytest.mark.parametrize('kind,c1,c2,hw,bs', [('conv', 128, 128, 48, 8), ('conv', 256, 128, 40, 6),
                                              ('conv', 128, 256, 33, 7), ('c3', 128, 128, 40, 4),
                                              ('c3', 256, 256, 24, 4), ('conv', 512, 128, 40, 4),
                                              ('conv', 256, 256, 30, 5), ('conv', 256, 64, 40, 4)])
def test_module_backward_fused_equals_three_pass(kind, c1, c2, hw, bs):
    """the same module, the same bf16 input and upstream gradient: the fused backward against the three-pass path
    (both product kernels): input gradient to one bf16 rounding of reordered sums, parameter gradients to fp32 order"""
    from dmayolo.models.common import Conv, C3
    torch.manual_seed(0)
    mod = (Conv(c1, c2, 1, 1) if kind == 'conv' else C3(c1, c2, n=2)).cuda().train()
    x = torch.randn(bs, c1, hw, hw, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        C = mod(x).shape[1]
    gup = torch.randn(bs, C, hw, hw, device='cuda') + torch.linspace(-0.5, 0.5, C, device='cuda').view(1, -1, 1, 1)
    sd = {k: v.clone() for k, v in mod.state_dict().items()}
    dx0, g0 = _module_grads(mod, x, gup, False)
    mod.load_state_dict(sd)
    dx1, g1 = _module_grads(mod, x, gup, True)
    assert _rel(dx1, dx0) < 3e-3, _rel(dx1, dx0)
    for k in g0:
        tol = 2e-3 if k.endswith('conv.weight') else 1e-3
        assert _rel(g1[k], g0[k]) < tol, (k, _rel(g1[k], g0[k]))
