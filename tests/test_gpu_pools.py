"""Kernel-level parity of the pooling kernels against ATen's CPU pooling (the reference's own ops):

* dmy_maxpool_fwd/bwd — nn.MaxPool2d(k, 1, k // 2) of SPPF (models/common.py:243-258), SPPFCSPC
  (:1257-1276) and SPP (:212-227, k = 3..13): pooled values and the argmax are bit-exact (inputs on a
  coarse grid so windows hold many ties; ATen keeps the first maximum in row-major window order),
  the gradient routes to the same pixel.  Both kernel forms run: the LDS-tiled separable one (16-B
  channel vectors) and the generic per-pixel one (channel counts that are not a vector multiple).
* dmy_gpool_fwd/bwd — AdaptiveAvgPool2d(1) / AdaptiveMaxPool2d(1) of CBAM's channel attention
  (common.py:270-271): max and argmax bit-exact (first maximum), mean to fp32 rounding, over pixel
  counts that split into many chunks.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _lib():
    from dmayolo.functional import call, ptr, stream
    return call, ptr, stream


def _grid_values(shape, gen, levels=7):
    # values on a coarse grid (exact in bf16): every window holds ties
    return torch.randint(-levels, levels + 1, shape, generator=gen).float() / 4


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
@pytest.mark.parametrize('k', [3, 5, 7, 9, 11, 13])
@pytest.mark.parametrize('N,C,H,W,extra', [(2, 16, 37, 53, 0), (1, 6, 19, 23, 0), (2, 8, 40, 33, 8)])
def test_maxpool_vs_aten(dtype, k, N, C, H, W, extra):
    call, ptr, stream = _lib()
    gen = torch.Generator().manual_seed(k * 100 + C)
    dt = 1 if dtype == torch.bfloat16 else 0
    xs = _grid_values((N, H, W, C + extra), gen)       # NHWC; `extra` leading channels -> pixel stride > C
    dy = torch.randn(N, H, W, C, generator=gen).to(dtype).float()
    xbuf = xs.to(dtype).cuda()
    x = xbuf[..., extra:]
    y = torch.empty(N, H, W, C, dtype=dtype, device='cuda')
    arg = torch.empty(N, H, W, C, dtype=torch.uint8, device='cuda')
    call('dmy_maxpool_fwd', dt, ptr(x), C + extra, ptr(y), C, ptr(arg), N, H, W, C, k, stream())
    dx = torch.empty(N, H, W, C, dtype=dtype, device='cuda')
    dyg = dy.to(dtype).cuda()
    call('dmy_maxpool_bwd', dt, ptr(dyg), C, ptr(arg), ptr(dx), C, 0, N, H, W, C, k, stream())
    torch.cuda.synchronize()

    xr = xs[..., extra:].permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    yr, ir = F.max_pool2d(xr, k, 1, k // 2, return_indices=True)
    yr.backward(dy.permute(0, 3, 1, 2))
    p = k // 2
    a = arg.long().cpu().permute(0, 3, 1, 2)
    oh = torch.arange(H).view(1, 1, H, 1)
    ow = torch.arange(W).view(1, 1, 1, W)
    flat = (oh - p + a // k) * W + (ow - p + a % k)
    assert torch.equal(y.float().cpu().permute(0, 3, 1, 2), yr.detach())
    assert torch.equal(flat, ir)
    ref_dx = xr.grad.permute(0, 2, 3, 1)
    if dtype == torch.float32:
        torch.testing.assert_close(dx.cpu(), ref_dx, rtol=1e-5, atol=1e-5)  # summation order only
    else:
        torch.testing.assert_close(dx.float().cpu(), ref_dx.to(dtype).float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
@pytest.mark.parametrize('k', [3, 5])
@pytest.mark.parametrize('N,C,H,W', [(1, 256, 20, 20), (2, 16, 37, 53), (1, 64, 48, 48), (2, 8, 5, 70), (2, 256, 45, 70)])
def test_maxpool_chain3_equals_three_launches(dtype, k, N, C, H, W):
    """the inference SPPF pyramid in one launch (dmy_maxpool_chain3_fwd) gives the bits of three chained
    dmy_maxpool_fwd launches, into three channel slices of one concat buffer, with signed zeros and NaNs among the
    ties (the update rule's order decides which zero survives)"""
    call, ptr, stream = _lib()
    gen = torch.Generator().manual_seed(k * 10 + C + H)
    dt = 1 if dtype == torch.bfloat16 else 0
    xs = _grid_values((N, H, W, C), gen)
    xs[xs == 0.25] = -0.0
    xs.view(-1)[torch.randint(0, xs.numel(), (3,), generator=gen)] = float('nan')
    x = xs.to(dtype).cuda()
    cat = torch.full((N, H, W, 4 * C), 7.0, dtype=dtype, device='cuda')
    call('dmy_maxpool_chain3_fwd', dt, ptr(x), C, ptr(cat[..., C:]), ptr(cat[..., 2 * C:]), ptr(cat[..., 3 * C:]),
         4 * C, N, H, W, C, k, stream())
    ref, cur = [], x
    arg = torch.empty(N, H, W, C, dtype=torch.uint8, device='cuda')
    for _ in range(3):
        y = torch.empty(N, H, W, C, dtype=dtype, device='cuda')
        call('dmy_maxpool_fwd', dt, ptr(cur), C, ptr(y), C, ptr(arg), N, H, W, C, k, stream())
        ref.append(y)
        cur = y
    torch.cuda.synchronize()
    iv = torch.int16 if dtype == torch.bfloat16 else torch.int32
    for i in range(3):
        assert torch.equal(cat[..., (i + 1) * C:(i + 2) * C].contiguous().view(iv), ref[i].view(iv)), i
    assert bool((cat[..., :C] == 7.0).all())  # the first slice is not touched


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
@pytest.mark.parametrize('N,C,H,W', [(2, 16, 120, 97), (3, 40, 9, 7), (1, 6, 64, 300), (2, 512, 30, 30)])
def test_gpool_vs_aten(dtype, N, C, H, W):
    call, ptr, stream = _lib()
    gen = torch.Generator().manual_seed(N * C + H)
    dt = 1 if dtype == torch.bfloat16 else 0
    xs = _grid_values((N, H, W, C), gen, levels=20)
    x = xs.to(dtype).cuda()
    out = torch.empty(2 * N, C, dtype=dtype, device='cuda')
    arg = torch.empty(N, C, dtype=torch.int32, device='cuda')
    ws = torch.empty(call('dmy_gpool_ws_bytes', dt, N, H * W, C) // 4, device='cuda')
    call('dmy_gpool_fwd', dt, ptr(x), C, N, H * W, C, ptr(out), ptr(arg), ptr(ws), stream())
    dz = torch.randn(2 * N, C, generator=gen).to(dtype)
    dx = torch.empty(N, H, W, C, dtype=dtype, device='cuda')
    dzg = dz.cuda()
    call('dmy_gpool_bwd', dt, ptr(dzg), ptr(arg), ptr(dx), C, 0, N, H * W, C, stream())
    torch.cuda.synchronize()

    xr = xs.permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    mean = F.adaptive_avg_pool2d(xr, 1).flatten(1)
    mx, idx = F.adaptive_max_pool2d(xr, 1, return_indices=True)
    (mean * dz[:N].float()).sum().backward(retain_graph=True)
    (mx.flatten(1) * dz[N:].float()).sum().backward()
    o = out.float().cpu()
    assert torch.equal(o[N:], mx.flatten(1).detach())
    assert torch.equal(arg.long().cpu(), idx.flatten(1))
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(o[:N], mean.detach().to(dtype).float(), rtol=tol, atol=tol)
    torch.testing.assert_close(dx.float().cpu(), xr.grad.permute(0, 2, 3, 1).to(dtype).float(), rtol=tol, atol=tol)


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
@pytest.mark.parametrize('M,C,acc', [(32 * 48 * 48, 256, 0), (3 * 37 * 41, 64, 1), (7, 16, 0)])
def test_slice_copy_dot_equals_two_launches(dtype, M, C, acc):
    """the BiFPN weighted-concat backward of one input in one pass (dmy_slice_copy_dot) gives the bits of
    dmy_slice_copy + dmy_dot_partial: the scaled (accumulated) gradient slice and (bf16 operands) every block partial
    of sum(dy * x)"""
    call, ptr, stream = _lib()
    gen = torch.Generator().manual_seed(M + C)
    dt = 1 if dtype == torch.bfloat16 else 0
    dyb = torch.randn(M, 3 * C, generator=gen).to(dtype).cuda()
    dy = dyb[:, C:2 * C]
    x = torch.randn(M, C, generator=gen).to(dtype).cuda()
    g0 = torch.randn(M, C, generator=gen).to(dtype).cuda()
    w = (torch.rand(3, generator=gen) + 0.5).cuda()
    nb = call('dmy_dot_partial_blocks', M, C)
    ga, gb = g0.clone(), g0.clone()
    pa, pb = torch.zeros(nb, device='cuda'), torch.zeros(nb, device='cuda')
    call('dmy_slice_copy_dot', dt, ptr(dy), 3 * C, ptr(ga), C, ptr(x), C, M, C, ptr(w), 1, 3, 1e-4, acc, ptr(pa), stream())
    call('dmy_slice_copy', dt, ptr(dy), 3 * C, ptr(gb), C, M, C, ptr(w), 1, 3, 1e-4, acc, stream())
    call('dmy_dot_partial', dt, ptr(dy), 3 * C, ptr(x), C, M, C, ptr(pb), stream())
    torch.cuda.synchronize()
    assert torch.equal(ga, gb)
    if dtype == torch.bfloat16:
        assert torch.equal(pa, pb)
    else:  # fp32: the two kernels' products may contract into FMAs differently (last-ulp partials)
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-4)
    ref = float((dy.double() * x.double()).sum())
    assert abs(float(pa.double().sum()) - ref) <= 1e-3 * max(1.0, abs(ref))
