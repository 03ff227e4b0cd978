"""GPU: the implicit-GEMM conv kernels (all tile paths: v2 64/128 tiles, the v3 LDS-DMA forward)
against a plain PyTorch fp32 convolution of the same bf16-rounded operands, including the BN
batch-statistic partials the forward epilogue emits and ragged M / K / C edges."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (N, C, H, W, K, k, s): small (v2 64-tiles), mid (v2 128-tiles), large (v3: M >= 16384, K >= 128)
SHAPES = [(2, 16, 20, 18, 24, 3, 1), (4, 64, 40, 40, 64, 3, 2), (8, 64, 40, 40, 128, 3, 1),
          (16, 128, 40, 40, 256, 1, 1), (16, 64, 64, 64, 128, 3, 2), (12, 96, 37, 45, 136, 3, 1),
          (9, 256, 48, 50, 384, 1, 1), (8, 8, 192, 192, 64, 6, 2), (8, 8, 192, 192, 128, 6, 2),
          (4, 40, 96, 70, 200, 3, 1),
          # narrow layers (K <= 64) on the LDS-DMA weight-grad tiles (BM 32/64 x BN 128/256), ragged K / columns
          (16, 32, 64, 64, 32, 3, 1), (4, 64, 80, 80, 64, 3, 1), (16, 256, 40, 40, 64, 1, 1),
          (8, 8, 192, 192, 32, 6, 2), (8, 136, 60, 50, 40, 1, 1), (8, 32, 96, 96, 64, 3, 2),
          # buffer-descriptor v3 loader (C % 64 == 0): ragged M and K, 3 K steps per tap, stride 2
          (11, 128, 37, 45, 200, 3, 1), (6, 192, 52, 60, 136, 3, 1), (4, 64, 130, 122, 256, 3, 2),
          # stride-2 data-grad on the buffer loader, one launch per parity class: odd sizes, 3 K steps per tap
          (12, 64, 75, 91, 128, 3, 2), (8, 128, 101, 99, 192, 3, 2),
          # wide 256 x 256 tiles (>= 256 GEMM columns, >= one block per CU): fwd + dgrad, and dgrad of a 1x1
          (16, 256, 64, 64, 256, 3, 1), (16, 512, 64, 64, 128, 1, 1), (17, 256, 61, 63, 264, 3, 1),
          # 512 x 128 tiles (65..128 GEMM columns, >= one block per CU), ragged M and columns
          (32, 128, 64, 64, 128, 3, 1), (33, 128, 65, 63, 104, 1, 1),
          # 1x1 streaming GEMM (conv_p1s, reduction 64 / 128 / 256): odd 64-row tile counts (zeroed pad partial row),
          # 32-column passes, the per-32-row partials of <= 64-column layers, several column groups
          (5, 128, 57, 63, 96, 1, 1), (6, 64, 55, 57, 64, 1, 1), (4, 256, 65, 67, 288, 1, 1), (5, 96, 57, 63, 128, 1, 1),
          (3, 64, 97, 89, 544, 1, 1), (5, 128, 57, 63, 288, 1, 1),
          # the 16-channel k3 view of the space-to-depth stem on the streaming GEMM's 3x3 gather (zero taps at the
          # borders, odd tile count, 32-column pass)
          (5, 16, 61, 67, 64, 3, 1), (8, 16, 64, 64, 32, 3, 1), (3, 16, 97, 99, 96, 3, 1),
          # 3x3 64 -> 64 halo kernel (whole 8 x 32 tiles, >= one tile per CU): one tile per block, two per block with
          # idle tail blocks, 8 tile rows per image
          (8, 64, 64, 128, 64, 3, 1), (10, 64, 64, 128, 64, 3, 1), (4, 64, 96, 256, 64, 3, 1)]


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-12))


@pytest.mark.parametrize('N,C,H,W,K,k,s', SHAPES)
def test_conv_fwd_bf16_vs_torch(N, C, H, W, K, k, s):
    from dmayolo.functional import call, ptr, stream, prep_weight
    g = torch.Generator().manual_seed(N * 1000 + C + K)
    p = k // 2 if k != 6 else 2
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    w = (torch.randn(K, C, k, k, generator=g) / (C * k * k) ** 0.5)
    ref = F.conv2d(x.float().cuda(), w.bfloat16().float().cuda(), stride=s, padding=p)
    OH, OW = ref.shape[2:]
    xd = x.cuda().contiguous(memory_format=torch.channels_last)
    wf, _ = prep_weight(w.cuda(), torch.bfloat16, False)
    y = torch.empty(N, K, OH, OW, dtype=torch.bfloat16, device='cuda', memory_format=torch.channels_last)
    M = N * OH * OW
    P = call('dmy_conv_fwd_bn_rows', 1, ptr(xd), ptr(wf), None, ptr(y), N, H, W, C, C, K, k, k, s, p, OH, OW, K)
    ps = torch.full((P, K), float('nan'), device='cuda')
    pq = torch.full((P, K), float('nan'), device='cuda')
    rc = call('dmy_conv_fwd', 1, ptr(xd), ptr(wf), None, ptr(y), ptr(ps), ptr(pq), N, H, W, C, C, K, k, k, s, p, OH,
              OW, K, stream())
    assert rc == 0
    torch.cuda.synchronize()
    assert _rel(y.float(), ref) < 1e-2
    assert torch.isfinite(ps).all() and torch.isfinite(pq).all(), 'every partial row must be written'
    s1 = ref.sum((0, 2, 3)).double()
    s2 = (ref.double() ** 2).sum((0, 2, 3))
    assert _rel(ps.sum(0), s1) < 1e-3 or float((ps.sum(0).double() - s1).abs().max()) < 1e-2 * M ** 0.5
    assert _rel(pq.sum(0), s2) < 1e-3


@pytest.mark.parametrize('N,C,H,W,K,k,s', SHAPES)
@pytest.mark.parametrize('acc', [0, 1])
def test_conv_dgrad_bf16_vs_torch(N, C, H, W, K, k, s, acc):
    """data gradient (v3 LDS-DMA for stride 1, v2 parity classes for stride 2), with accumulate."""
    from dmayolo.functional import call, ptr, stream, prep_weight
    if k == 6:
        pytest.skip('the 6x6 stem has no input gradient (image input)')
    g = torch.Generator().manual_seed(N * 1000 + C + K + 7)
    p = k // 2
    w = (torch.randn(K, C, k, k, generator=g) / (K * k * k) ** 0.5)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(N, K, OH, OW, generator=g).bfloat16()
    prev = torch.randn(N, C, H, W, generator=g).bfloat16()
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.bfloat16().float().cuda(), dy.float().cuda(), stride=s, padding=p)
    if acc:
        ref = ref + prev.float().cuda()
    _, wt = prep_weight(w.cuda(), torch.bfloat16, True)
    dyd = dy.cuda().contiguous(memory_format=torch.channels_last)
    dx = prev.cuda().contiguous(memory_format=torch.channels_last)
    rc = call('dmy_conv_dgrad', 1, ptr(dyd), ptr(wt), ptr(dx), acc, N, H, W, C, C, K, k, k, s, p, OH, OW, K, stream())
    assert rc == 0
    torch.cuda.synchronize()
    assert _rel(dx.float(), ref) < 1e-2


@pytest.mark.parametrize('N,H,W,K', [(4, 256, 256, 128), (3, 383, 257, 64), (10, 192, 160, 192)])
@pytest.mark.parametrize('acc', [0, 1])
@pytest.mark.parametrize('C', [32, 64, 128])
def test_conv_dgrad_s2_one_gemm_vs_torch(N, H, W, K, acc, C):
    """32- / 64- / 128-channel 3x3 stride-2 data-grad as one GEMM over dy pixels (conv_dgrad_q2 / _q2s: the 2 x 2 dy
    window against the parity classes' weights; 128 columns = four classes x 32 channels, 256 = four classes x 64, or
    one row class x two column classes x 128 channels per tile), taken when the grid has >= one 256-row tile per CU:
    even and odd maps (the a = 1 / b = 1 rows and columns past an odd edge are not stored), 64 / 128 / 192 dy channels,
    accumulate."""
    from dmayolo.functional import call, ptr, stream, prep_weight
    k, s, p = 3, 2, 1
    g = torch.Generator().manual_seed(N * 1000 + H + K)
    w = (torch.randn(K, C, k, k, generator=g) / (K * k * k) ** 0.5)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    assert N * OH * OW >= 256 * 256
    dy = torch.randn(N, K, OH, OW, generator=g).bfloat16()
    prev = torch.randn(N, C, H, W, generator=g).bfloat16()
    conv = torch.nn.grad.conv2d_input((N, C, H, W), w.bfloat16().float().cuda(), dy.float().cuda(), stride=s, padding=p)
    ref = conv + prev.float().cuda() if acc else conv
    _, wt = prep_weight(w.cuda(), torch.bfloat16, True)
    dyd = dy.cuda().contiguous(memory_format=torch.channels_last)
    dx = prev.cuda().contiguous(memory_format=torch.channels_last)
    rc = call('dmy_conv_dgrad', 1, ptr(dyd), ptr(wt), ptr(dx), acc, N, H, W, C, C, K, k, k, s, p, OH, OW, K, stream())
    assert rc == 0
    torch.cuda.synchronize()
    assert _rel(dx.float(), ref) < 1e-2
    # every pixel and channel, not just the norm: within the bf16 roundings of the stored result (the conv output,
    # and with accumulate the sum with the previous dx as well), so relative to |conv| (+ |prev|)
    scale = conv.abs() + (prev.float().cuda().abs() if acc else 0) + 1e-2
    err = (dx.float() - ref).abs() / scale
    assert float(err.max()) < 1.6e-2


@pytest.mark.parametrize('N,C,H,W,K,k,s', SHAPES)
def test_conv_wgrad_bf16_vs_torch(N, C, H, W, K, k, s):
    """weight gradient (v3 LDS-DMA split-K for wide layers, v2 otherwise), fp32 accumulation."""
    from dmayolo.functional import call, ptr, stream
    g = torch.Generator().manual_seed(N * 1000 + C + K + 11)
    p = k // 2 if k != 6 else 2
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    dy = torch.randn(N, K, OH, OW, generator=g).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float().cuda(), (K, C, k, k), dy.float().cuda(), stride=s, padding=p)
    xd = x.cuda().contiguous(memory_format=torch.channels_last)
    dyd = dy.cuda().contiguous(memory_format=torch.channels_last)
    dwo = torch.empty(K * C * k * k, device='cuda')
    dw = torch.empty(K, C, k, k, device='cuda')
    rc = call('dmy_conv_wgrad', 1, ptr(xd), ptr(dyd), ptr(dwo), N, H, W, C, C, K, k, k, s, p, OH, OW, K, stream())
    assert rc == 0
    call('dmy_conv_wgrad_to_oihw', ptr(dwo), ptr(dw), K, C, C, k, k, stream())
    torch.cuda.synchronize()
    assert _rel(dw, ref) < 2e-3


# small-M forward (batch-1 inference) on the split-K path: (N, C, H, W, K, k, s); 1x1 layers stay unsplit by default
SPLIT_SHAPES = [(1, 512, 48, 48, 512, 3, 1), (1, 256, 96, 96, 256, 3, 1), (1, 1024, 24, 24, 512, 3, 2),
                (1, 128, 40, 40, 64, 3, 1), (2, 192, 30, 34, 136, 3, 1)]


@pytest.mark.parametrize('N,C,H,W,K,k,s', SPLIT_SHAPES)
@pytest.mark.parametrize('epi', [False, True])
def test_conv_fwd_splitk_vs_torch(N, C, H, W, K, k, s, epi):
    from dmayolo.functional import call, ptr, stream, prep_weight
    from dmayolo._lib import ACT_SILU
    g = torch.Generator().manual_seed(N * 7 + C + K + k)
    p = k // 2
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    w = torch.randn(K, C, k, k, generator=g) / (C * k * k) ** 0.5
    b = torch.randn(K, generator=g) * 0.1
    ref = F.conv2d(x.float().cuda(), w.bfloat16().float().cuda(), b.cuda(), stride=s, padding=p)
    OH, OW = ref.shape[2:]
    xd = x.cuda().contiguous(memory_format=torch.channels_last)
    wf, _ = prep_weight(w.cuda(), torch.bfloat16, False)
    y = torch.empty(N, K, OH, OW, dtype=torch.bfloat16, device='cuda', memory_format=torch.channels_last)
    geo = (N, H, W, C, C, K, k, k, s, p, OH, OW, K)
    ne = call('dmy_conv_fwd_splitk_elems', 1, ptr(xd), ptr(wf), ptr(y), *geo)
    assert ne > 0, 'these shapes must take the split-K path'
    ws = torch.empty(ne, device='cuda')
    sc = (torch.rand(K, generator=g) + 0.5).cuda() if epi else None
    sh = (torch.randn(K, generator=g) * 0.2).cuda() if epi else None
    res = torch.randn(N, K, OH, OW, generator=g).bfloat16().cuda().contiguous(memory_format=torch.channels_last) \
        if epi else None
    call('dmy_conv_fwd_act_ws', 1, ptr(xd), ptr(wf), ptr(b.cuda()), ptr(y), *geo, ptr(sc), ptr(sh),
         ACT_SILU if epi else 0, ptr(res), K if epi else 0, ptr(ws), ne, stream())
    torch.cuda.synchronize()
    if epi:
        z = ref.bfloat16().float()  # the epilogue acts on the bf16-rounded conv output
        ref = F.silu(z * sc.view(1, K, 1, 1) + sh.view(1, K, 1, 1)) + res.float()
    assert _rel(y.float(), ref) < 1e-2
    # the split slabs are summed in split order: 20 launches on a NaN-filled workspace give the same bits every time
    first = y.clone()
    for i in range(20):
        ws.fill_(float('nan'))  # a reducer that read a slab before its producer's stores were visible would show NaN
        call('dmy_conv_fwd_act_ws', 1, ptr(xd), ptr(wf), ptr(b.cuda()), ptr(y), *geo, ptr(sc), ptr(sh),
             ACT_SILU if epi else 0, ptr(res), K if epi else 0, ptr(ws), ne, stream())
        assert torch.equal(y, first), i


@pytest.mark.parametrize('N,C,H,W,K', [(16, 64, 160, 160, 64), (16, 64, 150, 146, 48), (10, 128, 128, 136, 32),
                                       (16, 128, 100, 104, 128), (8, 256, 96, 96, 256), (10, 128, 96, 96, 192),
                                       (8, 16, 288, 288, 64), (8, 16, 290, 282, 32)])
def test_conv_wgrad_tap_two_planes_vs_torch(N, C, H, W, K):
    """3x3 s1 weight-grad on the tap-fused kernel against torch's fp32 conv2d_weight: two halo planes (64 input channels
    per block) for <= 64 output channels with C % 64 == 0, one plane otherwise (the 128-row tile, C % 64 != 0).  C = 16
    is the space-to-depth stem's view (half a plane, the rest loads zeros)"""
    from dmayolo.functional import call, ptr, stream
    g = torch.Generator().manual_seed(N + C + K + H)
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    dy = torch.randn(N, K, H, W, generator=g).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float().cuda(), (K, C, 3, 3), dy.float().cuda(), stride=1, padding=1)
    xd = x.cuda().contiguous(memory_format=torch.channels_last)
    dyd = dy.cuda().contiguous(memory_format=torch.channels_last)
    dwo = torch.empty(K * C * 9, device='cuda')
    dw = torch.empty(K, C, 3, 3, device='cuda')
    assert call('dmy_conv_wgrad', 1, ptr(xd), ptr(dyd), ptr(dwo), N, H, W, C, C, K, 3, 3, 1, 1, H, W, K, stream()) == 0
    call('dmy_conv_wgrad_to_oihw', ptr(dwo), ptr(dw), K, C, C, 3, 3, stream())
    torch.cuda.synchronize()
    assert _rel(dw, ref) < 2e-3, _rel(dw, ref)


def test_conv_fwd_1x1_small_m_unsplit():
    from dmayolo.functional import call, ptr
    x = torch.empty(1, 256, 96, 96, dtype=torch.bfloat16, device='cuda', memory_format=torch.channels_last)
    w = torch.empty(256, 256, dtype=torch.bfloat16, device='cuda')
    y = torch.empty_like(x)
    assert call('dmy_conv_fwd_splitk_elems', 1, ptr(x), ptr(w), ptr(y), 1, 96, 96, 256, 256, 256, 1, 1, 1, 0, 96, 96,
                256) == 0


# eval forwards (dmy_conv_fwd_act) whose 256-row tile grid leaves CUs idle (the v2 tiles, split-K, halo), ragged M /
# columns, a residual, a concat-slice output
FILL_SHAPES = [(1, 256, 96, 96, 256, 1, 1), (1, 128, 192, 192, 128, 1, 1), (1, 128, 190, 186, 128, 3, 1),
               (1, 512, 48, 48, 512, 1, 1), (1, 1024, 37, 41, 200, 1, 1), (2, 64, 45, 47, 136, 1, 1),
               (1, 256, 96, 96, 1024, 1, 1), (3, 128, 65, 67, 512, 3, 2),
               # output-heavy 1x1 eval forwards (M >= 16384, K >= 2C): 64-column tiles, a 32-column tail, a residual
               (1, 128, 192, 192, 512, 1, 1), (2, 64, 130, 126, 128, 1, 1), (1, 256, 128, 130, 544, 1, 1)]


@pytest.mark.parametrize('N,C,H,W,K,k,s', FILL_SHAPES)
@pytest.mark.parametrize('res', [False, True])
def test_conv_fwd_fill_tiles_vs_torch(N, C, H, W, K, k, s, res):
    from dmayolo.functional import call, ptr, stream, prep_weight
    from dmayolo._lib import ACT_SILU
    g = torch.Generator().manual_seed(N * 13 + C + K + k + int(res))
    p = k // 2
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    w = torch.randn(K, C, k, k, generator=g) / (C * k * k) ** 0.5
    ref = F.conv2d(x.float().cuda(), w.bfloat16().float().cuda(), stride=s, padding=p)
    OH, OW = ref.shape[2:]
    xd = x.cuda().contiguous(memory_format=torch.channels_last)
    wf, _ = prep_weight(w.cuda(), torch.bfloat16, False)
    Kt = K + 64  # output written into the first K channels of a wider (concat) buffer
    yb = torch.full((N, Kt, OH, OW), 7.0, dtype=torch.bfloat16, device='cuda').contiguous(
        memory_format=torch.channels_last)
    y = yb[:, :K]
    sc = (torch.rand(K, generator=g) + 0.5).cuda()
    sh = (torch.randn(K, generator=g) * 0.2).cuda()
    r = torch.randn(N, K, OH, OW, generator=g).bfloat16().cuda().contiguous(memory_format=torch.channels_last) \
        if res else None
    rc = call('dmy_conv_fwd_act', 1, ptr(xd), ptr(wf), None, ptr(y), N, H, W, C, C, K, k, k, s, p, OH, OW, Kt, ptr(sc),
              ptr(sh), ACT_SILU, ptr(r), K if res else 0, stream())
    assert rc == 0
    torch.cuda.synchronize()
    z = F.silu(ref.bfloat16().float() * sc.view(1, K, 1, 1) + sh.view(1, K, 1, 1))
    if res:
        z = z + r.float()
    assert _rel(y.float(), z) < 1e-2
    assert torch.equal(yb[:, K:].float().cpu(), torch.full((N, 64, OH, OW), 7.0)), 'columns past K must stay untouched'


# small-M eval forwards (batch-1 detect shapes, the inference routes): 1x1 and 3x3 stride 1 / 2, channel tiles past K,
# C % 64 != 0, M not a multiple of 64, bias + eval-BN + SiLU + residual, output into a concat-buffer slice
SK_SHAPES = [(1, 256, 96, 96, 256, 1, 1, True), (1, 1024, 48, 48, 1024, 1, 1, False), (1, 64, 97, 95, 64, 3, 1, True),
             (1, 128, 61, 59, 256, 3, 2, False), (2, 96, 33, 35, 96, 3, 1, True), (1, 32, 70, 66, 32, 1, 1, False),
             (1, 512, 24, 26, 160, 3, 1, True), (3, 192, 21, 23, 352, 1, 1, True), (1, 2048, 12, 12, 512, 1, 1, False)]


@pytest.mark.parametrize('N,C,H,W,K,k,s,res', SK_SHAPES)
def test_conv_fwd_small_m_eval_vs_torch(N, C, H, W, K, k, s, res):
    from dmayolo.functional import call, ptr, stream, prep_weight
    from dmayolo._lib import ACT_SILU
    g = torch.Generator().manual_seed(N * 31 + C + 3 * K + k + int(res))
    p = k // 2
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    w = torch.randn(K, C, k, k, generator=g) / (C * k * k) ** 0.5
    b = torch.randn(K, generator=g) * 0.1
    ref = F.conv2d(x.float().cuda(), w.bfloat16().float().cuda(), b.cuda(), stride=s, padding=p)
    OH, OW = ref.shape[2:]
    xd = x.cuda().contiguous(memory_format=torch.channels_last)
    wf, _ = prep_weight(w.cuda(), torch.bfloat16, False)
    Kt = K + 32
    yb = torch.full((N, Kt, OH, OW), 7.0, dtype=torch.bfloat16, device='cuda').contiguous(
        memory_format=torch.channels_last)
    y = yb[:, :K]
    sc = (torch.rand(K, generator=g) + 0.5).cuda()
    sh = (torch.randn(K, generator=g) * 0.2).cuda()
    r = torch.randn(N, K, OH, OW, generator=g).bfloat16().cuda().contiguous(memory_format=torch.channels_last) \
        if res else None
    rc = call('dmy_conv_fwd_act', 1, ptr(xd), ptr(wf), ptr(b.cuda()), ptr(y), N, H, W, C, C, K, k, k, s, p, OH, OW, Kt,
              ptr(sc), ptr(sh), ACT_SILU, ptr(r), K if res else 0, stream())
    assert rc == 0
    torch.cuda.synchronize()
    z = F.silu(ref.bfloat16().float() * sc.view(1, K, 1, 1) + sh.view(1, K, 1, 1))
    if res:
        z = z + r.float()
    assert _rel(y.float(), z) < 1e-2
    # elementwise: within 2 bf16 ulps of the reference almost everywhere (fp32 sums in another order)
    bad = ((y.float() - z).abs() > 2 ** -6 * z.abs() + 1e-2).float().mean().item()
    assert bad < 1e-3, bad
    assert torch.equal(yb[:, K:].float().cpu(), torch.full((N, 32, OH, OW), 7.0)), 'columns past K must stay untouched'


@pytest.mark.parametrize('DG', [False, True])
def test_halo_conv_strided_views(DG):
    """3x3 64 -> 64 halo kernel reading / writing channel slices of wider NHWC buffers (pixel strides 96 / 80), with
    the per-wave BN partial rows dmy_conv_fwd_bn_rows reports (forward) and the data-grad tap flip"""
    from dmayolo.functional import call, ptr, stream, prep_weight
    N, C, H, W, K = 8, 64, 64, 128, 64
    g = torch.Generator().manual_seed(77 + DG)
    xb = torch.randn(N, 96, H, W, generator=g).bfloat16().cuda().contiguous(memory_format=torch.channels_last)
    yb = torch.zeros(N, 80, H, W, dtype=torch.bfloat16, device='cuda').contiguous(memory_format=torch.channels_last)
    x, y = xb[:, 16:80], yb[:, 8:72]
    w = (torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5).cuda()
    wf, wt = prep_weight(w, torch.bfloat16, True)
    if not DG:
        ref = F.conv2d(x.float(), w.bfloat16().float(), padding=1)
        P = call('dmy_conv_fwd_bn_rows', 1, ptr(x), ptr(wf), None, ptr(y), N, H, W, C, 96, K, 3, 3, 1, 1, H, W, 80)
        assert P == 8 * 256 or P < 2 * N * H * W // 64, P
        ps = torch.full((P, K), float('nan'), device='cuda')
        pq = torch.full((P, K), float('nan'), device='cuda')
        rc = call('dmy_conv_fwd', 1, ptr(x), ptr(wf), None, ptr(y), ptr(ps), ptr(pq), N, H, W, C, 96, K, 3, 3, 1, 1, H,
                  W, 80, stream())
    else:
        ref = torch.nn.grad.conv2d_input((N, C, H, W), w.bfloat16().float(), x.float(), padding=1)
        rc = call('dmy_conv_dgrad', 1, ptr(x), ptr(wt), ptr(y), 0, N, H, W, C, 80, K, 3, 3, 1, 1, H, W, 96, stream())
    assert rc == 0
    torch.cuda.synchronize()
    assert _rel(y.float(), ref) < 1e-2
    assert float(yb[:, :8].float().abs().max()) == 0 and float(yb[:, 72:].float().abs().max()) == 0, 'slice overrun'
    if not DG:
        assert torch.isfinite(ps).all() and torch.isfinite(pq).all(), 'every partial row must be written'
        s1 = ref.sum((0, 2, 3)).double()
        assert float((ps.sum(0).double() - s1).abs().max()) < 1e-2 * (N * H * W) ** 0.5
        assert _rel(pq.sum(0), (ref.double() ** 2).sum((0, 2, 3))) < 1e-3


@pytest.mark.parametrize('res', [False, True])
def test_halo_conv_inference_epilogue(res):
    """batch-1 eval forward of a 3x3 64 -> 64 layer on the halo kernel's epilogue instantiation (eval BN scale / shift
    + SiLU (+ residual) on the bf16-rounded conv output), reading and writing channel slices of wider buffers"""
    from dmayolo.functional import call, ptr, stream, prep_weight
    from dmayolo._lib import ACT_SILU
    N, C, H, W, K = 1, 64, 384, 384, 64
    g = torch.Generator().manual_seed(91 + res)
    xb = torch.randn(N, 96, H, W, generator=g).bfloat16().cuda().contiguous(memory_format=torch.channels_last)
    yb = torch.full((N, 80, H, W), 7.0, dtype=torch.bfloat16, device='cuda').contiguous(
        memory_format=torch.channels_last)
    x, y = xb[:, 16:80], yb[:, 8:72]
    w = (torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5).cuda()
    wf, _ = prep_weight(w, torch.bfloat16, False)
    sc = (torch.rand(K, generator=g) + 0.5).cuda()
    sh = (torch.randn(K, generator=g) * 0.2).cuda()
    rb = torch.randn(N, 72, H, W, generator=g).bfloat16().cuda().contiguous(memory_format=torch.channels_last)
    r = rb[:, 8:] if res else None
    rc = call('dmy_conv_fwd_act', 1, ptr(x), ptr(wf), None, ptr(y), N, H, W, C, 96, K, 3, 3, 1, 1, H, W, 80, ptr(sc),
              ptr(sh), ACT_SILU, ptr(r), 72 if res else 0, stream())
    assert rc == 0
    torch.cuda.synchronize()
    ref = F.conv2d(x.float(), w.bfloat16().float(), padding=1)
    z = F.silu(ref.bfloat16().float() * sc.view(1, K, 1, 1) + sh.view(1, K, 1, 1))
    if res:
        z = z + r.float()
    assert _rel(y.float(), z) < 1e-2
    bad = ((y.float() - z).abs() > 2 ** -6 * z.abs() + 1e-2).float().mean().item()
    assert bad < 1e-3, bad
    assert float((yb[:, :8].float() - 7).abs().max()) == 0 and float((yb[:, 72:].float() - 7).abs().max()) == 0, \
        'slice overrun'



def test_wprep_multi_matches_permutes():
    """dmy_conv_wprep_multi (one launch for a model's weights; 32 x 32 x taps LDS tiles, elementwise for > 9 taps):
    the OHWI and IHWO bf16 copies equal torch's permute + cast of the fp32 OIHW masters, ragged K / C included"""
    from dmayolo.functional import WeightPrep
    g = torch.Generator().manual_seed(5)
    shapes = [(64, 32, 1, 1), (45, 70, 1, 1), (100, 36, 3, 3), (128, 256, 3, 3), (33, 17, 3, 3), (64, 3, 6, 6),
              (1024, 512, 1, 1)]
    ws = [torch.randn(s, generator=g).cuda() for s in shapes]
    wp = WeightPrep(ws, torch.bfloat16, torch.device('cuda')).launch()
    torch.cuda.synchronize()
    for w in ws:
        wf, wt = wp.get(w, torch.bfloat16)
        K, C, KH, KW = w.shape
        assert torch.equal(wf.view(K, KH, KW, C), w.permute(0, 2, 3, 1).bfloat16())
        assert torch.equal(wt.view(C, KH, KW, K), w.permute(1, 2, 3, 0).bfloat16())
