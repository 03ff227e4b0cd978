"""GPU: the fp8 (OCP e4m3fn) forward conv of config 5 (BASELINE configs[4], "fp8 MFMA conv"; csrc/conv.hip
conv_fwd_f8 on v_mfma_scale_f32_16x16x128_f8f6f4).

* dmy_fp8_quant / dmy_conv_wprep_fp8 against torch's own float8_e4m3fn cast of the same scaled fp32 values
  (bit-exact: amax, per-channel weight scales and every byte);
* dmy_conv_fwd_fp8 against a float64 convolution of the DEQUANTISED operands (x8 * amax / 448, w8 * wscale):
  the kernel's only error sources are the fp32 accumulation and the bf16 output rounding, so the bound is the
  bf16 one (relative L2 < 4e-3), including the BN partial sums of the training epilogue and the fused inference
  epilogue (eval BN + SiLU + residual);
* the whole config-5 model with fp8 forward convs against its bf16 forward at a stated tolerance: e4m3 keeps 3
  mantissa bits (relative step 2^-3, i.e. +-6 % per element), averaged over C*k*k products per output and
  compounded over ~60 layers.  Bound (measured 2026-10, tools/gpu/fp8_model_err): per-level output relative L2 <
  0.15, cosine > 0.98, loss within 5 %.
"""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _e4m3(t):
    return t.clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)


def _quant(x_cl, C):
    from dmayolo.functional import call, ptr, stream, pixel_stride
    xs, xps = pixel_stride(x_cl)
    N, _, H, W = xs.shape
    x8 = torch.empty(N * H * W * C, dtype=torch.uint8, device='cuda')
    ws = torch.empty(call('dmy_fp8_quant_ws_elems'), device='cuda')
    call('dmy_fp8_quant', ptr(xs), N * H * W, C, xps, ptr(x8), ptr(ws), stream())
    return x8, ws[:1]


@pytest.mark.parametrize('slice_', [False, True])
def test_fp8_quant_matches_torch_cast(slice_):
    g = torch.Generator().manual_seed(3)
    N, C, H, W = 3, 128, 17, 23
    full = (torch.randn(N, 2 * C if slice_ else C, H, W, generator=g) * 3).bfloat16().cuda()
    full = full.contiguous(memory_format=torch.channels_last)
    x = full[:, C:] if slice_ else full  # a concat slice: pixel stride 2C
    x8, amax = _quant(x, C)
    torch.cuda.synchronize()
    xf = x.float().permute(0, 2, 3, 1).reshape(-1, C)
    a = xf.abs().max()
    assert float(amax) == float(a)
    ref = _e4m3(xf * (torch.tensor(448.0, device='cuda') / a)).reshape(-1)
    assert torch.equal(x8, ref)


@pytest.mark.parametrize('headroom', [1.0, 2.0])
def test_bn_act_f8_delayed_amax_headroom_and_saturation(headroom):
    """dmy_bn_act_fwd_f8 (delayed scaling): y = z * scale + shift in bf16, its e4m3 copy quantised with the PREVIOUS
    amax (max of the pmax block maxima) x headroom -- torch's cast of the same scaled values, every byte --, this
    call's block maxima in nmax, and per block the count of elements above that amax in nsat (the clipping
    of a range that grew since the last step is counted, not silent)."""
    from dmayolo.functional import call, ptr, stream
    g = torch.Generator().manual_seed(8)
    M, C = 5000, 64
    z = (torch.randn(M, C, generator=g) * 2).bfloat16().cuda()
    scale = (torch.rand(C, generator=g) + 0.5).cuda()
    shift = (torch.randn(C, generator=g) * 0.1).cuda()
    G = call('dmy_bn_act_f8_blocks')
    prev = 3.0  # last step's amax: smaller than this step's range, so some elements clip
    pmax = torch.zeros(G, device='cuda')
    pmax[7] = prev
    nmax, nsat = torch.full((G,), -1.0, device='cuda'), torch.full((G,), -1.0, device='cuda')
    used = torch.empty(1, device='cuda')
    y = torch.empty(M, C, dtype=torch.bfloat16, device='cuda')
    y8 = torch.empty(M * C, dtype=torch.uint8, device='cuda')
    call('dmy_bn_act_fwd_f8', ptr(z), C, ptr(scale), ptr(shift), 0, None, 0, ptr(y), C, M, C, ptr(y8),
         ptr(pmax), ptr(nmax), ptr(used), headroom, ptr(nsat), stream())
    torch.cuda.synchronize()
    # the kernel forms z * scale + shift as one fma: float64 reference, at most one bf16 ulp apart on rare ties
    yr = (z.double() * scale.double() + shift.double()).float().bfloat16()
    d = (y.float() - yr.float()).abs()
    assert float(d.max()) <= float(yr.float().abs().max()) * 2 ** -7 and int((d > 0).sum()) <= 1e-3 * y.numel()
    a = prev * headroom
    assert float(used) == a
    yf = y.float()  # the e4m3 copy quantises the stored bf16 values
    ref = _e4m3(yf * (torch.tensor(448.0, device='cuda') / torch.tensor(a, device='cuda'))).reshape(-1)
    assert torch.equal(y8, ref)
    assert float(nmax.max()) == float(yf.abs().max()) and float(nmax.min()) >= 0
    nclip = int((yf.abs() > a).sum())
    assert nclip > 0 if headroom == 1.0 else True
    assert float(nsat.sum()) == nclip and float(nsat.min()) >= 0
    # a sub-1 headroom is refused
    with pytest.raises(RuntimeError):
        call('dmy_bn_act_fwd_f8', ptr(z), C, ptr(scale), ptr(shift), 0, None, 0, ptr(y), C, M, C, ptr(y8),
             ptr(pmax), ptr(nmax), ptr(used), 0.5, None, stream())


def test_fp8_wprep_matches_torch_cast():
    from dmayolo.functional import call, ptr, stream
    g = torch.Generator().manual_seed(4)
    K, C, k = 40, 256, 3
    w = (torch.randn(K, C, k, k, generator=g) * torch.linspace(0.01, 2, K).view(K, 1, 1, 1)).cuda()
    w[5] = 0  # an all-zero output channel: scale 1, bytes 0
    w8 = torch.empty(w.numel(), dtype=torch.uint8, device='cuda')
    ws = torch.empty(K, device='cuda')
    call('dmy_conv_wprep_fp8', ptr(w), ptr(w8), ptr(ws), K, C, k, k, stream())
    torch.cuda.synchronize()
    am = w.abs().amax((1, 2, 3))
    # tensor / tensor: torch turns a division by a Python scalar into a multiply by its rounded reciprocal
    exp_s = torch.where(am > 0, am / torch.full_like(am, 448.0), torch.ones_like(am))
    assert torch.equal(ws, exp_s)
    inv = torch.where(am > 0, torch.tensor(448.0, device='cuda') / am, torch.ones_like(am))
    ref = _e4m3(w * inv.view(K, 1, 1, 1)).permute(0, 2, 3, 1).reshape(-1)  # OHWI
    assert torch.equal(w8, ref)


def _dequant(x8, amax, shape_nhwc):
    v = x8.view(torch.float8_e4m3fn).double().reshape(shape_nhwc)
    return (v * (float(amax) / 448.0)).permute(0, 3, 1, 2)


# (N, C, H, W, K, k, s): 3x3 s1 / s2, 1x1, K <= 64 tile, ragged M, several K steps per tap
SHAPES = [(2, 128, 40, 36, 128, 3, 1), (4, 256, 33, 29, 64, 3, 2), (3, 128, 50, 41, 256, 1, 1),
          (2, 384, 21, 27, 136, 3, 1), (5, 128, 64, 64, 40, 3, 1)]


@pytest.mark.parametrize('N,C,H,W,K,k,s', SHAPES)
def test_conv_fwd_fp8_vs_dequantised_reference(N, C, H, W, K, k, s):
    from dmayolo.functional import call, ptr, stream
    g = torch.Generator().manual_seed(N * 100 + C + K)
    p = k // 2
    x = torch.randn(N, C, H, W, generator=g).bfloat16().cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, k, k, generator=g) / (C * k * k) ** 0.5).cuda()
    bias = torch.randn(K, generator=g).cuda() * 0.1
    x8, amax = _quant(x, C)
    w8 = torch.empty(w.numel(), dtype=torch.uint8, device='cuda')
    ws = torch.empty(K, device='cuda')
    call('dmy_conv_wprep_fp8', ptr(w), ptr(w8), ptr(ws), K, C, k, k, stream())
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    M = N * OH * OW
    y = torch.empty(N, K, OH, OW, dtype=torch.bfloat16, device='cuda', memory_format=torch.channels_last)
    P = call('dmy_conv_fwd_fp8_partial_rows', M, K)
    ps = torch.full((P, K), float('nan'), device='cuda')
    pq = torch.full((P, K), float('nan'), device='cuda')
    call('dmy_conv_fwd_fp8', ptr(x8), ptr(w8), ptr(amax), ptr(ws), ptr(bias), ptr(y), ptr(ps), ptr(pq), N, H, W, C, K,
         k, k, s, p, OH, OW, K, None, None, 0, None, 0, stream())
    torch.cuda.synchronize()
    xd = _dequant(x8, amax, (N, H, W, C)).cpu()
    wd = (w8.view(torch.float8_e4m3fn).double().reshape(K, k, k, C).permute(0, 3, 1, 2) * ws.double().view(K, 1, 1, 1))
    ref = F.conv2d(xd, wd.cpu(), bias.double().cpu(), stride=s, padding=p)
    got = y.float().cpu()
    assert _rel(got, ref) < 4e-3, _rel(got, ref)
    assert float((got.double() - ref).abs().max()) <= float(ref.abs().max()) * 2 ** -7
    assert torch.isfinite(ps).all() and torch.isfinite(pq).all()
    s1, s2 = ref.sum((0, 2, 3)), (ref ** 2).sum((0, 2, 3))
    assert float((ps.sum(0).double().cpu() - s1).abs().max()) < 1e-3 * float(ref.abs().sum((0, 2, 3)).max())
    assert _rel(pq.sum(0).cpu(), s2) < 1e-3
    # quantisation itself: the fp8 product stays close to the unquantised bf16 operands' convolution
    full = F.conv2d(x.double().cpu(), w.double().cpu(), bias.double().cpu(), stride=s, padding=p)
    assert _rel(got, full) < 0.06


def test_conv_fwd_fp8_inference_epilogue():
    """eval BN scale / shift + SiLU + residual in the fp8 kernel's store loop == the unfused composition"""
    from dmayolo.functional import call, ptr, stream
    from dmayolo._lib import ACT_SILU
    g = torch.Generator().manual_seed(9)
    N, C, H, W, K = 2, 256, 30, 34, 128
    x = torch.randn(N, C, H, W, generator=g).bfloat16().cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5).cuda()
    sc, sh = (torch.rand(K, generator=g) + 0.5).cuda(), torch.randn(K, generator=g).cuda() * 0.2
    res = torch.randn(N, K, H, W, generator=g).bfloat16().cuda().contiguous(memory_format=torch.channels_last)
    x8, amax = _quant(x, C)
    w8 = torch.empty(w.numel(), dtype=torch.uint8, device='cuda')
    ws = torch.empty(K, device='cuda')
    call('dmy_conv_wprep_fp8', ptr(w), ptr(w8), ptr(ws), K, C, 3, 3, stream())
    z = torch.empty_like(res)
    y = torch.empty_like(res)
    args = (N, H, W, C, K, 3, 3, 1, 1, H, W, K)
    call('dmy_conv_fwd_fp8', ptr(x8), ptr(w8), ptr(amax), ptr(ws), None, ptr(z), None, None, *args, None, None, 0,
         None, 0, stream())
    call('dmy_conv_fwd_fp8', ptr(x8), ptr(w8), ptr(amax), ptr(ws), None, ptr(y), None, None, *args, ptr(sc), ptr(sh),
         ACT_SILU, ptr(res), K, stream())
    torch.cuda.synchronize()
    u = z.float() * sc.view(1, K, 1, 1) + sh.view(1, K, 1, 1)
    ref = F.silu(u) + res.float()
    assert _rel(y.float(), ref) < 6e-3


def _c5_outputs(fp8, seed=0):
    from dmayolo.models.yolo import Model
    from dmayolo.functional import set_fp8
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.synthetic import images, targets, HYP_SCRATCH, scaled_hyp
    torch.manual_seed(seed)
    m = Model(os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs', 'yolov5l-xs-tr-cbam-spp-bifpn.yaml'), nc=3,
              act_dtype=torch.bfloat16).cuda()
    m.hyp = scaled_hyp(HYP_SCRATCH, 3, 256)
    n = set_fp8(m, fp8) if fp8 else 0
    x, t = images(2, 256, device='cuda'), targets(2, 3, device='cuda')
    out = m(x)
    loss, items = ComputeLoss(m)(out, t)
    return [o.float() for o in out], float(loss), n


def test_config5_fp8_forward_close_to_bf16():
    ref, lref, _ = _c5_outputs(False)
    got, lgot, n = _c5_outputs(True)
    assert n >= 10
    for a, b in zip(got, ref):
        cos = float(F.cosine_similarity(a.reshape(1, -1).double(), b.reshape(1, -1).double()))
        print(f'level rel {_rel(a, b):.4f} cos {cos:.5f}')
        assert _rel(a, b) < 0.15 and cos > 0.98
    print(f'loss bf16 {lref:.5f} fp8 {lgot:.5f}')
    assert abs(lgot - lref) < 0.05 * abs(lref)


def test_fp8_delayed_scaling_equals_jit_on_repeated_batch():
    """Delayed scaling (functional.F8Emit): from the third train-mode forward on, each fp8 conv's producer emits the
    e4m3 copy of its output in its BN-act pass with the previous step's amax (dmy_bn_act_fwd_f8) instead of the two
    dmy_fp8_quant passes.  On a repeated batch with unchanged weights the previous amax IS the current one, so the
    outputs must equal the just-in-time quantisation bit for bit, and the quantisation passes must be gone."""
    import dmayolo.functional as Fn
    from dmayolo.models.yolo import Model
    from dmayolo.synthetic import images
    cfg = os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs', 'yolov5l-xs-tr-cbam-spp-bifpn.yaml')
    x = images(2, 256, device='cuda')

    def run(delayed):
        Fn.F8_DELAYED[0] = delayed
        torch.manual_seed(0)
        m = Model(cfg, nc=3, act_dtype=torch.bfloat16).cuda().train()
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
        assert Fn.set_fp8(m, True) >= 10
        counts = {}
        orig = Fn.call

        def counting(name, *a):
            counts[name] = counts.get(name, 0) + 1
            return orig(name, *a)
        with torch.no_grad():
            for i in range(3):
                if i == 2:
                    Fn.call = counting
                try:
                    out = m(x)
                finally:
                    Fn.call = orig
        return [o.float() for o in out], counts, Fn.f8_saturation(m)

    try:
        jit, cj, _ = run(False)
        dly, cd, sat = run(True)
    finally:
        Fn.F8_DELAYED[0] = True
    # the same batch again: no element exceeds the previous step's amax, so nothing saturated
    print('saturation', sat)
    assert len(sat) >= 8 and all(n == 0 for n, _ in sat.values())
    print('jit', {k: v for k, v in cj.items() if 'f8' in k or 'fp8' in k}, 'delayed',
          {k: v for k, v in cd.items() if 'f8' in k or 'fp8' in k})
    assert cd.get('dmy_bn_act_fwd_f8', 0) >= 8
    assert cd.get('dmy_fp8_quant', 0) <= cj['dmy_fp8_quant'] - cd['dmy_bn_act_fwd_f8']
    for a, b in zip(dly, jit):
        assert torch.equal(a, b)


def test_config5_fp8_step_vs_fp32_oracle():
    """BASELINE config 5's fp8 leg against the fp32 CPU oracle (full-width yolov5l-xs-tr-cbam-spp-bifpn @256, bs 2):
    the product with every eligible conv forward on the e4m3 kernel, and the oracle under the matching storage
    emulation (tests/precision_emu.py 'fp8': bf16 storage + e4m3 forward operands with the product's per-tensor /
    per-channel scales, bf16 backward).  Bounds on what the e4m3 kernel computes, the forward: Detect outputs relative
    L2 per level <= 1.1 * emu + 2e-3 and loss <= 1.1 * emu + 5e-3 (round 3, measured: product 2.43/3.39/1.48/6.54e-2 vs
    emu 2.28/3.36/1.50/6.48e-2).  The gradient metrics are bounded against the envelope of the emulation realizations
    (below), loosely: at random init this config's gradient is chaotic under ANY rounding (its CBAM channel maxima, SPP / SPPF argmaxes and global attention route on
    near-ties) -- the bf16 emulation alone has whole-gradient cosine -0.11 against fp32, the fp8 one 0.007 -- so no
    gradient bound separates a correct kernel from a wrong one here; the fp8 kernels' backward is bf16 and is pinned
    by the bf16 tests.  The bf16 emulation's numbers are printed beside them (the e4m3 forward's cost on top of bf16)."""
    import dmayolo.functional as Fn
    from dmayolo.models.yolo import Model
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.synthetic import images, targets, HYP_SCRATCH, scaled_hyp
    from precision_emu import oracle_run, grad_metrics
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs', 'yolov5l-xs-tr-cbam-spp-bifpn.yaml')
    nc, img, bs = 3, 256, 2
    torch.manual_seed(0)
    m = Model(cfg, nc=nc, act_dtype=torch.bfloat16)
    # anchors: 4 placeholders (range(8), one of zero width): pin real ones as bench.py does, from the label statistics
    m.model[-1].anchors[:] = torch.tensor([[10, 13], [16, 30], [33, 23], [30, 61]], dtype=torch.float32).view(1, 4, 2) \
        / m.model[-1].stride.view(-1, 1, 1) * torch.tensor([1.0, 2.0, 4.0, 8.0]).view(-1, 1, 1)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    hyp = scaled_hyp(HYP_SCRATCH, nc, img, m.model[-1].nl)
    m.hyp = hyp
    m = m.cuda().train()
    assert Fn.set_fp8(m, True) >= 10
    x, t = images(bs, img, seed=1), targets(bs, nc, per_image=20, seed=1)
    anchors = m.model[-1].anchors.cpu()
    p = m(x.cuda())
    loss, items = ComputeLoss(m)(p, t.cuda())
    loss.backward()
    runs = {mode: oracle_run(cfg, nc, sd, x, t, anchors, hyp, mode) for mode in (None, 'fp8', 'bf16')}
    runs['fp8_gpu'] = oracle_run(cfg, nc, sd, x, t, anchors, hyp, 'fp8', 'cuda')  # a second rounding realization
    ref, pr, lr_, _ = runs[None]
    rg = dict(ref.named_parameters())
    names = [k for k in rg if rg[k].grad is not None]

    def errs(outs, lo, params):
        o = [_rel(a.detach().float().cpu(), b.detach()) for a, b in zip(outs, pr)]
        gn, cos = grad_metrics(params, rg, names)
        return o, abs(float(lo) - float(lr_)) / abs(float(lr_)), gn, cos
    got = errs(p, loss, dict(m.named_parameters()))
    e8 = errs(runs['fp8'][1], runs['fp8'][2], dict(runs['fp8'][0].named_parameters()))
    e16 = errs(runs['bf16'][1], runs['bf16'][2], dict(runs['bf16'][0].named_parameters()))
    e8g = errs(runs['fp8_gpu'][1], runs['fp8_gpu'][2], dict(runs['fp8_gpu'][0].named_parameters()))
    f = lambda r: 'outputs %s loss %.2e grad-norm vector %.2e cos %.4f' % (['%.2e' % v for v in r[0]], r[1], r[2], r[3])  # noqa: E731
    print(f'config 5 fp8 product: {f(got)}\n  fp8 emulation: {f(e8)}\n  fp8 emulation, GPU fp32 order: {f(e8g)}\n'
          f'  bf16 emulation: {f(e16)}')
    for a, e in zip(got[0], e8[0]):
        assert a <= 1.1 * e + 2e-3, (got[0], e8[0])
    assert got[1] <= 1.1 * e8[1] + 5e-3, (got[1], e8[1])
    assert max(e8[0]) > 0 and all(a < 0.15 for a in got[0])  # the e4m3 forward really ran and stayed close
    # gradient bounds against the envelope of the emulation realizations (fp8 on CPU / GPU order, and bf16 -- the
    # backward IS bf16): round 3 measured the grad-norm vector at 0.327 (product) vs 0.082 (fp8 emu) vs 0.336 (bf16
    # emu), i.e. realization noise at random init; the training-run check of this leg is test_gpu_trajectory.py's
    # 'c5-fp8@256' case
    env_gn = max(e8[2], e8g[2], e16[2])
    assert got[2] <= 1.5 * env_gn + 2e-2, (got[2], e8[2], e8g[2], e16[2])
    assert got[3] >= min(e8[3], e8g[3], e16[3]) - 0.1, (got[3], e8[3], e8g[3], e16[3])
