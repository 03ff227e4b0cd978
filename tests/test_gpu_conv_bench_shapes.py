"""GPU: every conv layer shape of the two bench configurations at the bench's own M (so the kernels take the tile /
persistent / halo / split-K plans the training step takes), against a plain PyTorch fp32 convolution of the same
bf16-rounded operands.  VERDICT r3 item 1: the product's per-tensor gradient norms sat 1.9-2.4x further from the fp32
oracle than the bf16-storage emulation's; a kernel that dropped or double-counted a split-K chunk, a parity class or a
partial tile at these M would show here as a NORM error (a bias), which bf16 rounding noise does not produce.

Per (layer shape, kind) the test measures the relative L2 error and the norm ratio |y| / |y_ref| - 1:
  forward / data-grad (bf16 output): rel L2 <= 2.5e-3 -- one round-to-nearest of each output to bf16 is 2^-8 / sqrt(12)
                                     = 1.13e-3 of ulp-relative, 1.66e-3 of rms for these Gaussian outputs, which is what
                                     every shape measures (round 4, gpurun_out r4/diag_tests.log) -- and
                                     |norm ratio - 1| <= 5e-5 (measured <= 3.8e-6: unbiased rounding)
  weight-grad (fp32 accumulation):   rel L2 <= 5e-5 (measured <= 5.6e-6), |norm ratio - 1| <= 1e-6 (measured 7e-8)
  forward BN partials:               sum / sum of squares per channel within 1e-6 relative (measured 1.8e-8; sum: or
                                     1e-2 sqrt(M) absolute)
A split-K chunk, a parity class or a tile dropped or counted twice moves these by orders of magnitude.
The shape lists are the unique (N, C, H, W, K, k, s) of profiles/r03/*_launches.csv (yolov5s @640 bs64, DMA-YOLO-l @1536
bs32) minus the 6x6 image stems, which the model runs as the space-to-depth k3 view (test_gpu_model.py covers it).
1x1 weight-grads go through dmy_conv_wgrad_ex with the OIHW | ZEROED flags the training step uses (arena slices)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

V5S = [(64, 32, 160, 160, 32, 1, 1), (64, 32, 160, 160, 32, 3, 1), (64, 32, 320, 320, 64, 3, 2),
       (64, 64, 80, 80, 64, 1, 1), (64, 64, 80, 80, 64, 3, 1), (64, 64, 160, 160, 32, 1, 1), (64, 64, 160, 160, 64, 1, 1),
       (64, 64, 160, 160, 128, 3, 2), (64, 128, 40, 40, 128, 1, 1), (64, 128, 40, 40, 128, 3, 1),
       (64, 128, 80, 80, 45, 1, 1), (64, 128, 80, 80, 64, 1, 1), (64, 128, 80, 80, 128, 1, 1),
       (64, 128, 80, 80, 128, 3, 2), (64, 128, 80, 80, 256, 3, 2), (64, 256, 20, 20, 256, 1, 1),
       (64, 256, 20, 20, 256, 3, 1), (64, 256, 40, 40, 45, 1, 1), (64, 256, 40, 40, 128, 1, 1),
       (64, 256, 40, 40, 256, 1, 1), (64, 256, 40, 40, 256, 3, 2), (64, 256, 40, 40, 512, 3, 2),
       (64, 256, 80, 80, 64, 1, 1), (64, 512, 20, 20, 45, 1, 1), (64, 512, 20, 20, 256, 1, 1),
       (64, 512, 20, 20, 512, 1, 1), (64, 512, 40, 40, 128, 1, 1), (64, 1024, 20, 20, 512, 1, 1)]

DMA = [(32, 64, 192, 192, 64, 3, 1), (32, 64, 384, 384, 64, 1, 1), (32, 64, 384, 384, 64, 3, 1),
       (32, 64, 768, 768, 64, 3, 1), (32, 64, 768, 768, 128, 3, 2), (32, 128, 96, 96, 128, 3, 1),
       (32, 128, 192, 192, 128, 1, 1), (32, 128, 192, 192, 128, 3, 1), (32, 128, 192, 192, 384, 1, 1),
       (32, 128, 192, 192, 512, 1, 1), (32, 128, 384, 384, 64, 1, 1), (32, 128, 384, 384, 128, 1, 1),
       (32, 128, 384, 384, 128, 3, 1), (32, 128, 384, 384, 256, 3, 2), (32, 256, 48, 48, 256, 3, 1),
       (32, 256, 96, 96, 256, 1, 1), (32, 256, 96, 96, 256, 3, 1), (32, 256, 96, 96, 768, 1, 1),
       (32, 256, 96, 96, 1024, 1, 1), (32, 256, 192, 192, 45, 1, 1), (32, 256, 192, 192, 128, 1, 1),
       (32, 256, 192, 192, 256, 1, 1), (32, 256, 192, 192, 256, 3, 1), (32, 256, 192, 192, 256, 3, 2),
       (32, 256, 192, 192, 512, 3, 2), (32, 512, 24, 24, 512, 3, 1), (32, 512, 48, 48, 512, 1, 1),
       (32, 512, 48, 48, 512, 3, 1), (32, 512, 48, 48, 1536, 1, 1), (32, 512, 48, 48, 2048, 1, 1),
       (32, 512, 96, 96, 45, 1, 1), (32, 512, 96, 96, 256, 1, 1), (32, 512, 96, 96, 512, 1, 1),
       (32, 512, 96, 96, 512, 3, 1), (32, 512, 96, 96, 512, 3, 2), (32, 512, 96, 96, 1024, 3, 2),
       (32, 512, 192, 192, 128, 1, 1), (32, 1024, 48, 48, 45, 1, 1), (32, 1024, 48, 48, 512, 1, 1),
       (32, 1024, 48, 48, 1024, 1, 1), (32, 1024, 48, 48, 1024, 3, 1), (32, 1024, 96, 96, 256, 1, 1),
       (32, 1280, 96, 96, 256, 1, 1), (32, 1536, 48, 48, 512, 1, 1), (32, 2048, 48, 48, 512, 1, 1),
       (32, 2048, 48, 48, 1024, 1, 1), (32, 4096, 48, 48, 1024, 1, 1)]


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _nr(a, b):
    return float(a.double().norm() / b.double().norm().clamp_min(1e-30)) - 1.0


def _ref_convs(x, dy, wb, k, s, p):
    """fp32 reference forward / data-grad / weight-grad from im2col (F.unfold / F.fold) + fp32 GEMMs, in image chunks
    (bounded memory; TF32 off): no per-shape kernel compilation, unlike the library convolutions at these sizes"""
    N, C, H, W = x.shape
    K = wb.shape[0]
    OH, OW = dy.shape[2:]
    w2 = wb.reshape(K, C * k * k)
    y = torch.empty(N, K, OH, OW, device=x.device)
    dx = torch.empty(N, C, H, W, device=x.device)
    dw = torch.zeros(K, C * k * k, device=x.device, dtype=torch.float64)
    nb = max(1, int(2e9 // (C * k * k * OH * OW)))
    for b0 in range(0, N, nb):
        xb = x[b0:b0 + nb].float()
        cols = F.unfold(xb, k, padding=p, stride=s) if k > 1 else xb.reshape(xb.shape[0], C, -1)  # [n, C k k, L]
        y[b0:b0 + nb] = torch.matmul(w2, cols).view(-1, K, OH, OW)
        dyb = dy[b0:b0 + nb].float().reshape(-1, K, OH * OW)
        dw += torch.matmul(dyb, cols.transpose(1, 2)).sum(0).double()
        dcols = torch.matmul(w2.t(), dyb)
        dx[b0:b0 + nb] = F.fold(dcols, (H, W), k, padding=p, stride=s) if k > 1 else dcols.view(-1, C, H, W)
        del cols, dcols
    return y, dx, dw.float().view(K, C, k, k)


def _check_shape(N, C, H, W, K, k, s, seed):
    from dmayolo.functional import call, ptr, stream, prep_weight
    dev = 'cuda'
    g = torch.Generator(device=dev).manual_seed(seed)
    p = k // 2
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    M = N * OH * OW
    x = torch.randn(N, C, H, W, generator=g, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, OH, OW, generator=g, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, k, k, generator=g, device=dev) / (C * k * k) ** 0.5
    wf, wt = prep_weight(w, torch.bfloat16, True)
    ry, rdx, rdw = _ref_convs(x, dy, w.bfloat16().float(), k, s, p)
    out = {}
    # forward with the train-mode BN partials
    y = torch.empty(N, K, OH, OW, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    P = call('dmy_conv_fwd_bn_rows', 1, ptr(x), ptr(wf), None, ptr(y), N, H, W, C, C, K, k, k, s, p, OH, OW, K)
    ps = torch.full((P, K), float('nan'), device=dev)
    pq = torch.full((P, K), float('nan'), device=dev)
    assert call('dmy_conv_fwd', 1, ptr(x), ptr(wf), None, ptr(y), ptr(ps), ptr(pq), N, H, W, C, C, K, k, k, s, p, OH,
                OW, K, stream()) == 0
    # the rows the launch reports writing (what the product passes to the finalize) = the prediction, and fit the bound
    assert call('dmy_conv_fwd_last_rows') == P <= call('dmy_conv_fwd_bound_rows', M, K)
    out['fwd'] = (_rel(y.float(), ry), _nr(y.float(), ry))
    s1 = ry.double().sum((0, 2, 3))
    s2 = (ry.double() ** 2).sum((0, 2, 3))
    psd = ps.double().sum(0)
    out['bn'] = (max(_rel(psd, s1) if float((psd - s1).abs().max()) > 1e-2 * M ** 0.5 else 0.0,
                     _rel(pq.double().sum(0), s2)), float(torch.isfinite(ps).all() and torch.isfinite(pq).all()) - 1)
    del ry, y, ps, pq
    # data gradient
    dx = torch.empty(N, C, H, W, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    assert call('dmy_conv_dgrad', 1, ptr(dy), ptr(wt), ptr(dx), 0, N, H, W, C, C, K, k, k, s, p, OH, OW, K,
                stream()) == 0
    out['dgrad'] = (_rel(dx.float(), rdx), _nr(dx.float(), rdx))
    del rdx, dx
    # weight gradient, as the training step issues it
    if k == 1:
        dw = torch.zeros(K, C, 1, 1, device=dev)
        assert call('dmy_conv_wgrad_ex', 1, ptr(x), ptr(dy), ptr(dw), N, H, W, C, C, K, 1, 1, s, p, OH, OW, K, 3,
                    stream()) == 0
    else:
        dwo = torch.empty(K * C * k * k, device=dev)
        dw = torch.empty(K, C, k, k, device=dev)
        assert call('dmy_conv_wgrad_ex', 1, ptr(x), ptr(dy), ptr(dwo), N, H, W, C, C, K, k, k, s, p, OH, OW, K, 0,
                    stream()) == 0
        call('dmy_conv_wgrad_to_oihw', ptr(dwo), ptr(dw), K, C, C, k, k, stream())
    out['wgrad'] = (_rel(dw, rdw), _nr(dw, rdw))
    torch.cuda.synchronize()
    return out


BOUNDS = {'fwd': (2.5e-3, 5e-5), 'dgrad': (2.5e-3, 5e-5), 'wgrad': (5e-5, 1e-6), 'bn': (1e-6, 0.0)}


# the same layers at batch 2 (the whole-model bench-shape tests' batch): M of 1152..294912 rows, where the plans
# switch to the small-grid tiles (v2 64 x 64 / 128 x 128, split shapes) -- round 6 caught a BN partial-row count there
# that did not follow the tile rule (the finalize read rows no kernel wrote) only through the whole-model test
DMA2 = sorted({(2,) + sh[1:] for sh in DMA})


@pytest.mark.parametrize('cfg,shape', [('v5s', sh) for sh in V5S] + [('dma', sh) for sh in DMA] +
                         [('dma-bs2', sh) for sh in DMA2])
def test_conv_kernels_at_bench_shapes(cfg, shape):
    torch.backends.cuda.matmul.allow_tf32 = False
    r = _check_shape(*shape, seed=sum(shape))
    print(f'{cfg} {shape}: ' + ' '.join(f'{kd} rel {e:.2e} norm {n:+.2e}' for kd, (e, n) in r.items()), flush=True)
    bad = [(kd, e, n) for kd, (e, n) in r.items() if e > BOUNDS[kd][0] or abs(n) > BOUNDS[kd][1]]
    torch.cuda.empty_cache()
    assert not bad, bad


def test_halo_bn_statistics_large_mean_at_bench_shape():
    """the persistent halo kernel (3x3 s1 64 -> 64, DMA-YOLO-l's 768^2 bs32 layer: ~288 tiles per block)
    sums each lane's BN sum / sum of squares over every tile of its block; with mean >> std, var = E[z^2] - E[z]^2
    amplifies a running-sum error by (mean / std)^2.  Inputs 1 + 0.02 n (bf16) and positive weights give mean / std
    = 42 (amplification ~1.8e3); the batch mean and variance from the kernel's partial rows (summed in float64, as
    dmy_bn_finalize does) against float64 statistics of an fp32 reference convolution: mean within 1e-6, variance
    within 2e-3 relative.  Measured (round 4): mean 1.2e-8, variance 4.5e-5 with the per-lane fp32 sums; a
    Kahan-compensated version measured 3.7e-5 and cost 4 % of the kernel's time, so the plain sums stay."""
    from dmayolo.functional import call, ptr, stream, prep_weight
    torch.backends.cuda.matmul.allow_tf32 = False
    N, C, H, W, K = 32, 64, 768, 768, 64
    dev = 'cuda'
    g = torch.Generator(device=dev).manual_seed(5)
    x = (1 + 0.02 * torch.randn(N, C, H, W, generator=g, device=dev)).bfloat16().contiguous(
        memory_format=torch.channels_last)
    w = (1 + 0.2 * torch.randn(K, C, 3, 3, generator=g, device=dev)) / (C * 9)
    wf, _ = prep_weight(w, torch.bfloat16, False)
    y = torch.empty(N, K, H, W, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    P = call('dmy_conv_fwd_bn_rows', 1, ptr(x), ptr(wf), None, ptr(y), N, H, W, C, C, K, 3, 3, 1, 1, H, W, K)
    ps = torch.full((P, K), float('nan'), device=dev)
    pq = torch.full((P, K), float('nan'), device=dev)
    call('dmy_conv_fwd', 1, ptr(x), ptr(wf), None, ptr(y), ptr(ps), ptr(pq), N, H, W, C, C, K, 3, 3, 1, 1, H, W, K,
         stream())
    M = N * H * W
    mean_p = ps.double().sum(0) / M
    var_p = pq.double().sum(0) / M - mean_p ** 2
    del ps, pq, y
    wb = w.bfloat16().float().reshape(K, C * 9)
    s1 = torch.zeros(K, device=dev, dtype=torch.float64)
    s2 = torch.zeros(K, device=dev, dtype=torch.float64)
    for b in range(N):
        z = torch.matmul(wb, F.unfold(x[b:b + 1].float(), 3, padding=1)[0]).double()  # [K, H W]
        s1 += z.sum(1)
        s2 += (z * z).sum(1)
        del z
    mean_r = s1 / M
    var_r = s2 / M - mean_r ** 2
    em = float(((mean_p - mean_r).abs() / mean_r.abs()).max())
    ev = float(((var_p - var_r).abs() / var_r).max())
    ratio = float((mean_r / var_r.sqrt()).mean())
    print(f'halo BN statistics at {N}x{C}x{H}x{W}: P {P} rows, mean / std {ratio:.0f}, max rel err mean {em:.2e} '
          f'var {ev:.2e}')
    assert P >= 64 and em < 1e-6 and ev < 2e-3, (em, ev)
