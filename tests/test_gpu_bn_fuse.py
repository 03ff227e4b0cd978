"""GPU: the producer-BN backward-reduce partials written by the consumer conv's data-grad epilogue
(dmy_conv_dgrad_bn, csrc/conv.hip store_dgrad_bn) instead of a separate dmy_bn_bwd_reduce pass over dy.
Off by default (measured slower end to end, functional.FUSE_BN_REDUCE); these tests turn it on.

* kernel level: dx is bit-identical to dmy_conv_dgrad's, and the column sums of the fused partials equal those of
  dmy_bn_bwd_reduce over the same dx (both are fp32 sums of the same bf16 products in different groupings:
  rtol 1e-4 on sum du, atol 1e-4 * sum |du * xhat| on the xhat term), for the v3 256x128, wide 256x256 and 1x1 paths,
  plain and accumulating into an existing gradient;
* training step: with the fusion on, a yolov5s step takes the fused path for most BN layers and gives the same
  gradients as with it off, to the same closeness as two unfused steps whose BN backward reductions group the
  rows differently (each reduce split at ~M/2): BN's backward subtracts the per-channel means from du, so an fp32
  reorder in those sums moves dz by far more than one rounding and, through bf16 storage, propagates and grows
  towards the stem (measured ~1e-2 whole-gradient relative L2 on yolov5s) -- that pair is the noise floor
  (bound: 2x its whole-gradient relative L2 + 1e-3, and its worst per-parameter cosine gap x2 + 1e-4).
  Fusable: data-grads on the v3 / wide kernels (>= 16384 rows) with >= 128 columns whose output is the whole
  gradient of a conv+BN output (C3 / bottleneck inputs through their GradSinks); the rest keep dmy_bn_bwd_reduce.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


# (N, C, H, W, K, k): C = the producer's channels = data-grad columns (>= 128), K = this conv's outputs
SHAPES = [(16, 128, 64, 64, 128, 3), (16, 256, 64, 64, 128, 3), (16, 512, 64, 64, 128, 1), (8, 256, 72, 60, 96, 1),
          (16, 136, 64, 64, 64, 3)]


@pytest.mark.parametrize('acc', [0, 1])
@pytest.mark.parametrize('N,C,H,W,K,k', SHAPES)
def test_dgrad_bn_partials_match_bn_bwd_reduce(N, C, H, W, K, k, acc):
    from dmayolo.functional import call, ptr, stream, prep_weight
    from dmayolo._lib import ACT_SILU
    g = torch.Generator().manual_seed(N + C + K + k + acc)
    p = k // 2
    cl = dict(memory_format=torch.channels_last)
    dy = torch.randn(N, K, H, W, generator=g).bfloat16().cuda().contiguous(**cl)
    w = (torch.randn(K, C, k, k, generator=g) / (K * k * k) ** 0.5).cuda()
    _, wt = prep_weight(w, torch.bfloat16, True)
    z = torch.randn(N, C, H, W, generator=g).bfloat16().cuda().contiguous(**cl)
    scale, shift = (torch.rand(C, generator=g) + 0.5).cuda(), (torch.randn(C, generator=g) * 0.3).cuda()
    mean, invstd = (torch.randn(C, generator=g) * 0.1).cuda(), (torch.rand(C, generator=g) + 0.5).cuda()
    base = torch.randn(N, C, H, W, generator=g).bfloat16().cuda().contiguous(**cl)
    geo = (N, H, W, C, C, K, k, k, 1, p, H, W, K)
    P = call('dmy_conv_dgrad_bn_rows', 1, ptr(dy), ptr(wt), ptr(base), *geo)
    assert P == -(-N * H * W // 256)  # one partial row per 256-row tile
    dx_ref = base.clone() if acc else torch.empty_like(base)
    dx = base.clone() if acc else torch.empty_like(base)
    call('dmy_conv_dgrad', 1, ptr(dy), ptr(wt), ptr(dx_ref), acc, *geo, stream())
    pdb = torch.full((P, C), float('nan'), device='cuda')
    pdg = torch.full((P, C), float('nan'), device='cuda')
    call('dmy_conv_dgrad_bn', 1, ptr(dy), ptr(wt), ptr(dx), acc, *geo, ptr(z), C, ptr(scale), ptr(shift), ptr(mean),
         ptr(invstd), ACT_SILU, ptr(pdb), ptr(pdg), stream())
    M = N * H * W
    R = call('dmy_bn_reduce_rows', 1, ptr(z), C, ptr(dx_ref), C, M, C)
    rdb, rdg = torch.empty(R * C, device='cuda'), torch.empty(R * C, device='cuda')
    call('dmy_bn_bwd_reduce', 1, ptr(z), C, ptr(dx_ref), C, ptr(scale), ptr(shift), ptr(mean), ptr(invstd), ACT_SILU,
         M, C, ptr(rdb), ptr(rdg), stream())
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_ref), 'the fused epilogue must store exactly what dmy_conv_dgrad stores'
    assert torch.isfinite(pdb).all() and torch.isfinite(pdg).all(), 'every partial row must be written'
    sdb, sdg = pdb.sum(0).double(), pdg.sum(0).double()
    edb, edg = rdb.view(R, C).sum(0).double(), rdg.view(R, C).sum(0).double()
    # magnitude references for the absolute bounds (fp32 sums of ~M terms)
    zf = z.float().permute(0, 2, 3, 1).reshape(-1, C)
    u = zf * scale + shift
    du = dx_ref.float().permute(0, 2, 3, 1).reshape(-1, C) * (torch.sigmoid(u) * (1 + u * (1 - torch.sigmoid(u))))
    mag_b = du.abs().sum(0).double()
    mag_g = (du * (zf - mean) * invstd).abs().sum(0).double()
    assert float(((sdb - edb).abs() / mag_b.clamp_min(1e-9)).max()) < 1e-4
    assert float(((sdg - edg).abs() / mag_g.clamp_min(1e-9)).max()) < 1e-4


def test_training_step_uses_fusion_and_matches_unfused():
    import dmayolo.functional as Fn
    from dmayolo.models.yolo import Model
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp
    counts = {}
    orig = Fn.call

    def counting(name, *a):
        counts[name] = counts.get(name, 0) + 1
        return orig(name, *a)

    def grads(fuse):
        Fn.FUSE_BN_REDUCE[0] = fuse
        torch.manual_seed(0)
        m = Model(os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs', 'yolov5s.yaml'), nc=10,
                  act_dtype=torch.bfloat16).cuda()
        m.hyp = scaled_hyp(HYP_VISDRONE, 10, 640)
        x, t = images(16, 640, device='cuda'), targets(16, 10, device='cuda')  # stride-16 layers: M = 25600
        loss, _ = ComputeLoss(m)(m(x), t)
        loss.backward()
        return {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}

    import ctypes

    def shifted_reduce(name, *a):
        """dmy_bn_bwd_reduce over rows [0, M1) and [M1, M) separately: the same sums, other fp32 groupings"""
        if name == 'dmy_bn_reduce_rows' and a[3] is not None:  # (dy None: the bias-gradient column sums)
            dt, z, zps, dy, dps, M, C = a
            M1 = (M // 2 + 8) // 8 * 8 + 8
            off = lambda p, ps: ctypes.c_void_p(p.value + M1 * ps * 2)
            return orig(name, dt, z, zps, dy, dps, M1, C) + orig(name, dt, off(z, zps), zps, off(dy, dps), dps, M - M1, C)
        if name == 'dmy_bn_bwd_reduce':
            dt, z, zps, dy, dps, sc, sh, mu, iv, act, M, C, pdb, pdg, st = a
            M1 = (M // 2 + 8) // 8 * 8 + 8
            off = lambda p, ps: ctypes.c_void_p(p.value + M1 * ps * 2)
            R1 = orig('dmy_bn_reduce_rows', dt, z, zps, dy, dps, M1, C)
            orig(name, dt, z, zps, dy, dps, sc, sh, mu, iv, act, M1, C, pdb, pdg, st)
            poff = lambda p: ctypes.c_void_p(p.value + R1 * C * 4)
            return orig(name, dt, off(z, zps), zps, off(dy, dps), dps, sc, sh, mu, iv, act, M - M1, C, poff(pdb),
                        poff(pdg), st)
        return orig(name, *a)

    prev_fuse = Fn.FUSE_BN_REDUCE[0]
    try:
        Fn.set_deterministic(True)
        Fn.call = shifted_reduce
        noise = grads(False)  # the unfused step with every BN reduce grouped differently (noise floor)
        Fn.call = orig
        ref = grads(False)
        Fn.call = counting
        got = grads(True)
    finally:
        Fn.call = orig
        Fn.FUSE_BN_REDUCE[0] = prev_fuse
        Fn.set_deterministic(False)
    fused, unfused = counts.get('dmy_conv_dgrad_bn', 0), counts.get('dmy_bn_bwd_reduce', 0)
    print(f'fused {fused} unfused {unfused}')
    assert fused >= 6  # the v3 data-grads of >= 128 input channels (yolov5s: C3 inputs, bottlenecks of width >= 128)
    assert set(got) == set(ref)
    # bf16 storage: an fp32 reorder in one BN reduction can flip the rounding of some dz elements, and the per-channel
    # BN bias / weight gradients are sums with heavy cancellation, so a single parameter's relative L2 is no bound;
    # the whole gradient (relative L2) and every parameter's direction (cosine) are
    keys = [k for k in ref if ref[k].norm() > 0]

    def cmp(a):
        allg, allr = torch.cat([a[k].flatten() for k in keys]), torch.cat([ref[k].flatten() for k in keys])
        cos = min((float(torch.nn.functional.cosine_similarity(a[k].flatten().double(), ref[k].flatten().double(),
                                                               dim=0)), k) for k in keys)
        return _rel(allg, allr), cos

    (rel_f, cos_f), (rel_n, cos_n) = cmp(got), cmp(noise)
    order = [k for k in ref]  # registration order ~ forward order
    for k in order:
        r = _rel(got[k], ref[k]) if ref[k].norm() > 0 else 0.0
        if r > 1e-4:
            print(f'  {k}: rel {r:.3e}')
    print(f'fused vs unfused: rel {rel_f:.3e} worst cos {cos_f}; regrouped unfused reduce (noise floor): '
          f'rel {rel_n:.3e} worst cos {cos_n}')
    assert rel_f < 2 * rel_n + 1e-3
    assert cos_f[0] > 1 - 2 * (1 - cos_n[0]) - 1e-4


@pytest.mark.parametrize('N,C,H,W', [(2, 64, 96, 128), (3, 128, 40, 56), (1, 256, 24, 24)])
def test_scconv_gate_applies_k3_bn(N, C, H, W):
    """SCConv with k3's BatchNorm folded into the gate (conv_bn_act(defer=True) + dmy_scgate_bn_fwd / _bwd, whose
    backward hands k3 its BN reduce partials through the BnLink) against the unfused path (DMY_DEFER_AFFINE off:
    bn_act_fwd + dmy_scgate_fwd, bn_bwd_reduce): the forward output, every parameter gradient, the input gradient and
    the running statistics agree (same value contract: u3 = bf16(z * scale + shift), the reduce over du3 as stored)"""
    import dmayolo.functional as Fn
    from dmayolo.models.common import SCConv
    torch.manual_seed(0)
    m = SCConv(C, 2 * C, 2).cuda()
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.2, 0.2)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x0 = torch.randn(N, C, H, W, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
    gup = torch.randn(N, 2 * C, H // 2, W // 2, device='cuda')
    res = []
    for on in (False, True):
        m.load_state_dict(sd)
        m.zero_grad(set_to_none=True)
        Fn.DEFER_AFFINE[0] = on
        try:
            x = x0.clone().requires_grad_(True)
            y = m(x)
            (y.float() * gup).sum().backward()
        finally:
            Fn.DEFER_AFFINE[0] = True
        torch.cuda.synchronize()
        res.append((y.float(), x.grad.float(), {k: p.grad.clone() for k, p in m.named_parameters()},
                    {k: v.clone() for k, v in m.state_dict().items() if 'running' in k}))
    (y0, gx0, gp0, rs0), (y1, gx1, gp1, rs1) = res
    rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))  # noqa: E731
    assert torch.equal(y0, y1), rel(y1, y0)
    assert rel(gx1, gx0) < 1e-6, rel(gx1, gx0)
    for k in gp0:
        assert rel(gp1[k], gp0[k]) < 1e-5 or float((gp1[k] - gp0[k]).abs().max()) < 1e-6, (k, rel(gp1[k], gp0[k]))
    for k in rs0:
        assert torch.equal(rs0[k], rs1[k]), k
