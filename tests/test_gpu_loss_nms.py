"""GPU parity for ComputeLoss (incl. build_targets) and non_max_suppression against golden
vectors captured from the reference: integer/index outputs bit-exact, NMS rows bit-exact,
loss / dL/dp within fp32 tolerance."""
import types

import pytest
import torch

from golden_util import Fixture, golden_names

pytestmark = pytest.mark.gpu


def _loss_obj(fx, device):
    from dmayolo.utils.loss import ComputeLoss
    meta = fx.meta
    det = types.SimpleNamespace(nl=3, na=3, nc=meta['nc'], anchors=fx.t('anchors').to(device))
    model = types.SimpleNamespace(hyp=meta['hyp'], model=[det])
    return ComputeLoss(model)


@pytest.mark.parametrize('hyp', ['VisDrone', 'scratch'])
def test_build_targets_exact(hyp):
    fx = Fixture(f'loss_{hyp}')
    cl = _loss_obj(fx, 'cuda')
    p = [fx.t(f'p.{i}').cuda() for i in range(3)]
    tcls, tbox, indices, anch = cl.build_targets(p, fx.t('targets').cuda())
    for i in range(3):
        for j, k in enumerate(('b', 'a', 'gj', 'gi')):
            assert torch.equal(indices[i][j].cpu(), fx.t(f'{k}.{i}').long()), (i, k)
        assert torch.equal(tcls[i].cpu(), fx.t(f'tcls.{i}').long())
        assert torch.equal(tbox[i].cpu(), fx.t(f'tbox.{i}'))
        assert torch.equal(anch[i].cpu(), fx.t(f'anch.{i}'))


@pytest.mark.parametrize('hyp', ['VisDrone', 'scratch'])
@pytest.mark.parametrize('layout', ['contiguous', 'nhwc'])
def test_loss_and_grad(hyp, layout):
    fx = Fixture(f'loss_{hyp}')
    cl = _loss_obj(fx, 'cuda')
    ps = []
    for i in range(3):
        p = fx.t(f'p.{i}').cuda()
        if layout == 'nhwc':  # the Detect head's native layout: [N,H,W,na,no] permuted view
            N, na, H, W, no = p.shape
            p = p.permute(0, 2, 3, 1, 4).contiguous().permute(0, 3, 1, 2, 4)
        ps.append(p.requires_grad_(True))
    loss, items = cl(ps, fx.t('targets').cuda())
    loss.backward()
    torch.testing.assert_close(loss.cpu(), fx.t('loss'), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(items.cpu(), fx.t('items'), rtol=1e-5, atol=1e-6)
    for i in range(3):
        g = fx.t(f'gp.{i}')
        torch.testing.assert_close(ps[i].grad.cpu(), g, rtol=1e-4, atol=1e-6 * max(1.0, float(g.abs().max())))


def test_loss_no_targets():
    fx = Fixture('loss_VisDrone')
    cl = _loss_obj(fx, 'cuda')
    ps = [fx.t(f'p.{i}').cuda().requires_grad_(True) for i in range(3)]
    loss, items = cl(ps, torch.zeros((0, 6), device='cuda'))
    loss.backward()
    from oracle.loss import compute_loss
    l2, i2 = compute_loss([fx.t(f'p.{i}') for i in range(3)], torch.zeros((0, 6)), fx.t('anchors'), fx.meta['hyp'],
                          fx.meta['nc'])
    torch.testing.assert_close(loss.cpu(), l2, rtol=1e-5, atol=1e-6)
    assert float(items[0]) == 0.0 and float(items[2]) == 0.0


def test_siou_kernel_vs_golden():
    """The loss kernel's SIoU device function (forward-mode dual numbers, csrc/detect_loss.hip) through the
    C ABI (dmy_siou_eval) against the reference's bbox_iou(..., SIoU=True) value and its autograd gradient
    w.r.t. the predicted box (tools/gen_golden.py gen_siou: incl. near-coincident centres and
    sin_alpha == 1 rows)."""
    from dmayolo.functional import call, ptr, stream
    fx = Fixture('siou')
    b1, b2 = fx.t('b1').cuda().contiguous(), fx.t('b2').cuda().contiguous()
    n = b1.shape[0]
    iou = torch.empty(n, device='cuda')
    g = torch.empty(n, 4, device='cuda')
    call('dmy_siou_eval', ptr(b1), ptr(b2), ptr(iou), ptr(g), n, stream())
    ref_iou, ref_g = fx.t('iou'), fx.t('g')
    torch.testing.assert_close(iou.cpu(), ref_iou, rtol=1e-5, atol=1e-6, equal_nan=True)
    ok = torch.isfinite(ref_g).all(1)
    torch.testing.assert_close(g.cpu()[ok], ref_g[ok], rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize('name', golden_names('nms_'))
def test_nms_exact(name):
    from dmayolo.utils.general import non_max_suppression
    fx = Fixture(name)
    out = non_max_suppression(fx.t('pred').cuda(), **fx.meta)
    ref = fx.seq('out')
    assert len(out) == len(ref)
    for a, b in zip(out, ref):
        assert a.shape == b.shape, (a.shape, b.shape)
        assert torch.equal(a.cpu(), b), (a.cpu() - b).abs().max()


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_nms_vs_oracle_random(seed):
    """Random clustered predictions incl. a >30k-candidate multi-label case: bit-exact vs oracle."""
    from dmayolo.utils.general import non_max_suppression
    from oracle.general import non_max_suppression as onms
    g = torch.Generator().manual_seed(seed)
    A, nc = (8000, 6) if seed < 2 else (12000, 4)
    pred = torch.rand(2, A, nc + 5, generator=g)
    pred[..., :2] *= 300
    pred[..., 2:4] = pred[..., 2:4] * 30 + 1
    kw = dict(conf_thres=0.2, iou_thres=0.5, multi_label=seed != 1, max_det=500)
    if seed == 2:
        kw = dict(conf_thres=0.001, iou_thres=0.6, multi_label=True, max_det=300)
    out = non_max_suppression(pred.cuda(), **kw)
    ref = onms(pred, **kw)
    for a, b in zip(out, ref):
        assert torch.equal(a.cpu(), b)


@pytest.mark.parametrize('case', [0, 1, 2, 3])
def test_nms_bitmask_path_vs_oracle(case):
    """Candidate counts that fit the bitmask path (sort capacity <= dmy_nms_mask_rows()): dense clusters, ties in the
    score order, class offsets, agnostic mode and a max_det that stops inside a 64-row block; bit-exact vs oracle and
    vs the lazy greedy kernel on the same sorted keys."""
    from dmayolo.functional import call, ptr, stream
    from dmayolo.utils.general import non_max_suppression
    from oracle.general import non_max_suppression as onms
    g = torch.Generator().manual_seed(100 + case)
    A, nc = (3000, 5) if case < 3 else (900, 3)
    pred = torch.rand(2, A, nc + 5, generator=g)
    pred[..., :2] *= 200 if case != 1 else 60  # case 1: heavy overlap
    pred[..., 2:4] = pred[..., 2:4] * 40 + 1
    if case == 2:
        pred[..., 4] = torch.round(pred[..., 4] * 8) / 8  # many exact score ties
    kw = [dict(conf_thres=0.3, iou_thres=0.45, max_det=300), dict(conf_thres=0.25, iou_thres=0.5, max_det=77),
          dict(conf_thres=0.2, iou_thres=0.6, agnostic=True, max_det=1000),
          dict(conf_thres=0.05, iou_thres=0.45, multi_label=True, max_det=300)][case]
    out = non_max_suppression(pred.cuda(), **kw)
    ref = onms(pred, **kw)
    for a, b in zip(out, ref):
        assert torch.equal(a.cpu(), b)
    # the two greedy kernels on identical sorted keys
    p = pred.cuda().contiguous()
    cap = 4096
    cnt = torch.zeros(4, dtype=torch.int32, device='cuda')
    keys = torch.empty((2, cap), dtype=torch.int64, device='cuda')
    multi = int(kw.get('multi_label', False))
    call('dmy_nms_candidates', ptr(p), 2, A, nc + 5, float(kw['conf_thres']), multi, None, ptr(keys), cap, ptr(cnt),
         stream())
    call('dmy_nms_sort', ptr(keys), cap, ptr(cnt), 2, stream())
    assert int(cnt[:2].max()) <= cap
    res = []
    for fn in ('dmy_nms_greedy', 'dmy_nms_greedy_mask'):
        boxes = torch.empty((2, 30000, 5), device='cuda')
        o = torch.full((2, kw['max_det'], 6), float('nan'), device='cuda')
        nk = torch.zeros(2, dtype=torch.int32, device='cuda')
        args = [ptr(p), 2, A, nc + 5, float(kw['iou_thres']), int(kw.get('agnostic', False)), kw['max_det'], 30000,
                ptr(keys), cap, ptr(cnt), ptr(boxes)]
        if fn.endswith('mask'):
            args.append(ptr(torch.empty(2 * cap * (cap // 64), dtype=torch.int64, device='cuda')))
        call(fn, *args, ptr(o), ptr(nk), None, stream())
        torch.cuda.synchronize()
        res.append([o[b, :int(nk[b])].cpu() for b in range(2)])
        # the self-resetting counter form (ncand): the counts leave through ncand and the counter is zero afterwards
        ctr, nc_out = cnt[:2].clone(), torch.full((2,), -1, dtype=torch.int32, device='cuda')
        o2 = torch.full_like(o, float('nan'))
        args2 = args[:10] + [ptr(ctr)] + args[11:]
        call(fn, *args2, ptr(o2), ptr(nk), ptr(nc_out), stream())
        torch.cuda.synchronize()
        assert torch.equal(nc_out, cnt[:2]) and not bool(ctr.any())
        assert all(torch.equal(o2[b, :int(nk[b])].cpu(), res[-1][b]) for b in range(2))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize('cap', [2048, 4096, 8192])
def test_nms_sort_any_count(cap):
    """dmy_nms_sort (pad + bitonic network) leaves each image's first count keys ascending and pad keys after, for
    counts from 0 to cap: the first tile-local pass skips pad-only tiles and, at cap 2048, sorts only the pow2 prefix
    holding the candidates (round 5) and writes the pad keys itself (no pad launch); later passes must not skip (a
    descending merge moves real keys to a block end)"""
    from dmayolo.functional import call, ptr, stream
    g = torch.Generator().manual_seed(cap)
    counts = [0, 1, 5, 100, 1000, 2047, 2048, min(3000, cap), min(5000, cap), cap]
    nimg = len(counts)
    keys = torch.randint(0, 2 ** 62, (nimg, cap), generator=g, dtype=torch.int64)
    ref = [torch.sort(keys[b, :n])[0] for b, n in enumerate(counts)]
    kd = keys.cuda()
    cnt = torch.tensor(counts + [0] * nimg, dtype=torch.int32, device='cuda')
    call('dmy_nms_sort', ptr(kd), cap, ptr(cnt), nimg, stream())
    out = kd.cpu()
    for b, n in enumerate(counts):
        assert torch.equal(out[b, :n], ref[b]), (cap, n)
        assert bool((out[b, n:] == -1).all()), (cap, n)  # PADKEY = all ones
