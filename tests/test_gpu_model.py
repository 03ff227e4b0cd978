"""GPU parity of whole models (product Model/parse_model) against golden vectors captured from
the reference: train-mode outputs, parameter gradients, eval-mode decoded predictions."""
import os

import pytest
import torch

from golden_util import Fixture, load_sd

pytestmark = pytest.mark.gpu
CFG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'dma-yolo_amd', 'dmayolo', 'configs')


def _model(fx, dtype=torch.float32):
    from dmayolo.models.yolo import Model
    m = Model(fx.meta['yaml'], nc=fx.meta['nc'], act_dtype=dtype)
    load_sd(m, fx.group('sd'))
    for mod in m.modules():
        if type(mod).__name__ == 'SwinTransformerLayer':
            mod.drop_path = torch.nn.Identity()
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    return m.cuda()


@pytest.mark.parametrize('name', ['model_v5s', 'model_dma', 'model_c5'])
def test_model_train_eval_fp32(name):
    fx = Fixture(name)
    m = _model(fx)
    if name == 'model_c5':
        # config 5's CBAM channel-max / SPP max-pool argmaxes sit on near-ties at this fixture: the s2d stem's
        # different fp32 summation order (layer-0 output within 5e-7 relative, measured round 1) flips a
        # few of them and reroutes C3TR gradients.  Pin c5 with the direct stem; s2d is pinned on v5s / dma
        # here and against the direct stem in test_s2d_stem_matches_strided_stem.
        m.s2d_stem = False
    x = fx.t('in.0').cuda()
    m.train()
    outs = m(x)
    gups = [g.cuda() for g in fx.seq('gup')]
    loss = sum((o.float() * g).sum() for o, g in zip(outs, gups))
    loss.backward()
    for a, b in zip(outs, fx.seq('out')):
        torch.testing.assert_close(a.float().cpu(), b, rtol=1e-3, atol=1e-3)
    params = dict(m.named_parameters())
    for k, g in fx.group('gp').items():
        torch.testing.assert_close(params[k].grad.cpu(), g, rtol=2e-3, atol=2e-3 * max(1.0, float(g.abs().max())))
    gn = fx.t('gnorm')
    names = [str(s) for s in fx.z['pnames']]
    got = torch.tensor([float(params[k].grad.norm()) if params[k].grad is not None else 0.0 for k in names],
                       dtype=torch.float64)
    torch.testing.assert_close(got, gn, rtol=5e-3, atol=1e-5)  # zero-grad biases before BN: noise in the reference
    load_sd(m, fx.group('sd'))
    m.eval()
    with torch.no_grad():
        z, _ = m(x)
    torch.testing.assert_close(z.cpu(), fx.t('eout.0'), rtol=1e-3, atol=2e-3)


def test_model_bf16_close_to_fp32():
    fx = Fixture('model_v5s')
    m32, m16 = _model(fx), _model(fx, torch.bfloat16)
    x = fx.t('in.0').cuda()
    m32.eval()
    m16.eval()
    with torch.no_grad():
        z32, _ = m32(x)
        z16, _ = m16(x)
    err = (z16 - z32).abs().max() / z32.abs().max()
    assert float(err) < 2e-2, float(err)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_s2d_stem_matches_strided_stem(dtype):
    """The space-to-depth stem (image_s2d + k3 s1 p1 over Cs channels) against the direct k6 s2 p2 stem over
    the channel-padded image: layer-0 output, stem weight gradient and BN gradients (uint8 input as train.py)."""
    from dmayolo.models.yolo import Model
    import dmayolo.functional as Fn
    torch.manual_seed(0)
    ms = []
    for s2d in (True, False):
        torch.manual_seed(0)
        m = Model(os.path.join(CFG, 'yolov5n.yaml'), nc=10, act_dtype=dtype).cuda().train()
        m.s2d_stem = s2d
        ms.append(m)
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 256, (2, 3, 96, 160), generator=g, dtype=torch.uint8).cuda()
    assert Fn.image_s2d(x, dtype)._dmy_s2d == 3
    outs, grads = [], []
    for m in ms:
        y0 = m.model[0](m.to_input(x))
        gup = torch.randn(y0.shape, generator=torch.Generator().manual_seed(2)).to(y0.device)
        (y0.float() * gup).sum().backward()
        outs.append(y0.float())
        grads.append([m.model[0].conv.weight.grad.clone(), m.model[0].bn.weight.grad.clone()])
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(outs[0], outs[1], **tol)
    for a, b in zip(grads[0], grads[1]):
        scale = float(b.abs().max())
        torch.testing.assert_close(a, b, rtol=tol['rtol'] * 5, atol=tol['atol'] * 5 * max(1.0, scale))


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_inference_epilogue_matches_unfused_and_tracks_updates(dtype):
    """no-grad eval forward (one launch per conv: conv + eval-BN + act + residual epilogue, cached prepped weights
    and BN coefficients) vs the training-path kernels on the same eval model; again after a FusedSGD step and a
    train-mode forward changed weights / running stats behind torch's back (cache invalidation); and fused."""
    from dmayolo.models.yolo import Model
    from dmayolo.optim import FusedSGD
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, 'yolov5n.yaml'), nc=10, act_dtype=dtype).cuda()
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 256, (2, 3, 160, 192), generator=g, dtype=torch.uint8).cuda()
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)

    def both():
        m.eval()
        with torch.no_grad():
            a, _ = m(x)
        with torch.enable_grad():  # parameters require grad -> the unfused training-path kernels
            b, _ = m(x)
        return a.float(), b.detach().float()

    a, b = both()
    torch.testing.assert_close(a, b, **tol)
    opt = FusedSGD(m.parameters(), lr=0.1, momentum=0.9)
    m.train()
    outs = m(x)
    sum(o.float().square().mean() for o in outs).backward()
    opt.step()
    a2, b2 = both()
    torch.testing.assert_close(a2, b2, **tol)
    assert float((a2 - a).abs().max()) > 1e-3  # the step changed the predictions: caches were refreshed
    m.fuse()
    with torch.no_grad():
        c, _ = m.eval()(x)
    torch.testing.assert_close(c.float(), a2, **(tol if dtype == torch.float32 else dict(rtol=5e-2, atol=6e-2)))


def test_graphed_detector_replays_eager_forward():
    """infer.GraphedDetector (HIP-graph replay of the eval forward) == the eager forward, bit for bit, and it
    re-captures after the weights change (FusedSGD writes them through raw pointers)."""
    from dmayolo.models.yolo import Model
    from dmayolo.infer import GraphedDetector
    from dmayolo.optim import FusedSGD
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, 'yolov5s.yaml'), nc=10, act_dtype=torch.bfloat16).cuda().eval()
    gd = GraphedDetector(m)
    g = torch.Generator().manual_seed(4)
    xs = [torch.randint(0, 256, (1, 3, 256, 320), generator=g, dtype=torch.uint8).cuda() for _ in range(3)]
    with torch.no_grad():
        for x in xs:
            torch.testing.assert_close(gd(x)[0], m(x)[0], rtol=0, atol=0)
    m.train()
    opt = FusedSGD(m.parameters(), lr=0.1)
    sum(o.float().square().mean() for o in m(xs[0])).backward()
    opt.step()
    m.eval()
    with torch.no_grad():
        torch.testing.assert_close(gd(xs[1])[0], m(xs[1])[0], rtol=0, atol=0)


def test_graphed_detect_equals_eager_forward_and_nms():
    """infer.GraphedDetector.detect (eval forward + the NMS kernels recorded in ONE graph, one host read) == the eager
    forward + utils.general.non_max_suppression, bit for bit, at conf 0.25 and at conf 0.001 -- the latter leaves
    thousands of candidates, more than the first recorded sort capacity: that call falls back to the eager NMS at the
    exact capacity and the next one re-records at it"""
    from dmayolo.models.yolo import Model
    from dmayolo.infer import GraphedDetector
    from dmayolo.utils.general import non_max_suppression
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, 'yolov5s.yaml'), nc=10, act_dtype=torch.bfloat16).cuda().eval()
    gd = GraphedDetector(m)
    g = torch.Generator().manual_seed(5)
    xs = [torch.randint(0, 256, (1, 3, 256, 320), generator=g, dtype=torch.uint8).cuda() for _ in range(3)]
    with torch.no_grad():
        for conf in (0.25, 0.001):
            for x in xs:
                dets, (z, _) = gd.detect(x, conf, 0.45, max_det=300)
                ze = m(x)[0]
                de = non_max_suppression(ze, conf, 0.45, max_det=300)
                assert torch.equal(z, ze)
                assert len(dets) == len(de) and all(torch.equal(a, b) for a, b in zip(dets, de)), conf
        assert sum(d.shape[0] for d in dets) > 0  # conf 0.001 keeps boxes


def test_graphed_detect_after_call_recapture():
    """detect(), then a weight change, then __call__ (which re-records the forward-only graph and its static input),
    then detect() again: the detect graph keeps its own input buffer and state key, so the second detect re-records
    with the new weights and reads the new input (it used to replay the old graph on a stale input)"""
    from dmayolo.models.yolo import Model
    from dmayolo.infer import GraphedDetector
    from dmayolo.utils.general import non_max_suppression
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, 'yolov5s.yaml'), nc=10, act_dtype=torch.bfloat16).cuda().eval()
    gd = GraphedDetector(m)
    g = torch.Generator().manual_seed(6)
    xs = [torch.randint(0, 256, (1, 3, 256, 320), generator=g, dtype=torch.uint8).cuda() for _ in range(3)]

    def check(dets, z, x):
        ze = m(x)[0]
        de = non_max_suppression(ze, 0.01, 0.45, max_det=300)
        assert torch.equal(z, ze)
        assert len(dets) == len(de) and all(torch.equal(a, b) for a, b in zip(dets, de))

    with torch.no_grad():
        dets, (z, _) = gd.detect(xs[0], 0.01, 0.45)
        check(dets, z, xs[0])
        det0 = z.clone()
        for p in m.parameters():  # an in-place weight change torch sees (its _version moves)
            p.mul_(1.01)
            break
        m.model[-1].m[0].bias.add_(0.5)
        torch.testing.assert_close(gd(xs[1])[0], m(xs[1])[0], rtol=0, atol=0)  # __call__ re-records
        dets, (z, _) = gd.detect(xs[2], 0.01, 0.45)
        check(dets, z, xs[2])
        dets, (z, _) = gd.detect(xs[0], 0.01, 0.45)  # same input as the first call, new weights
        check(dets, z, xs[0])
        assert not torch.equal(z, det0)


def test_graphed_train_step_matches_eager():
    """train_graph.GraphedTrainStep (fwd + loss + bwd replayed as one HIP graph, optimizer / EMA eager) against
    the eager step on an identical model copy over batches with different target counts (zero-row padding,
    re-capture when the count outgrows the capacity).  In deterministic mode (split-K weight-grads reduced in
    split order, order-fixed loss sums) the replayed step and the eager step run the same kernels on the same
    data, so losses and parameters must agree bit for bit after every step."""
    import copy
    import dmayolo.functional as Fn
    from dmayolo.models.yolo import Model
    from dmayolo.optim import FusedSGD
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.synthetic import targets as synth_targets, HYP_VISDRONE, scaled_hyp
    from dmayolo.train_graph import GraphedTrainStep
    Fn.set_deterministic(True)
    try:
        torch.manual_seed(0)
        m1 = Model(os.path.join(CFG, 'yolov5n.yaml'), nc=10, act_dtype=torch.float32).cuda().train()
        m1.hyp = scaled_hyp(HYP_VISDRONE, 10, 160, 3)
        m2 = copy.deepcopy(m1)
        o1 = FusedSGD(m1.parameters(), lr=0.01, momentum=0.9, nesterov=True)
        o2 = FusedSGD(m2.parameters(), lr=0.01, momentum=0.9, nesterov=True)
        l1, l2 = ComputeLoss(m1), ComputeLoss(m2)
        gstep = GraphedTrainStep(m2, l2, o2, tcap=16)
        g = torch.Generator().manual_seed(5)
        for i, nt_per in enumerate([3, 5, 4, 12, 6]):
            x = torch.randint(0, 256, (2, 3, 160, 160), generator=g, dtype=torch.uint8).cuda()
            t = synth_targets(2, 10, per_image=nt_per, seed=10 + i, device='cuda')
            o1.zero_grad(set_to_none=True)
            a, ai = l1(m1(x), t)
            a.backward()
            o1.step()
            b, bi = gstep(x, t)
            assert torch.equal(b, a.detach()) and torch.equal(bi, ai), (i, b, a)
            diff = [k for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()) if not torch.equal(p1, p2)]
            assert not diff, (i, diff[:5])
        assert gstep.captures == 2  # first call + the 12-targets/img batch outgrowing tcap 16
    finally:
        Fn.set_deterministic(False)


@pytest.mark.parametrize('name', ['model_v5s', 'model_dma'])
def test_attempt_load_fused_eval_matches_reference(name, tmp_path):
    """§8(f) row 3: a checkpoint written by save_checkpoint and read back by attempt_load(fuse=True) -- the
    models/experimental.py:113-131 path: ema/model entry, BN folded into every YAML-level Conv, eval -- gives the
    reference's eval output (the fixture's unfused eval: folding is exact up to fp32 rounding)."""
    from dmayolo.utils.ckpt import save_checkpoint, attempt_load
    fx = Fixture(name)
    m = _model(fx).cpu()
    p = str(tmp_path / 'best.pt')
    save_checkpoint(p, m, half=False)
    fm = attempt_load(p, device='cuda', fuse=True)
    assert not any(hasattr(mm, 'bn') for mm in fm.model if type(mm).__name__ == 'Conv')
    with torch.no_grad():
        z, _ = fm(fx.t('in.0').cuda())
    torch.testing.assert_close(z.cpu(), fx.t('eout.0'), rtol=1e-3, atol=2e-3)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_detect_module_vs_reference_golden(dtype):
    """a11: the product Detect head alone (three 1x1 convs + the dmy_detect_decode kernel) against the reference's
    own Detect outputs (tests/golden/detect.npz): train-mode raw maps and eval-mode decoded boxes.  bf16 inputs /
    weights: outputs within bf16 rounding of the fp32 golden (rtol 2e-2 on the raw maps, decoded boxes relative to
    their scale)."""
    from dmayolo.models.yolo import Detect
    fx = Fixture('detect')
    meta = fx.meta
    d = Detect(meta['nc'], meta['anchors'], meta['ch'])
    d.stride = torch.tensor(meta['stride'], dtype=torch.float32)
    load_sd(d, fx.group('sd'))
    d = d.cuda()
    xs = [t.to(dtype).cuda().contiguous(memory_format=torch.channels_last) for t in fx.seq('in')]
    d.train()
    outs = d(xs)
    tol = dict(rtol=1e-4, atol=1e-5) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    for a, b in zip(outs, fx.seq('out')):
        torch.testing.assert_close(a.float().cpu(), b, **tol)
    d.eval()
    with torch.no_grad():
        z, _ = d(xs)
    ref = fx.t('eout.0')
    if dtype == torch.float32:
        torch.testing.assert_close(z.cpu(), ref, rtol=1e-4, atol=1e-3)
    else:
        assert float((z.cpu() - ref).abs().max()) < 2e-2 * float(ref.abs().max())


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_detect_decode_one_launch_equals_per_level(dtype):
    """Detect.decode's one launch over every level (dmy_detect_decode_levels) gives the bits of one dmy_detect_decode
    per level, for strided (permuted NHWC head) level views and a batch of 2"""
    from dmayolo.functional import call, ptr, stream, dcode
    from dmayolo.models.yolo import Detect
    torch.manual_seed(3)
    d = Detect(7, [[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [116, 90, 156, 198, 373, 326]], (32, 64, 128))
    d.stride = torch.tensor([8., 16., 32.])
    d = d.cuda().eval()
    xs = [torch.randn(2, c, 80 // s, 72 // s, device='cuda').to(dtype).contiguous(memory_format=torch.channels_last)
          for c, s in ((32, 1), (64, 2), (128, 4))]
    with torch.no_grad():
        z, out = d(xs)
    total = sum(d.na * p.shape[2] * p.shape[3] for p in out)
    ref = torch.empty_like(z)
    anchors = d.anchors.float().contiguous()
    off = 0
    for i, p in enumerate(out):
        _, na, ny, nx, no = p.shape
        sd = p.stride()
        call('dmy_detect_decode', dcode(p), ptr(p), sd[0], sd[2], sd[3], 2, ny, nx, na, no, float(d.stride[i]),
             ptr(anchors[i]), ptr(ref), off, total, stream())
        off += na * ny * nx
    torch.cuda.synchronize()
    assert torch.equal(z.view(torch.int32), ref.view(torch.int32))


def test_jit_trace_like_reference_logger():
    """Missing-item #7 of round 1: the reference's train.py logs the graph at the first batch with
    torch.jit.trace(de_parallel(model), imgs[0:1], strict=False) (utils/loggers/__init__.py:86, plots on by default).
    Under tracing the product forward is one registered op (dmayolo::model_forward); the trace must succeed, record
    that op, and replay to the eager outputs (train and eval mode)."""
    import warnings
    from dmayolo.models.yolo import Model
    from dmayolo.synthetic import images
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, 'yolov5s.yaml'), nc=10, act_dtype=torch.bfloat16).cuda()
    x = images(2, 256, device='cuda')
    for train in (True, False):
        m.train(train)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            tr = torch.jit.trace(m, x[0:1], strict=False)
        assert any(n.kind() == 'dmayolo::model_forward' for n in tr.inlined_graph.nodes())
        with torch.no_grad():
            got, ref = tr(x[0:1]), m(x[0:1])
        if not train:
            got, ref = [got[0]] + list(got[1]), [ref[0]] + list(ref[1])
        for a, b in zip(got, ref):
            torch.testing.assert_close(a.float(), b.float(), rtol=0, atol=0)


def test_no_grad_eval_takes_fused_path_with_trainable_params():
    """a no-grad eval forward must use the one-launch conv + eval-BN + act kernels even when the parameters
    require grad (detect.py / val on a freshly loaded model): ctx.needs_input_grad mirrors requires_grad under
    torch.no_grad(), so it alone would send every layer down the training path (weight prep, separate BN)"""
    import dmayolo.functional as Fn
    from dmayolo.models.yolo import Model
    from dmayolo.synthetic import images
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, 'yolov5s.yaml'), nc=10, act_dtype=torch.bfloat16).cuda().eval()
    assert all(p.requires_grad for p in m.parameters())
    x = images(1, 320, device='cuda')
    counts = {}
    orig = Fn.call

    def counting(name, *a):
        counts[name] = counts.get(name, 0) + 1
        return orig(name, *a)
    with torch.no_grad():
        ref, _ = m(x)  # fills the per-layer caches
        Fn.call = counting
        try:
            z, _ = m(x)
        finally:
            Fn.call = orig
    assert counts.get('dmy_bn_act_fwd', 0) == 0 and counts.get('dmy_conv_wprep', 0) == 0, counts
    assert counts.get('dmy_conv_fwd_act', 0) > 0
    torch.testing.assert_close(z, ref, rtol=0, atol=0)
