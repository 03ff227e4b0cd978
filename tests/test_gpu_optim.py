"""GPU parity of the fused optimizer / EMA kernels (csrc/optim.hip) against tests/golden/optim.npz
(tools/gen_golden.py `gen_optim`, captured from the reference): train.py:216-222 grouping (g0 BN weights, g1
weights + AdConcat.w with weight decay, g2 biases; Adam hard-codes g0 lr=3e-4), per-group lr / momentum written
into param_groups as the warmup does (train.py:416-420), two steps; ModelEMA.update (utils/torch_utils.py:329-339)
twice over params AND float buffers.

The fixture's `sd.*`, `grad.*`, group lists and `ema.*` entries are the reference's.  Its `sgd.*` / `adam.*`
entries are NOT usable: the round-1 capture stored numpy views of the live parameters (npy() did not copy yet),
so both hold the model's final state (sd + 0.1 from the EMA section, verified: exactly sd + 0.1).  The reference
import is refused from round 1 on, so they cannot be regenerated; the expected values are
recomputed here with torch.optim.SGD / Adam on the CPU -- the very optimizers train.py:216-222 calls -- over the
reference-captured groups, state_dict and gradients."""
import pytest
import torch

from golden_util import Fixture, load_sd

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-6, atol=1e-7)  # fp32 kernels vs torch CPU: one rounding of an fma at most
# Adam: m / (sqrt(v) / bc2 + eps) is O(1) per element, so each update is ~lr-sized and a few ulps of it (fused
# multiply-adds in the kernel vs torch's separate CPU ops) reach ~1e-6 absolute at the bias group's lr 0.05
TOL_ADAM = dict(rtol=1e-5, atol=2e-6)


def _model(fx):
    from dmayolo.models.yolo import Model
    m = Model(fx.meta['yaml'], nc=10)
    load_sd(m, fx.group('sd'))
    return m.cuda()


def _torch_reference(fx, kind):
    """torch.optim on CPU over the fixture's groups / sd / grads, stepped as gen_optim did"""
    from dmayolo.models.yolo import Model
    m = Model(fx.meta['yaml'], nc=10)
    load_sd(m, fx.group('sd'))
    P = dict(m.named_parameters())
    g0, g1, g2 = ([P[k] for k in fx.meta['groups'][n]] for n in ('g0', 'g1', 'g2'))
    if kind == 'adam':
        opt = torch.optim.Adam(g0, lr=3e-4, betas=(0.937, 0.999))
    else:
        opt = torch.optim.SGD(g0, lr=0.01, momentum=0.937, nesterov=True)
    opt.add_param_group({'params': g1, 'weight_decay': 0.0005})
    opt.add_param_group({'params': g2})
    for j, g in enumerate(opt.param_groups):
        g['lr'] = [0.001, 0.002, 0.05][j]
        if 'momentum' in g:
            g['momentum'] = 0.8
    grads = fx.group('grad')
    for step in range(2):
        for k, p in P.items():
            p.grad = grads[k] * (1 + step)
        opt.step()
    return {k: v.detach() for k, v in P.items()}


def test_fixture_optimizer_entries_alias_final_state():
    """documents why _torch_reference exists: the captured sgd.* / adam.* equal the final model state sd + 0.1"""
    fx = Fixture('optim')
    sd = fx.group('sd')
    for kind in ('sgd', 'adam'):
        for k, v in fx.group(kind).items():
            torch.testing.assert_close(v, sd[k] + 0.1, rtol=0, atol=1e-6)


def _check_groups(opt, m, fx):
    names = {id(p): k for k, p in m.named_parameters()}
    got = [[names[id(p)] for p in g['params']] for g in opt.param_groups]
    assert got == [fx.meta['groups'][k] for k in ('g0', 'g1', 'g2')]


@pytest.mark.parametrize('kind', ['sgd', 'adam'])
def test_fused_optimizer_matches_reference(kind):
    from dmayolo.optim import build_optimizer
    fx = Fixture('optim')
    m = _model(fx)
    opt = build_optimizer(m, kind, 0.01, 0.937, 0.0005)
    _check_groups(opt, m, fx)
    for j, g in enumerate(opt.param_groups):
        g['lr'] = [0.001, 0.002, 0.05][j]
        if 'momentum' in g:
            g['momentum'] = 0.8
    grads = fx.group('grad')
    params = dict(m.named_parameters())
    for step in range(2):
        for k, p in params.items():
            p.grad = (grads[k] * (1 + step)).cuda()
        opt.step()
    exp = _torch_reference(fx, kind)
    assert set(exp) == set(params)
    for k, p in params.items():
        torch.testing.assert_close(p.detach().cpu(), exp[k], **(TOL_ADAM if kind == 'adam' else TOL),
                                   msg=lambda s: f'{kind} {k}: {s}')


def test_fused_sgd_late_parameter_starts_from_zero_momentum():
    """A parameter whose grad first appears at step 2 gets torch's clone-on-first-step buffer (no stale
    momentum from uninitialised memory)."""
    from dmayolo.optim import FusedSGD
    torch.manual_seed(0)
    a = torch.nn.Parameter(torch.randn(3000, device='cuda'))
    b = torch.nn.Parameter(torch.randn(5000, device='cuda'))
    ra, rb = [torch.nn.Parameter(t.detach().cpu().clone()) for t in (a, b)]
    opt = FusedSGD([a, b], lr=0.1, momentum=0.9, nesterov=True)
    ref = torch.optim.SGD([ra, rb], lr=0.1, momentum=0.9, nesterov=True)
    ga, gb = torch.randn(3000), torch.randn(5000)
    a.grad, ra.grad = ga.cuda(), ga.clone()
    opt.step()
    ref.step()
    a.grad, b.grad, ra.grad, rb.grad = ga.cuda(), gb.cuda(), ga.clone(), gb.clone()
    opt.step()
    ref.step()
    for p, r in ((a, ra), (b, rb)):
        torch.testing.assert_close(p.detach().cpu(), r.detach(), **TOL)


def test_model_ema_matches_reference():
    from dmayolo.utils.torch_utils import ModelEMA
    fx = Fixture('optim')
    m = _model(fx)
    ema = ModelEMA(m)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.1)
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.add_(0.2)
    ema.update(m)
    ema.update(m)
    got = ema.ema.state_dict()
    exp = fx.group('ema')
    assert set(exp) == set(got)
    for k, v in exp.items():
        g = got[k].cpu()
        if v.dtype.is_floating_point:
            torch.testing.assert_close(g, v, **TOL, msg=lambda s: f'ema {k}: {s}')
        else:
            assert torch.equal(g.to(v.dtype), v), k


@pytest.mark.parametrize('yml', ['yolov5n.yaml', 'yolov5l-xs-tr-cbam-spp-bifpn.yaml'])
def test_trainer_steady_state_reuses_pointer_tables(yml):
    """Every gradient the conv path produces (weights, BN gamma / beta, conv biases) is a slice of the per-forward
    gradient arena, so after the first steps the optimizer / scaler / EMA pointer tables are cache hits: no
    per-step host tensor pinning or H2D table uploads (they showed up as ~100 runtime copy kernels per step).  Config
    5 (C3TR: nn.MultiheadAttention's in_proj_weight gradient is assembled by autograd from three slices, at addresses
    that move between steps) refreshes its tables in place instead of building new ones (round 5; round 4 cached a
    new table per pointer set: ~190 KB of device memory per step)."""
    import os
    from dmayolo import optim
    from dmayolo.models.yolo import Model
    from dmayolo.trainer import Trainer
    from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    torch.manual_seed(0)
    m = Model(os.path.join(root, 'dma-yolo_amd', 'dmayolo', 'configs', yml), nc=10).cuda()
    m.hyp = scaled_hyp(HYP_VISDRONE, 10, 256)
    tr = Trainer(m, m.hyp, 64, nb=100)
    x, t = images(4, 256, device='cuda'), targets(4, 10, device='cuda')
    for _ in range(4):
        tr.step(x, t)
    n0 = sum(1 for _ in optim._Table._cache)
    built = [0]
    orig = optim._Table.__init__

    def counting(self, *a, **k):
        built[0] += 1
        orig(self, *a, **k)
    optim._Table.__init__ = counting
    try:
        for _ in range(4):
            tr.step(x, t)
    finally:
        optim._Table.__init__ = orig
    assert built[0] == 0, (built[0], n0)


def test_fused_adam_skipped_step_leaves_bias_correction():
    """a step the GradScaler skips (non-finite gradient) must not advance Adam's t.  torch: scaler.step()
    never calls optimizer.step(), so the bias corrections 1 - b^t of the next real step use the old t.  FusedAdam keeps t
    on the device and the kernel advances it only when the step ran: steps (finite, non-finite, finite) here equal
    torch.optim.Adam taking the two finite steps."""
    from dmayolo.optim import FusedAdam, GradScaler
    torch.manual_seed(0)
    a = torch.nn.Parameter(torch.randn(10000, device='cuda'))
    ra = torch.nn.Parameter(a.detach().cpu().clone())
    opt = FusedAdam([a], lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-4)
    ref = torch.optim.Adam([ra], lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-4)
    scaler = GradScaler(a.device, enabled=True)
    g = torch.Generator().manual_seed(3)
    for i in range(3):
        gr = torch.randn(10000, generator=g)
        s = float(scaler.scale.cpu())
        a.grad = (gr * s).cuda()
        if i == 1:
            a.grad[17] = float('inf')
        scaler.step(opt)
        scaler.update()
        if i != 1:
            ra.grad = gr.clone()
            ref.step()
    assert int(opt.state[a]['step'].cpu()) == 2
    torch.testing.assert_close(a.detach().cpu(), ra.detach(), **TOL_ADAM)


def test_fused_adam_checkpoint_resume_cpu_map_location(tmp_path):
    """FusedAdam's state_dict is torch Adam's format (a float32 CPU 'step' per parameter, no device counter in
    param_groups); a checkpoint saved with it and loaded with torch.load(map_location='cpu', weights_only=True) resumes
    on the GPU with the right bias corrections (the counter is rebuilt on the parameters' device), and a parameter whose
    gradient first appears later starts at t = 0, as in torch.  Compared with torch.optim.Adam doing the same."""
    from dmayolo.optim import FusedAdam
    g = torch.Generator().manual_seed(5)
    a0, b0 = torch.randn(5000, generator=g), torch.randn(300, generator=g)
    a, b = torch.nn.Parameter(a0.cuda()), torch.nn.Parameter(b0.cuda())
    ra, rb = torch.nn.Parameter(a0.clone()), torch.nn.Parameter(b0.clone())
    opt = FusedAdam([a, b], lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-4)
    ref = torch.optim.Adam([ra, rb], lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-4)
    grads = [(torch.randn(5000, generator=g), torch.randn(300, generator=g)) for _ in range(6)]
    for i in range(3):  # b has no gradient for the first 2 steps
        ga, gb = grads[i]
        a.grad, ra.grad = ga.cuda(), ga.clone()
        b.grad, rb.grad = (gb.cuda(), gb.clone()) if i >= 2 else (None, None)
        opt.step()
        ref.step()
    sd = opt.state_dict()
    assert all('_dstep' not in grp for grp in sd['param_groups'])
    for st in sd['state'].values():
        assert st['step'].device.type == 'cpu' and st['step'].dtype == torch.float32
    assert [float(sd['state'][i]['step']) for i in (0, 1)] == [float(ref.state[ra]['step']), float(ref.state[rb]['step'])]
    path = tmp_path / 'opt.pt'
    torch.save({'optimizer': sd}, path)
    loaded = torch.load(path, map_location='cpu', weights_only=True)['optimizer']
    opt2 = FusedAdam([a, b], lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-4)
    opt2.load_state_dict(loaded)
    for st in opt2.state.values():  # torch moves the moments to the parameters' device on load
        st['exp_avg'], st['exp_avg_sq'] = st['exp_avg'].cuda(), st['exp_avg_sq'].cuda()
    for i in range(3, 6):
        ga, gb = grads[i]
        a.grad, ra.grad = ga.cuda(), ga.clone()
        b.grad, rb.grad = gb.cuda(), gb.clone()
        opt2.step()
        ref.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(a.detach().cpu(), ra.detach(), **TOL_ADAM)
    torch.testing.assert_close(b.detach().cpu(), rb.detach(), **TOL_ADAM)
    assert int(opt2.state[a]['step'].cpu()) == 6 and int(opt2.state[b]['step'].cpu()) == 4


def test_fused_adam_member_that_skips_a_step_keeps_its_count():
    """a and b start together (one device counter); b has no gradient in step 3.  torch leaves b's 'step'
    (and so its bias corrections) alone in that step; FusedAdam moves b onto its own copy of the counter before the
    launch, so both parameters and both counts equal torch.optim.Adam's after 5 steps."""
    from dmayolo.optim import FusedAdam
    g = torch.Generator().manual_seed(7)
    a0, b0 = torch.randn(4000, generator=g), torch.randn(500, generator=g)
    a, b = torch.nn.Parameter(a0.cuda()), torch.nn.Parameter(b0.cuda())
    ra, rb = torch.nn.Parameter(a0.clone()), torch.nn.Parameter(b0.clone())
    opt = FusedAdam([a, b], lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-4)
    ref = torch.optim.Adam([ra, rb], lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-4)
    for i in range(5):
        ga, gb = torch.randn(4000, generator=g), torch.randn(500, generator=g)
        a.grad, ra.grad = ga.cuda(), ga.clone()
        b.grad, rb.grad = (None, None) if i == 2 else (gb.cuda(), gb.clone())
        opt.step()
        ref.step()
    torch.cuda.synchronize()
    assert int(opt.state[a]['step'].cpu()) == 5 and int(opt.state[b]['step'].cpu()) == 4
    torch.testing.assert_close(a.detach().cpu(), ra.detach(), **TOL_ADAM)
    torch.testing.assert_close(b.detach().cpu(), rb.detach(), **TOL_ADAM)
