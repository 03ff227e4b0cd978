"""Multi-step training trajectories (test infrastructure, used by test_gpu_trajectory.py and tools/gpu/diag_trajectory.py).

VERDICT r3 item 1: at random init the single-step gradient of these BN networks is dominated by storage-rounding noise,
so a one-step comparison cannot tell a kernel bias from bf16 noise.  An overfit trajectory can: a few fixed synthetic
batches, `steps` SGD steps (train.py's optimizer: nesterov SGD over the g0 / g1 / g2 groups of train.py:197-222, weight
decay on g1 only, constant lr -- no warmup, so the loss actually falls within the run), run

  * by the product (bf16 storage, HIP kernels, FusedSGD + the device GradScaler, as bench.py's step), and
  * by the oracle (oracle/nn.py + oracle/loss.py) in fp32, and under tests/precision_emu.py's emulations: 'fp16' (the
    reference's own CUDA-autocast training precision, train.py:432-445, with its 2^16 loss scale) and 'bf16' (the
    product's storage model),

all from the same state_dict on the same batches.  The oracle's plain-torch ops run on the GPU in fp32 for these
trajectories (TF32 off); `pin_device_oracle` checks that device run against the CPU oracle on the first step.
"""
import os

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs')
LR, MOM, WD = 0.01, 0.937, 5e-4  # data/hyps/hyp.scratch.yaml lr0 / momentum / weight_decay (train.py:216-222)


def groups(model):
    """train.py:197-214 on any module tree: g0 BN weights (no decay), g1 weights + AdConcat.w (decay), g2 biases"""
    g0, g1, g2 = [], [], []
    for v in model.modules():
        if isinstance(getattr(v, 'bias', None), nn.Parameter):
            g2.append(v.bias)
        if isinstance(v, nn.BatchNorm2d):
            g0.append(v.weight)
        elif isinstance(getattr(v, 'weight', None), nn.Parameter):
            g1.append(v.weight)
        elif isinstance(getattr(v, 'w', None), nn.Parameter):
            g1.append(v.w)
    return g0, g1, g2


def _no_drop(model):
    for mod in model.modules():
        if hasattr(mod, 'drop_prob'):
            mod.drop_prob = 0.0
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
        if type(mod).__name__ == 'SwinTransformerLayer' and hasattr(mod, 'drop_path'):
            mod.drop_path = nn.Identity()
    return model


def load_cfg(yml, width=None, depth=None):
    import yaml
    with open(os.path.join(CFG, yml)) as f:
        cfg = yaml.safe_load(f)
    if width is not None:
        cfg['width_multiple'], cfg['depth_multiple'] = width, depth
    return cfg


def make_batches(nb, bs, img, nc, per_image=20):
    from dmayolo.synthetic import images, targets
    return [(images(bs, img, seed=11 + i), targets(bs, nc, per_image=per_image, seed=11 + i)) for i in range(nb)]


def product_model(cfg, nc, seed=0, fp8=False):
    """the bf16 product Model (fp8: functional.set_fp8, config 5's e4m3 forward) and its initial state_dict.  `anchors: N`
    placeholders (config 5) get fixed anchors, as tests/test_gpu_fp8.py pins them."""
    import dmayolo.functional as Fn
    from dmayolo.models.yolo import Model
    torch.manual_seed(seed)
    m = Model(cfg, nc=nc, act_dtype=torch.bfloat16)
    if isinstance(cfg.get('anchors'), int):
        det = m.model[-1]
        det.anchors[:] = torch.tensor([[10, 13], [16, 30], [33, 23], [30, 61]], dtype=torch.float32).view(1, 4, 2) \
            / det.stride.view(-1, 1, 1) * torch.tensor([1.0, 2.0, 4.0, 8.0]).view(-1, 1, 1)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    if fp8:
        assert Fn.set_fp8(m, True) >= 10
    return _no_drop(m), sd


class deterministic:
    """context: run-to-run identical trajectories.  The product in its deterministic mode (functional.set_deterministic:
    the split-K and fused-backward weight gradients through workspaces summed in a fixed order instead of fp32 atomics)
    and torch's deterministic algorithms for the oracle's GPU ops (warn_only: adaptive_max_pool2d's backward has no
    deterministic kernel, measured bit-identical across runs all the same, profiles/r05/traj_determinism.log).  Both
    curves being fixed, the trajectory bounds need no allowance for either side's run-to-run noise."""

    def __enter__(self):
        from dmayolo import functional as fn
        os.environ.setdefault('CUBLAS_WORKSPACE_CONFIG', ':4096:8')
        self.prev = (fn.DETERMINISTIC[0], torch.are_deterministic_algorithms_enabled(),
                     torch.is_deterministic_algorithms_warn_only_enabled())
        fn.set_deterministic(True)
        torch.use_deterministic_algorithms(True, warn_only=True)
        return self

    def __exit__(self, *a):
        from dmayolo import functional as fn
        fn.set_deterministic(self.prev[0])
        torch.use_deterministic_algorithms(self.prev[1], warn_only=self.prev[2])


def product_trajectory(m, batches, hyp, steps, probe=0):
    """bench.py's training step (forward, ComputeLoss, backward seeded by the GradScaler, FusedSGD) for `steps` steps
    over the batches in turn; returns (losses [steps], train-mode outputs on batches[probe] after the last step)"""
    from dmayolo.optim import build_optimizer, GradScaler
    from dmayolo.utils.loss import ComputeLoss
    m = m.cuda().train()
    m.hyp = hyp
    cl = ComputeLoss(m)
    opt = build_optimizer(m, 'sgd', LR, MOM, WD)
    scaler = GradScaler(torch.device('cuda'))
    dev = [(x.cuda(), t.cuda()) for x, t in batches]
    losses = []
    for i in range(steps):
        x, t = dev[i % len(dev)]
        loss, _ = cl(m(x), t)
        loss.backward(scaler.upstream)
        scaler.step(opt)
        scaler.update()
        opt.zero_grad(set_to_none=True)
        losses.append(loss.detach().reshape(1))
        if i % 40 == 39:
            print(f'  product step {i + 1}/{steps}', flush=True)
    with torch.no_grad():
        out = [o.float() for o in m(dev[probe][0])]
    return torch.cat(losses).double().cpu(), [o.cpu() for o in out]


class _TargetCache:
    """oracle.loss.build_targets depends only on the level shapes, the targets and the anchors: the trajectories reuse
    a few fixed batches, so the (python-loop) matching runs once per batch"""

    def __init__(self):
        from oracle import loss as ol
        self.ol, self.orig, self.memo = ol, ol.build_targets, {}

    def __enter__(self):
        def cached(shapes, targets, anchors, anchor_t):
            k = (tuple(tuple(s) for s in shapes), targets.data_ptr(), anchors.data_ptr(), float(anchor_t))
            if k not in self.memo:
                self.memo[k] = self.orig(shapes, targets, anchors, anchor_t)
            return self.memo[k]
        self.ol.build_targets = cached
        return self

    def __exit__(self, *a):
        self.ol.build_targets = self.orig


def oracle_model(cfg, nc, sd, mode, dev):
    from oracle import nn as onn
    from precision_emu import emulate
    ref = onn.bn_defaults(onn.Model(cfg, nc=nc))
    ref.load_state_dict(sd)
    _no_drop(ref)
    if mode is not None:
        emulate(ref, mode)
    return ref.to(dev).train()


def oracle_trajectory(cfg, nc, sd, batches, hyp, steps, mode=None, dev='cuda', probe=0):
    """the same trajectory on the oracle (fp32, or emulation `mode`); the loss (oracle/loss.py) runs on the CPU over
    the level outputs copied back; returns (losses [steps], outputs on batches[probe] after the last step)"""
    from oracle.loss import compute_loss
    from precision_emu import input_round, LOSS_SCALE
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    ref = oracle_model(cfg, nc, sd, mode, dev)
    anchors = sd['model.%d.anchors' % (len(ref.model) - 1)].float().cpu()
    g0, g1, g2 = groups(ref)
    opt = torch.optim.SGD(g0, lr=LR, momentum=MOM, nesterov=True)
    opt.add_param_group({'params': g1, 'weight_decay': WD})
    opt.add_param_group({'params': g2})
    sc = LOSS_SCALE[mode] if mode else 1.0
    xs = [(input_round(x.to(dev).float() / 255, mode), t) for x, t in batches]
    losses = []
    with _TargetCache():
        for i in range(steps):
            x, t = xs[i % len(xs)]
            pr = ref(x)
            lo, _ = compute_loss([p.cpu() for p in pr], t, anchors, hyp, nc)
            opt.zero_grad(set_to_none=True)
            (lo * sc).backward()
            if sc != 1.0:
                for p in ref.parameters():
                    if p.grad is not None:
                        p.grad.div_(sc)
            opt.step()
            losses.append(float(lo))
            if i % 40 == 39:
                print(f'  oracle ({mode or "fp32"}) step {i + 1}/{steps}', flush=True)
    with torch.no_grad():
        out = [o.float().cpu() for o in ref(xs[probe][0])]
    return torch.tensor(losses, dtype=torch.float64), out


def pin_device_oracle(cfg, nc, sd, batch, hyp, dtype=torch.float64):
    """first step of the device-run oracle vs the CPU oracle, both in float64 (default): (loss rel err, max
    Detect-output rel L2, whole-grad rel L2).  In fp64 the two summation orders agree to ~1e-12, so this pins that the
    device run computes the same FUNCTION as the CPU oracle (in fp32 the same comparison measured only
    summation order, 1e-4 .. 1.6e-4 on the outputs and up to 1e-1 on the gradient through max-pool / CBAM near-ties).
    The loss restatement (oracle/loss.py) returns fp32 whatever its inputs, so its pin is at fp32 resolution."""
    from oracle.loss import compute_loss
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    res = []
    for dev in ('cpu', 'cuda'):
        ref = oracle_model(cfg, nc, sd, None, dev).to(dtype)
        anchors = sd['model.%d.anchors' % (len(ref.model) - 1)].to(dtype).cpu()
        x, t = batch
        pr = ref(x.to(dev).to(dtype) / 255)
        lo, _ = compute_loss([p.cpu() for p in pr], t, anchors, hyp, nc)
        lo.backward()
        res.append((float(lo), [p.detach().double().cpu() for p in pr],
                    torch.cat([p.grad.double().cpu().flatten() for p in ref.parameters() if p.grad is not None])))
    (lc, oc, gc), (lg, og, gg) = res
    return (abs(lg - lc) / abs(lc), max(float((a - b).norm() / b.norm()) for a, b in zip(og, oc)),
            float((gg - gc).norm() / gc.norm()))


def curve_err(a, b):
    """loss-curve distance: mean over steps of |a - b| / b, and the same over the last quarter"""
    r = (a - b).abs() / b.abs()
    return float(r.mean()), float(r[-max(1, len(r) // 4):].mean())


def out_err(po, ro):
    return [float((a.double() - b.double()).norm() / b.double().norm()) for a, b in zip(po, ro)]
