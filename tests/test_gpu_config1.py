"""BASELINE.json config 1 as stated: models/yolov5n.yaml, nc=80 (coco128's class count), @640, batch 1, the scratch
hyperparameters (data/hyps/hyp.scratch.yaml, gains scaled as train.py:330-335), fp32.

The reference runs this config with `train.py --device cpu`; the CPU leg here is the oracle (oracle/nn.py +
oracle/loss.py, pinned by the model_v5s / loss_scratch goldens).  The HIP product (fp32 storage: exact-fp32 MFMA convs,
split-K weight-gradients, the s2d stem, ComputeLoss kernels) must reproduce the oracle on the same state_dict, image
and targets:
  Detect train outputs      rtol 1e-3 / atol 1e-3 (fp32 summation order through ~25 conv layers)
  loss, items               rtol 1e-4
  every parameter gradient  relative L2 <= 2e-3 per tensor, floor 1e-4 * sqrt(numel) (the exactly-zero gradients of
                            conv biases feeding a train-mode BN are rounding noise in both)
  eval (decoded) output     rtol 1e-3 / atol 2e-3 (after the train step's running-stat update, on both sides)
and, at batch 1, the Trainer's accumulate (64, train.py:190 / 408-422) and one FusedSGD step must equal
train.py:216-222's torch.optim.SGD over the same groups / lr / momentum / weight decay / gradients."""
import os

import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu
CFG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'dma-yolo_amd', 'dmayolo', 'configs')
NC, IMG, BS = 80, 640, 1


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(float(b.norm()), 1e-4 * b.numel() ** 0.5))


def test_config1_yolov5n_nc80_640_bs1_fp32_vs_oracle():
    from oracle import nn as onn
    from oracle.loss import compute_loss
    from dmayolo.models.yolo import Model
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.synthetic import images, targets, HYP_SCRATCH, scaled_hyp
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, 'yolov5n.yaml'), nc=NC, act_dtype=torch.float32)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    hyp = scaled_hyp(HYP_SCRATCH, NC, IMG, 3)
    m.hyp = hyp
    m = m.cuda().train()
    x = images(BS, IMG, seed=1)
    t = targets(BS, NC, seed=1)
    anchors = m.model[-1].anchors.cpu()

    p = m(x.cuda())
    loss, items = ComputeLoss(m)(p, t.cuda())
    loss.backward()

    with open(os.path.join(CFG, 'yolov5n.yaml')) as f:
        ref = onn.bn_defaults(onn.Model(yaml.safe_load(f), nc=NC))
    ref.load_state_dict(sd)
    ref.train()
    pr = ref(x.float() / 255)
    lr_, ir_ = compute_loss(pr, t, anchors, hyp, NC)
    lr_.backward()

    for a, b in zip(p, pr):
        assert a.shape == b.shape == (BS, 3, b.shape[2], b.shape[3], NC + 5)
        torch.testing.assert_close(a.detach().float().cpu(), b.detach(), rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(loss.detach().cpu().view(-1), lr_.detach().view(-1), rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(items.cpu(), ir_.detach(), rtol=1e-4, atol=1e-7)
    pg, rg = dict(m.named_parameters()), dict(ref.named_parameters())
    assert set(pg) == set(rg)
    errs = {k: _rel(pg[k].grad.cpu(), rg[k].grad) for k in rg if rg[k].grad is not None}
    assert len(errs) == len(rg)
    worst = max(errs.items(), key=lambda kv: kv[1])
    print(f'config 1: loss {float(loss):.6f} vs {float(lr_):.6f}; {len(errs)} grads, worst rel L2 {worst[1]:.2e} ({worst[0]})')
    assert worst[1] <= 2e-3, worst

    # running statistics after the train forward, then the decoded eval output
    for k, v in ref.state_dict().items():
        if 'running' in k:
            torch.testing.assert_close(m.state_dict()[k].cpu(), v, rtol=1e-4, atol=1e-6, msg=lambda s: f'{k}: {s}')
    m.eval()
    ref.eval()
    with torch.no_grad():
        z, _ = m(x.cuda())
        zr, _ = ref(x.float() / 255)
    assert z.shape == zr.shape == (BS, 25200, NC + 5)
    torch.testing.assert_close(z.cpu(), zr, rtol=1e-3, atol=2e-3)


def test_config1_batch1_accumulate_and_sgd_step_match_torch_optim():
    """train.py:197-222 (three groups: BN weights no decay, weights with decay, biases) + one SGD step (nesterov,
    momentum from hyp) through the product's GradScaler + FusedSGD vs torch.optim.SGD on the same (unscaled) gradients,
    at the nc=80 yolov5n parameter set."""
    from dmayolo.models.yolo import Model
    from dmayolo.trainer import Trainer
    from dmayolo.synthetic import images, targets, HYP_SCRATCH, scaled_hyp
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, 'yolov5n.yaml'), nc=NC, act_dtype=torch.float32).cuda().train()
    m.hyp = scaled_hyp(HYP_SCRATCH, NC, IMG, 3)
    tr = Trainer(m, m.hyp, BS, nb=128, ema=False)  # batch 1: accumulate = 64 (train.py:190) -> no step inside warmup
    assert tr.accumulate == 64
    tr.i = 1000  # end of warmup (nw = max(3 * 128, 1000)): accumulate back to 64, lr at lr0 * lf(0)
    tr.warmup(tr.ni)
    assert tr.accumulate == 64
    x = images(BS, IMG, seed=1, device='cuda')
    t = targets(BS, NC, seed=1, device='cuda')
    before = {k: v.detach().clone() for k, v in m.named_parameters()}
    loss, _ = tr.compute_loss(m(x), t)
    loss.backward(tr.scaler.upstream)
    grads = {k: v.grad.detach().clone() for k, v in m.named_parameters()}
    tr.scaler.step(tr.optimizer)
    # reference optimizer on CPU over the same groups / hyperparameters
    params = {k: before[k].cpu().clone().requires_grad_(True) for k in before}
    pid = {id(p): k for k, p in m.named_parameters()}
    ref_groups = []
    for g in tr.optimizer.param_groups:
        names = [pid[id(p)] for p in g['params']]
        ref_groups.append(dict(params=[params[k] for k in names], lr=g['lr'], momentum=g['momentum'],
                               weight_decay=g['weight_decay'], nesterov=g['nesterov']))
    opt = torch.optim.SGD(ref_groups, lr=ref_groups[0]['lr'])
    scale = float(tr.scaler.scale.cpu())  # world 1: upstream == scale; the fused update unscales by it
    for k, p in params.items():
        p.grad = grads[k].cpu() / scale
    opt.step()
    assert len(ref_groups) == 3
    for k, v in m.named_parameters():
        torch.testing.assert_close(v.detach().cpu(), params[k].detach(), rtol=1e-6, atol=1e-7, msg=lambda s: f'{k}: {s}')
