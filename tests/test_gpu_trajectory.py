"""GPU: bf16 training parity over a multi-step trajectory (reference train.py:432-445).

An overfit run -- a few fixed synthetic VisDrone-shaped batches, constant-lr nesterov SGD on train.py's parameter
groups -- by the product (bf16 storage, HIP kernels) and by the oracle in fp32, under the reference's own fp16 autocast
emulation, and under the product's bf16 storage emulation, from one state_dict (tests/trajectory_util.py).  Compared:
the loss curves and the train-mode Detect outputs on the first batch after the last step.  Bounds are fixed numbers
(below) and, in addition, relative to the bf16-storage emulation's own distance from fp32 on the same trajectory.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (yaml, width, depth, img, bs, batches, steps)
CASES = {
    'yolov5s@320': ('yolov5s.yaml', None, None, 320, 8, 2, 120),
    'dma-l@384': ('yolov5l-ca-sppfcspc-bifpn-scconv.yaml', None, None, 384, 4, 2, 120),
}


@pytest.mark.parametrize('case', list(CASES))
def test_bf16_training_trajectory(case):
    import trajectory_util as tu
    from dmayolo.synthetic import HYP_VISDRONE, scaled_hyp
    yml, gw, gd, img, bs, nb, steps = CASES[case]
    nc = 10
    cfg = tu.load_cfg(yml, gw, gd)
    hyp = scaled_hyp(HYP_VISDRONE, nc, img, 3)
    batches = tu.make_batches(nb, bs, img, nc)
    m, sd = tu.product_model(cfg, nc)
    pin_loss, pin_grad = tu.pin_device_oracle(cfg, nc, sd, batches[0], hyp)
    lp, op = tu.product_trajectory(m, batches, hyp, steps)
    lr_, or_ = tu.oracle_trajectory(cfg, nc, sd, batches, hyp, steps, None)
    lh, oh = tu.oracle_trajectory(cfg, nc, sd, batches, hyp, steps, 'fp16')
    lb, ob = tu.oracle_trajectory(cfg, nc, sd, batches, hyp, steps, 'bf16')
    cp, ch, cb = tu.curve_err(lp, lr_), tu.curve_err(lh, lr_), tu.curve_err(lb, lr_)
    ep, eh, eb = tu.out_err(op, or_), tu.out_err(oh, or_), tu.out_err(ob, or_)
    f = lambda v: ' '.join('%.3e' % e for e in v)  # noqa: E731
    q = max(1, steps // 8)
    print(f'{case}: device fp32 oracle vs CPU oracle, step 1: loss {pin_loss:.2e} grad {pin_grad:.2e}\n'
          f'  loss fp32 oracle   first {float(lr_[0]):.4f} last-{q} mean {float(lr_[-q:].mean()):.4f}\n'
          f'  loss product bf16  first {float(lp[0]):.4f} last-{q} mean {float(lp[-q:].mean()):.4f}  curve err mean '
          f'{cp[0]:.3e} last quarter {cp[1]:.3e}; outputs {f(ep)}\n'
          f'  fp16 autocast emu  last-{q} mean {float(lh[-q:].mean()):.4f}  curve err mean {ch[0]:.3e} last quarter '
          f'{ch[1]:.3e}; outputs {f(eh)}\n'
          f'  bf16 storage emu   last-{q} mean {float(lb[-q:].mean()):.4f}  curve err mean {cb[0]:.3e} last quarter '
          f'{cb[1]:.3e}; outputs {f(eb)}')
    print('  loss curves (every %d steps): fp32 %s\n  product %s\n  fp16 %s\n  bf16 %s' % (
        q, f(lr_[::q].tolist()), f(lp[::q].tolist()), f(lh[::q].tolist()), f(lb[::q].tolist())))
    assert pin_loss < 1e-4 and pin_grad < 1e-3, (pin_loss, pin_grad)
    assert torch.isfinite(lp).all()
    # the run learns: the last eighth's mean loss is well under the first step's, for product and oracle alike
    assert float(lr_[-q:].mean()) < 0.7 * float(lr_[0])
    assert float(lp[-q:].mean()) < 0.7 * float(lp[0])
