"""GPU: bf16 training parity over a multi-step trajectory (reference train.py:432-445).

An overfit run -- a few fixed synthetic VisDrone-shaped batches, constant-lr nesterov SGD on train.py's parameter
groups -- by the product (bf16 storage, HIP kernels) and by the oracle in fp32, under the reference's own fp16 autocast
emulation, and under the product's bf16 storage emulation, from one state_dict (tests/trajectory_util.py).  Compared:
the loss curves (mean relative distance from the fp32 curve over all steps) and the train-mode Detect outputs on the
first batch after the last step (relative L2 per level).  Bounds are fixed numbers and, in addition, relative to the
emulations' own distance from fp32 on the same trajectory (see the asserts).  Measured (round 4, profiles/r04):
yolov5s@320 product curve 4.3e-2 vs fp16 3.6e-2 / bf16 5.0e-2 / bf16_sink 4.0e-2, outputs 0.16-0.21 vs fp16 0.16-0.19;
DMA-YOLO-l@384 product curve 2.8e-2 vs 3.3e-2 / 5.7e-2 / 4.4e-2, outputs 0.15-0.16 vs fp16 0.15-0.16: over a training
run the bf16 product tracks the fp32 oracle as closely as the reference's own fp16 autocast does.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (yaml, width, depth, img, bs, batches, steps, nc, fp8, learn: last-eighth loss / first-step loss must be below)
CASES = {
    'yolov5s@320': ('yolov5s.yaml', None, None, 320, 8, 2, 120, 10, False, 0.7),
    'dma-l@384': ('yolov5l-ca-sppfcspc-bifpn-scconv.yaml', None, None, 384, 4, 2, 120, 10, False, 0.7),
    # BASELINE config 5's fp8 leg: every eligible conv forward on the e4m3 kernel (delayed activation scaling from the
    # second step on), bf16 backward; its own emulation is precision_emu 'fp8'
    'c5-fp8@256': ('yolov5l-xs-tr-cbam-spp-bifpn.yaml', None, None, 256, 4, 2, 100, 3, True, 0.95),
}


@pytest.mark.parametrize('case', list(CASES))
def test_bf16_training_trajectory(case):
    import trajectory_util as tu
    from dmayolo.synthetic import HYP_VISDRONE, scaled_hyp
    yml, gw, gd, img, bs, nb, steps, nc, fp8, learn = CASES[case]
    cfg = tu.load_cfg(yml, gw, gd)
    batches = tu.make_batches(nb, bs, img, nc)
    m, sd = tu.product_model(cfg, nc, fp8=fp8)
    hyp = scaled_hyp(HYP_VISDRONE, nc, img, m.model[-1].nl)
    pin_loss, pin_out, pin_grad = tu.pin_device_oracle(cfg, nc, sd, batches[0], hyp)
    with tu.deterministic():
        lp, op = tu.product_trajectory(m, batches, hyp, steps)
        lr_, or_ = tu.oracle_trajectory(cfg, nc, sd, batches, hyp, steps, None)
        lh, oh = tu.oracle_trajectory(cfg, nc, sd, batches, hyp, steps, 'fp16')
        lb, ob = tu.oracle_trajectory(cfg, nc, sd, batches, hyp, steps, 'fp8' if fp8 else 'bf16')
        ls, os_ = tu.oracle_trajectory(cfg, nc, sd, batches, hyp, steps, 'bf16' if fp8 else 'bf16_sink')
    # the shipped default mode as well (fp32 atomics in the split-K / fused 1x1 weight-grads, a run-dependent summation
    # order): one more product realization of the same trajectory from the same initial state
    ld = od = None
    if not fp8:
        md, _ = tu.product_model(cfg, nc)
        ld, od = tu.product_trajectory(md, batches, hyp, steps)
    cp, ch, cb, cs = tu.curve_err(lp, lr_), tu.curve_err(lh, lr_), tu.curve_err(lb, lr_), tu.curve_err(ls, lr_)
    ep, eh, eb, es = tu.out_err(op, or_), tu.out_err(oh, or_), tu.out_err(ob, or_), tu.out_err(os_, or_)
    f = lambda v: ' '.join('%.3e' % e for e in v)  # noqa: E731
    q = max(1, steps // 8)
    print(f'{case}: device fp32 oracle vs CPU oracle, step 1: loss {pin_loss:.2e} outputs {pin_out:.2e} grad '
          f'{pin_grad:.2e}\n'
          f'  loss fp32 oracle   first {float(lr_[0]):.4f} last-{q} mean {float(lr_[-q:].mean()):.4f}\n'
          f'  loss product bf16  first {float(lp[0]):.4f} last-{q} mean {float(lp[-q:].mean()):.4f}  curve err mean '
          f'{cp[0]:.3e} last quarter {cp[1]:.3e}; outputs {f(ep)}\n'
          f'  fp16 autocast emu  last-{q} mean {float(lh[-q:].mean()):.4f}  curve err mean {ch[0]:.3e} last quarter '
          f'{ch[1]:.3e}; outputs {f(eh)}\n'
          f'  {"fp8 e4m3 fwd emu " if fp8 else "bf16 storage emu "}  last-{q} mean {float(lb[-q:].mean()):.4f}  curve err mean {cb[0]:.3e} last quarter '
          f'{cb[1]:.3e}; outputs {f(eb)}\n'
          f'  {"bf16 storage emu " if fp8 else "bf16_sink emu    "}  last-{q} mean {float(ls[-q:].mean()):.4f}  curve err mean {cs[0]:.3e} last quarter '
          f'{cs[1]:.3e}; outputs {f(es)}')
    print('  loss curves (every %d steps): fp32 %s\n  product %s\n  fp16 %s\n  bf16 %s\n  bf16_sink %s' % (
        q, f(lr_[::q].tolist()), f(lp[::q].tolist()), f(lh[::q].tolist()), f(lb[::q].tolist()),
        f(ls[::q].tolist())))
    # the device-run oracle against the CPU one, both in float64 (round 5 measured: outputs 5e-14 .. 4.3e-9, gradient
    # 6e-13 .. 8.2e-8): the same function, not just the same function up to fp32 summation order
    assert pin_loss < 1e-6 and pin_out < 1e-6 and pin_grad < 1e-5, (pin_loss, pin_out, pin_grad)
    assert torch.isfinite(lp).all()
    # the run learns: the last eighth's mean loss is well under the first step's, for product and oracle alike
    assert float(lr_[-q:].mean()) < learn * float(lr_[0])
    assert float(lp[-q:].mean()) < learn * float(lp[0])
    # fixed bounds (round 4 measured, two box runs: yolov5s curve err 4.3-4.4e-2, outputs 0.16-0.21; DMA-YOLO-l 2.8e-2,
    # 0.15-0.16) and relative ones: the product is no further from the fp32 trajectory than 2x the furthest of the
    # three storage emulations (fp16 autocast = the reference's precision, bf16, bf16_sink), whose own spread between
    # realizations is about that wide (chaotic divergence of 120 SGD steps)
    emu_curve = max(ch[0], cb[0], cs[0])
    assert cp[0] <= 0.08 and cp[0] <= 2.0 * emu_curve, (cp, emu_curve)
    # outputs: every level <= 0.3 and <= 1.5 x the furthest emulation's at that level + 0.01 (both trajectories are
    # deterministic now, tu.deterministic: round 4 had summed the levels because one run's level 0 had moved 4x between
    # runs of the same code -- the fp32 oracle's own loss curve moved with it, its backward summing with atomics)
    emu_out = [max(eh[lvl], eb[lvl], es[lvl]) for lvl in range(len(ep))]
    assert max(ep) <= 0.3 and all(a <= 1.5 * e + 0.01 for a, e in zip(ep, emu_out)), (ep, emu_out)
    # the final loss level (last eighth) within 8 % of the fp32 oracle's
    assert abs(float(lp[-q:].mean()) / float(lr_[-q:].mean()) - 1) <= 0.08
    if ld is not None:
        # the default-mode realization: a different chaotic realization of the same run, so a little more room than the
        # deterministic one (which the bounds above were fixed on), the same kind of bound
        cd, ed = tu.curve_err(ld, lr_), tu.out_err(od, or_)
        print(f'  product default mode: curve err mean {cd[0]:.3e} last quarter {cd[1]:.3e}; outputs {f(ed)}; '
              f'last-{q} mean {float(ld[-q:].mean()):.4f}')
        assert torch.isfinite(ld).all() and float(ld[-q:].mean()) < learn * float(ld[0])
        assert cd[0] <= 0.1 and cd[0] <= 2.5 * emu_curve, (cd, emu_curve)
        assert max(ed) <= 0.35 and all(a <= 2.0 * e + 0.01 for a, e in zip(ed, emu_out)), (ed, emu_out)
        assert abs(float(ld[-q:].mean()) / float(lr_[-q:].mean()) - 1) <= 0.1
