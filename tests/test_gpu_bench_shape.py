"""The bench's own configuration end to end: full-width models at the bench resolutions, bf16 HIP product (v3 LDS-DMA
convs at these M, split-K weight-grads into the gradient arena, s2d stem, one-launch weight prep, GradSinks) against
the fp32 CPU oracle on the same state_dict, images and targets.

Compared: the three Detect outputs, the loss and its items (ComputeLoss, utils/loss.py:167-218), the vector of
per-parameter gradient norms and the direction of the whole gradient.  At random init these BN networks lose a large
part of the gradient direction to 8-bit-mantissa storage alone, so fixed fp32-style bounds do not apply; the same test
runs the oracle again under tests/precision_emu.py's emulation of the product's storage ('bf16': every stored
activation and its gradient, the conv / linear weight copies and the stored composite outputs rounded to bf16) and
holds the product to that run's error, with fixed factors:
  outputs relative L2 per level        <= 1.1 * emu + 2e-3
  loss relative                        <= 1.1 * emu + 5e-3 ; items relative <= 1.1 * emu + 1e-2 each
  grads  relative L2 of the whole gradient            <= 1.1 * emu + 1e-2
         median over the top-level layers of (product layer error / emulation layer error) <= 1.1
         cosine(product, fp32 oracle) >= cosine(emu, fp32 oracle) - 0.08: at these shapes the rounding noise is as large
         as the gradient itself (whole-gradient relative L2 ~0.9-1.0 for the emulation too), so the cosine moves with
         the noise REALIZATION -- two product builds that differ only in the fp32 summation order of the BN partials
         (the 1x1 register-epilogue GEMM on / off, round 3) measured cos 0.506 / 0.566 on DMA-YOLO-l @1536 bs2
         relative L2 of the per-parameter grad-norm vector <= 3 * emu + 2e-2 (a loose sanity bound: at random init the
         per-tensor rounding noise is ~50 % of the signal in BOTH runs, so single tensors' norms swing by several % with
         how that noise happens to correlate -- yolov5s @640: the product's stride-2 conv weights 5.8 % off in norm vs
         the emulation's 1.4 %, while its per-layer errors are 15-35 % BELOW the emulation's; tools/gpu/diag_precision.py)
Round 3 measured (tools/gpu/diag_precision.py): the product sits ON the bf16 storage floor -- DMA-YOLO-l
@1536 bs2 outputs 3.33/3.69/4.08e-2 vs emu 3.31/3.70/4.05e-2, grad-norm vector 1.83e-2 vs 1.80e-2, cos 0.5655 vs
0.5682 -- the 1.5x "excess" of round 2 was the earlier emulation's missing roundings (bf16 weight copies, residual
sums).  The reference itself trains under CUDA autocast (fp16 activations, train.py:434); its emulation ('fp16') is
run and printed too: about 7x closer to fp32 than bf16 storage (cos 0.976 vs 0.566 on DMA-YOLO-l), which the test
asserts as a documented property of the two formats, not of the product.
"""
import os

import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu
CFG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'dma-yolo_amd', 'dmayolo', 'configs')


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _oracle_grads(yml, nc, sd, x, t, anchors, hyp, mode):
    from precision_emu import oracle_run
    return oracle_run(os.path.join(CFG, yml), nc, sd, x, t, anchors, hyp, mode)


@pytest.mark.parametrize('yml,img,bs', [('yolov5s.yaml', 640, 64),
                                        ('yolov5l-ca-sppfcspc-bifpn-scconv.yaml', 1536, 2)])
def test_bench_shape_bf16_vs_oracle(yml, img, bs):
    from dmayolo.models.yolo import Model
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    nc = 10
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, yml), nc=nc, act_dtype=torch.bfloat16)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    for mod in m.modules():
        if type(mod).__name__ == 'SwinTransformerLayer':
            mod.drop_path = torch.nn.Identity()
    hyp = scaled_hyp(HYP_VISDRONE, nc, img, 3)
    m.hyp = hyp
    m = m.cuda().train()
    x = images(bs, img, seed=1)
    t = targets(bs, nc, seed=1)
    anchors = m.model[-1].anchors.cpu()

    p = m(x.cuda())
    loss, items = ComputeLoss(m)(p, t.cuda())
    loss.backward()
    ref, pr, lr_, ir_ = _oracle_grads(yml, nc, sd, x, t, anchors, hyp, None)
    emu, pe_, le_, ie_ = _oracle_grads(yml, nc, sd, x, t, anchors, hyp, 'bf16')
    h16, ph_, lh_, ih_ = _oracle_grads(yml, nc, sd, x, t, anchors, hyp, 'fp16')

    def errs(po, lo, io, pg):
        out = [_rel(a.detach().float().cpu(), b.detach()) for a, b in zip(po, pr)]
        le = abs(float(lo) - float(lr_)) / abs(float(lr_))
        ie = [abs(float(a) - float(b)) / max(abs(float(b)), 1e-12) for a, b in zip(io.cpu(), ir_)]
        gn = torch.tensor([float(pg[k].grad.norm()) if pg[k].grad is not None else 0.0 for k in names], dtype=torch.float64)
        g = torch.cat([pg[k].grad.double().cpu().flatten() for k in names])
        layers = {}  # per top-level layer: relative L2 of its concatenated parameter gradients
        for lid in sorted({int(k.split('.')[1]) for k in names}):
            ks = [k for k in names if int(k.split('.')[1]) == lid]
            layers[lid] = _rel(torch.cat([pg[k].grad.double().cpu().flatten() for k in ks]),
                               torch.cat([pq[k].grad.double().flatten() for k in ks]))
        return out, le, ie, (_rel(gn, gn_b), _rel(g, gb), layers), float(g @ gb / (g.norm() * gb.norm()))

    pq = dict(ref.named_parameters())
    names = [k for k in pq if pq[k].grad is not None]
    gn_b = torch.tensor([float(pq[k].grad.norm()) for k in names], dtype=torch.float64)
    gb = torch.cat([pq[k].grad.double().flatten() for k in names])
    out_err, loss_err, item_err, gn_err, cos = errs(p, loss, items, dict(m.named_parameters()))
    e_out, e_loss, e_item, e_gn, e_cos = errs(pe_, le_, ie_, dict(emu.named_parameters()))
    h_out, h_loss, h_item, h_gn, h_cos = errs(ph_, lh_, ih_, dict(h16.named_parameters()))
    f = lambda v: ['%.2e' % e for e in v]  # noqa: E731
    print(f'{yml}@{img} bs{bs} product: outputs {f(out_err)} loss {loss_err:.2e} items {f(item_err)} grad-norm vector '
          f'{gn_err[0]:.2e} whole gradient {gn_err[1]:.2e} cos {cos:.4f}\n  bf16-storage emulation: outputs {f(e_out)} loss '
          f'{e_loss:.2e} items {f(e_item)} grad-norm vector {e_gn[0]:.2e} whole gradient {e_gn[1]:.2e} cos {e_cos:.4f}\n'
          f'  fp16 autocast emulation (the reference): outputs {f(h_out)} loss {h_loss:.2e} grad-norm vector '
          f'{h_gn[0]:.2e} whole gradient {h_gn[1]:.2e} cos {h_cos:.4f}')
    for a, e in zip(out_err, e_out):
        assert a <= 1.1 * e + 2e-3, (out_err, e_out)
    assert loss_err <= 1.1 * e_loss + 5e-3, (loss_err, e_loss)
    for a, e in zip(item_err, e_item):
        assert a <= 1.1 * e + 1e-2, (item_err, e_item)
    ratios = sorted(gn_err[2][i] / max(e_gn[2][i], 1e-12) for i in gn_err[2])
    med = ratios[len(ratios) // 2]
    print(f'  per-layer gradient error product / emulation: median {med:.3f}, range {ratios[0]:.3f}..{ratios[-1]:.3f}')
    assert gn_err[1] <= 1.1 * e_gn[1] + 1e-2, (gn_err[:2], e_gn[:2])
    assert med <= 1.1, ratios
    assert gn_err[0] <= 3.0 * e_gn[0] + 2e-2, (gn_err[:2], e_gn[:2])
    assert cos >= e_cos - 0.08, (cos, e_cos)
    # the formats themselves: fp16 storage (10-bit mantissa) keeps the gradient direction much better than bf16 (7)
    assert h_cos > e_cos and max(h_out) < min(e_out), (h_cos, e_cos, h_out, e_out)
