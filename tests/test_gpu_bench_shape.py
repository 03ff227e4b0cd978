"""The bench's own configuration end to end: full-width models at the bench resolutions, bf16 HIP product (v3 LDS-DMA
convs at these M, split-K weight-grads into the gradient arena, s2d stem, one-launch weight prep, GradSinks) against
the fp32 oracle on the same state_dict, images and targets.

Compared: the three Detect outputs, the loss and its items (ComputeLoss, utils/loss.py:167-218), the vector of
per-parameter gradient norms and the direction of the whole gradient.  At random init these BN networks lose a large
part of the gradient direction to 8-bit-mantissa storage alone, so fixed fp32-style bounds do not apply; the oracle is
run again under tests/precision_emu.py's emulation of the product's storage ('bf16': every stored activation and its
gradient, the conv / linear weight copies and the stored composite outputs rounded to bf16) in several realizations --
the state_dict as is, and with the weights moved by one fp32 ulp -- and the product is held to their envelope:
  outputs relative L2 per level <= 1.1 * env + 2e-3 ; loss <= 1.5 * env + 5e-3 ; items <= 1.5 * env + 1e-2
  grads  relative L2 of the whole gradient <= 1.1 * env + 1e-2; median over the top-level layers of (product layer
         error / emulation layer error) <= 1.1; per-parameter grad-norm vector <= 1.5 * env + 2e-3;
         cosine(product, fp32) >= min(emulation cosines) - 0.05   (round 2's strictness)
The fp32 oracle and the emulations run their torch ops on the GPU (TF32 off): the same algorithm as the CPU oracle
(pinned to it in float64 by test_gpu_trajectory.py), another fp32 summation order.  A kernel bias is caught by
test_gpu_conv_bench_shapes.py (every conv shape of both bench configs exact to one bf16 rounding), by the per-layer tests
below and by test_gpu_trajectory.py (120-step training runs).  The reference itself trains under CUDA autocast (fp16
activations, train.py:434); its emulation ('fp16') is run and printed too, closer to fp32 than bf16 storage -- asserted
as a documented property of the two formats, not of the product."""
import os

import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu
CFG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'dma-yolo_amd', 'dmayolo', 'configs')


# Configs whose whole-model single-step bf16 gradient at random init is chaotic (round 4, DMA-YOLO-l @1536 bs2,
# gpurun_out r4 dma3 / dma4 / diag_modules logs): layer by layer the product matches the bf16 emulation (input-gradient
# error 1.0-1.6x the emulation's, norms within 2e-4, test_bench_shape_layers_bf16_vs_emulation), the fp32 product
# matches the fp32 oracle to 6.5e-4 (test_bench_shape_fp32_product_vs_oracle), but SPPFCSPC's max-pools route its input
# gradient on near-ties (10.6 % error per module for the emulation itself) and the AdConcat weights' gradients are sums
# over whole feature maps, so the whole-model gradient metrics of the SAME emulation move between runs on one box by
# more than 10x (grad-norm vector 9e-3 .. 1.1e-1, per-layer backbone norms 0.94 .. 1.03 of fp32), and the product's
# slightly higher per-layer noise (GradSink roundings) lands it at 7.5e-2 .. 1.8e-1.
CHAOTIC = ('yolov5l-ca-sppfcspc-bifpn-scconv.yaml',)


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _oracle_grads(yml, nc, sd, x, t, anchors, hyp, mode, dev='cpu'):
    from precision_emu import oracle_run
    return oracle_run(os.path.join(CFG, yml), nc, sd, x, t, anchors, hyp, mode, dev)


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

    def perturbed(seed):  # every float tensor moved by up to one fp32 ulp (relative 2^-24), seeded
        g = torch.Generator().manual_seed(seed)
        return {k: (v * (1 + (torch.rand(v.shape, generator=g) * 2 - 1) * 2.0 ** -24)).to(v.dtype)
                if v.is_floating_point() else v for k, v in sd.items()}

    def product_run(sd_):
        m.load_state_dict(sd_)
        m.zero_grad(set_to_none=True)
        p_ = m(x.cuda())
        lo_, it_ = ComputeLoss(m)(p_, t.cuda())
        lo_.backward()
        return ([o.detach().float().cpu() for o in p_], lo_.detach(), it_,
                {k: q.grad.detach().clone() for k, q in m.named_parameters() if q.grad is not None})

    chaotic = yml in CHAOTIC
    # product realizations: the state_dict as is, and (chaotic configs) ulp-perturbed copies, seeds 1, 2 -- the product
    # decides its bf16 roundings on slightly different fp32 values, exactly as the emulation realizations below do.  An
    # odd count, so the median is one realization
    prods = [product_run(sd)] + ([product_run(perturbed(s_)) for s_ in (1, 2)] if chaotic else [])
    p, loss, items, pgrads = prods[0]
    # the fp32 oracle and its emulations run their torch ops on the GPU (TF32 off; DropPath / dropout off): the CPU runs
    # of round 5 took most of this test's time, and the fp32 order is one more realization of the same sums
    ref, pr, lr_, ir_ = _oracle_grads(yml, nc, sd, x, t, anchors, hyp, None, 'cuda')
    emu, pe_, le_, ie_ = _oracle_grads(yml, nc, sd, x, t, anchors, hyp, 'bf16', 'cuda')
    h16, ph_, lh_, ih_ = _oracle_grads(yml, nc, sd, x, t, anchors, hyp, 'fp16', 'cuda')
    snk, ps_, ls_, is_ = _oracle_grads(yml, nc, sd, x, t, anchors, hyp, 'bf16_sink', 'cuda')
    # more realizations of the emulation, with the weights moved by one fp32 ulp (relative 2^-24 noise, seeds 1..):
    # each decides its bf16 roundings on slightly different fp32 values, as the product's kernels do.  Chaotic configs:
    # 'bf16_sink', the product's own storage model (GradSink roundings), for the distribution comparison
    reals = [_oracle_grads(yml, nc, perturbed(seed), x, t, anchors, hyp, 'bf16_sink' if chaotic else 'bf16', 'cuda')
             for seed in ((1, 2, 3, 4) if chaotic else (1, 2, 3))]

    def errs(po, lo, io, pg):
        """pg: parameter name -> its gradient tensor"""
        out = [_rel(a.detach().float().cpu(), b.detach()) for a, b in zip(po, pr)]
        le = abs(float(lo) - float(lr_)) / abs(float(lr_))
        ie = [abs(float(a) - float(b)) / max(abs(float(b)), 1e-12) for a, b in zip(io.cpu(), ir_)]
        gn = torch.tensor([float(pg[k].norm()) if pg.get(k) is not None else 0.0 for k in names], dtype=torch.float64)
        g = torch.cat([pg[k].double().cpu().flatten() for k in names])
        layers = {}  # per top-level layer: relative L2 of its concatenated parameter gradients
        for lid in sorted({int(k.split('.')[1]) for k in names}):
            ks = [k for k in names if int(k.split('.')[1]) == lid]
            layers[lid] = _rel(torch.cat([pg[k].double().cpu().flatten() for k in ks]),
                               torch.cat([pq[k].grad.double().flatten() for k in ks]))
        return out, le, ie, (_rel(gn, gn_b), _rel(g, gb), layers), float(g @ gb / (g.norm() * gb.norm()))

    def grads_of(mod):
        return {k: q.grad for k, q in mod.named_parameters() if q.grad is not None}

    pq = dict(ref.named_parameters())
    names = [k for k in pq if pq[k].grad is not None]
    gn_b = torch.tensor([float(pq[k].grad.norm()) for k in names], dtype=torch.float64)
    gb = torch.cat([pq[k].grad.double().flatten() for k in names])
    out_err, loss_err, item_err, gn_err, cos = errs(p, loss, items, pgrads)
    perr = [errs(*pr_) for pr_ in prods]
    e_out, e_loss, e_item, e_gn, e_cos = errs(pe_, le_, ie_, grads_of(emu))
    h_out, h_loss, h_item, h_gn, h_cos = errs(ph_, lh_, ih_, grads_of(h16))
    s_out, s_loss, s_item, s_gn, s_cos = errs(ps_, ls_, is_, grads_of(snk))
    rerr = [errs(pp, ll, ii, grads_of(mm)) for mm, pp, ll, ii in reals]
    # envelope over the realizations (CPU one included): worst output / loss / item / gradient metrics, lowest cosine
    r_out = [max(v) for v in zip(*[r[0] for r in rerr])]
    r_loss = max(r[1] for r in rerr)
    r_item = [max(v) for v in zip(*[r[2] for r in rerr])]
    r_gn = (max(r[3][0] for r in rerr), max(r[3][1] for r in rerr))
    r_cos = min(r[4] for r in rerr)
    f = lambda v: ['%.2e' % e for e in v]  # noqa: E731
    print(f'{yml}@{img} bs{bs} product: outputs {f(out_err)} loss {loss_err:.2e} items {f(item_err)} grad-norm vector '
          f'{gn_err[0]:.2e} whole gradient {gn_err[1]:.2e} cos {cos:.4f}\n  bf16-storage emulation: outputs {f(e_out)} loss '
          f'{e_loss:.2e} items {f(e_item)} grad-norm vector {e_gn[0]:.2e} whole gradient {e_gn[1]:.2e} cos {e_cos:.4f}\n'
          f'  fp16 autocast emulation (the reference): outputs {f(h_out)} loss {h_loss:.2e} grad-norm vector '
          f'{h_gn[0]:.2e} whole gradient {h_gn[1]:.2e} cos {h_cos:.4f}\n'
          f'  bf16 storage + per-contribution gradient rounding (bf16_sink): outputs {f(s_out)} loss {s_loss:.2e} '
          f'grad-norm vector {s_gn[0]:.2e} whole gradient {s_gn[1]:.2e} cos {s_cos:.4f}\n'
          + ''.join(f'\n  emulation realization {i + 2} (ulp-perturbed weights): '
                    f'outputs {f(r[0])} loss {r[1]:.2e} grad-norm vector {r[3][0]:.2e} whole gradient {r[3][1]:.2e} cos '
                    f'{r[4]:.4f}' for i, r in enumerate(rerr)))
    sr = sorted(gn_err[2][i] / max(s_gn[2][i], 1e-12) for i in gn_err[2])
    print(f'  per-layer gradient error product / bf16_sink: median {sr[len(sr) // 2]:.3f}, range {sr[0]:.3f}..{sr[-1]:.3f}')
    # bounds: round-2 strictness, against the ENVELOPE of two realizations of the bf16 emulation (CPU fp32 order and
    # GPU fp32 order: the same roundings, decided on sums that differ in the last fp32 bits).  Round 4 measured how far
    # two realizations of the same emulation sit apart on the gradient metrics -- yolov5s grad-norm vector 8.2e-3 vs
    # 1.36e-2, DMA-YOLO-l 1.80e-2 vs 5.54e-2, cosine 0.568 vs 0.619 -- i.e. those metrics measure the noise
    # REALIZATION at random init, and the product (1.94e-2 / 3.47e-2, cos 0.879 / 0.539) lies inside that spread.
    # The conv kernels themselves are exact to one bf16 rounding at every bench shape (test_gpu_conv_bench_shapes.py),
    # and over a training run the product tracks fp32 like the reference's fp16 autocast (test_gpu_trajectory.py).
    env_out = [max(a, b) for a, b in zip(e_out, r_out)]
    for a, e in zip(out_err, env_out):
        assert a <= 1.1 * e + 2e-3, (out_err, env_out)
    assert loss_err <= 1.5 * max(e_loss, r_loss) + 5e-3, (loss_err, e_loss, r_loss)
    for a, e1, e2 in zip(item_err, e_item, r_item):
        assert a <= 1.5 * max(e1, e2) + 1e-2, (item_err, e_item, r_item)
    ratios = sorted(gn_err[2][i] / max(e_gn[2][i], 1e-12) for i in gn_err[2])
    med = ratios[len(ratios) // 2]
    print(f'  per-layer gradient error product / emulation: median {med:.3f}, range {ratios[0]:.3f}..{ratios[-1]:.3f}')
    worst = sorted(gn_err[2], key=lambda i: -gn_err[2][i] / max(e_gn[2][i], 1e-12))[:4]
    print('  worst layers (id: product err / emulation err): ' +
          ', '.join(f'{i}: {gn_err[2][i]:.2e}/{e_gn[2][i]:.2e}' for i in worst))
    # the parameters that carry the grad-norm-vector error: |norm(product grad) - norm(fp32 grad)|, largest first
    pm, pe = pgrads, grads_of(emu)
    dn = sorted(((abs(float(pm[k].norm()) - float(gn_b[j])), k, float(gn_b[j])) for j, k in enumerate(names)
                 if pm.get(k) is not None), reverse=True)[:6]
    lids = sorted({int(k.split('.')[1]) for k in names})

    def lnorm(pg, lid):
        return float(torch.cat([pg[k].double().flatten().cpu() for k in names if int(k.split('.')[1]) == lid]).norm())
    prs = [grads_of(mm) for mm, _, _, _ in reals]
    pq = grads_of(ref)
    print('  per-layer gradient norm / fp32 (product, bf16 emulation CPU, GPU realizations): ' + ' '.join(
        f'{lid}:{lnorm(pm, lid) / lnorm(pq, lid):.3f},{lnorm(pe, lid) / lnorm(pq, lid):.3f},' +
        ','.join(f'{lnorm(q, lid) / lnorm(pq, lid):.3f}' for q in prs) for lid in lids))
    print('  largest grad-norm differences (fp32 norm: product, bf16 emulation): ' +
          ', '.join(f'{k} {b:.3e}: {float(pm[k].norm()):.3e}, {float(pe[k].norm()):.3e}' for d, k, b in dn))
    if chaotic:
        # see CHAOTIC: the whole-model single-step gradient of this config is a noise realization, so one product
        # realization against one emulation realization says nothing.  Compared as DISTRIBUTIONS instead (VERDICT r4
        # item 2b, r5 item 8): 3 product realizations (ulp-perturbed weights) against 5 realizations of the product's
        # storage model ('bf16_sink': the unperturbed one and 4 ulp-perturbed).  The product's MEDIAN whole-gradient
        # error must be within 1.25x the emulation's median and its median cosine within 0.05 of theirs.  The
        # per-parameter grad-norm vector is too heavy-tailed for a median bound at these sample sizes: over three runs
        # (round 6, profiles/r06/dma1536_distribution.log) the 15 emulation realizations spread 1.2e-2 .. 1.9e-1
        # (median 4.1e-2) and the product realizations 2.8e-2 .. 7.5e-2 (median 5.2e-2), and a run's 5-sample
        # emulation median moved from 3.2e-2 to 6.0e-2; it keeps a sanity bound: median within 1.5x the largest
        # emulation realization.  The emulation side is not run-to-run deterministic (torch's GPU weight-grad
        # reductions), and the product's median (5.1e-2 at HEAD) sits at about the 85th percentile of the pooled
        # emulation realizations (1.3e-2 .. 5.8e-2 over three runs, profiles/r06/dist_rerun.log), so 'within the 5
        # realizations' max' failed one run in three; a broken kernel sits far outside (a BN partial-row count that did
        # not follow the tile rule gave 2.1e-1 with outputs 3.4x the emulation's, profiles/r06/gpu_suite_bs2_bug.log)
        med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
        p_gn = [r[3][0] for r in perr]
        p_wg = [r[3][1] for r in perr]
        p_cos = [r[4] for r in perr]
        e_all = rerr + [(s_out, s_loss, s_item, s_gn, s_cos)]
        e_gnv = [r[3][0] for r in e_all]
        e_wg = [r[3][1] for r in e_all]
        e_cs = [r[4] for r in e_all]
        print(f'  distribution: product grad-norm vector {f(p_gn)} whole {f(p_wg)} cos {f(p_cos)}\n'
              f'                emulation    grad-norm vector {f(e_gnv)} whole {f(e_wg)} cos {f(e_cs)}')
        assert med(p_wg) <= 1.25 * med(e_wg), (p_wg, e_wg)
        assert med(p_cos) >= med(e_cs) - 0.05, (p_cos, e_cs)
        assert med(p_gn) <= 1.5 * max(e_gnv), (p_gn, e_gnv)
        for r in perr:  # every product realization's outputs / loss inside the per-realization bounds too
            for a, e in zip(r[0], env_out):
                assert a <= 1.1 * e + 2e-3, (r[0], env_out)
    else:
        assert gn_err[1] <= 1.1 * max(e_gn[1], r_gn[1]) + 1e-2, (gn_err[:2], e_gn[:2], r_gn[:2])
        assert med <= 1.1, ratios
        assert gn_err[0] <= 1.5 * max(e_gn[0], r_gn[0]) + 2e-3, (gn_err[:2], e_gn[:2], r_gn[:2])
        assert cos >= min(e_cos, r_cos) - 0.05, (cos, e_cos, r_cos)
    # the formats themselves: fp16 storage (10-bit mantissa) keeps the gradient direction much better than bf16 (7)
    assert h_cos > max(e_cos, r_cos) and max(h_out) < min(e_out), (h_cos, e_cos, h_out, e_out)


def test_bench_shape_fp32_product_vs_oracle():
    """The product in fp32 storage (act_dtype float32: the fp32 kernels) at DMA-YOLO-l's bench shape against the fp32
    CPU oracle on the same state_dict, images and targets: no storage rounding on either side, so what is left is fp32
    summation order.  Measured (round 4): loss equal to 7e-8, top-parameter gradients relative 6.3e-4..6.6e-4, cosine
    1.0000, every layer's gradient norm 1.000.  Bounds: loss 1e-5, outputs 1e-4, whole gradient 5e-3, per-layer norm
    ratios within 1e-3."""
    from dmayolo.models.yolo import Model
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    yml, img, bs, nc = 'yolov5l-ca-sppfcspc-bifpn-scconv.yaml', 1536, 2, 10
    torch.manual_seed(0)
    m = Model(os.path.join(CFG, yml), nc=nc, act_dtype=torch.float32)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    for mod in m.modules():
        if type(mod).__name__ == 'SwinTransformerLayer':
            mod.drop_path = torch.nn.Identity()
    hyp = scaled_hyp(HYP_VISDRONE, nc, img, 3)
    m.hyp = hyp
    m = m.cuda().train()
    x, t = images(bs, img, seed=1), targets(bs, nc, seed=1)
    anchors = m.model[-1].anchors.cpu()
    p = m(x.cuda())
    loss, _ = ComputeLoss(m)(p, t.cuda())
    loss.backward()
    ref, pr, lr_, _ = _oracle_grads(yml, nc, sd, x, t, anchors, hyp, None)
    pm, pq = dict(m.named_parameters()), dict(ref.named_parameters())
    names = [k for k in pq if pq[k].grad is not None]
    a = torch.cat([pm[k].grad.double().cpu().flatten() for k in names])
    b = torch.cat([pq[k].grad.double().flatten() for k in names])
    out = [_rel(o.detach().float().cpu(), r.detach()) for o, r in zip(p, pr)]
    lids = sorted({int(k.split('.')[1]) for k in names})

    def lnorm(pg, lid):
        return float(torch.cat([pg[k].grad.double().cpu().flatten() for k in names if int(k.split('.')[1]) == lid]).norm())
    lr = {lid: lnorm(pm, lid) / lnorm(pq, lid) for lid in lids}
    le = abs(float(loss) - float(lr_)) / abs(float(lr_))
    print(f'fp32 product @{img} bs{bs}: loss {le:.2e} outputs {out} whole gradient {_rel(a, b):.2e} cos '
          f'{float(a @ b / (a.norm() * b.norm())):.6f} per-layer norm ratios ' +
          ' '.join(f'{k}:{v:.4f}' for k, v in lr.items()))
    assert le < 1e-5 and max(out) < 1e-4, (le, out)
    assert _rel(a, b) < 5e-3, _rel(a, b)
    assert all(abs(v - 1) < 1e-3 for v in lr.values()), lr


def _layer_bounds(rows, k=1.25, floor=5e-4, outputs=True):
    """per layer: output, input- and parameter-gradient relative L2 <= k x the emulation's + floor; norm ratios within
    1e-3 of 1 or of 1.5 x the emulation's own deviation + 2e-3.  Returns the violations."""
    bad = []
    for i, name, row in rows:
        if isinstance(row, Exception):
            if i != 0:  # the stem's product module takes the space-to-depth image input, not the oracle's
                bad.append((i, name, repr(row)))
            continue
        for kd in (('y', 'dx', 'w') if outputs else ('dx', 'w')):
            v = row.get(kd)
            if v is not None and v[0] > k * v[1] + floor:
                bad.append((i, name, kd, v))
        for kd in ('dxn', 'wn'):
            if kd in row and abs(row[kd][0] - 1) > max(1e-3, 1.5 * abs(row[kd][1] - 1) + 2e-3):
                bad.append((i, name, kd, row[kd]))
    return bad


def _collect(gen):
    from module_parity import fmt
    rows = []
    for i, name, row in gen:
        print(fmt(i, name, row), flush=True)
        rows.append((i, name, row))
    return rows


@pytest.mark.parametrize('yml,img,bs', [('yolov5l-ca-sppfcspc-bifpn-scconv.yaml', 1536, 2),
                                        ('yolov5l-xs-tr-cbam-spp-bifpn.yaml', 1920, 2)])
def test_bench_shape_layers_bf16_vs_emulation(yml, img, bs, monkeypatch):
    """Every top-level layer of a bench model alone at its bench resolution on the inputs the fp32 oracle sees there
    (tests/module_parity.py): the bf16 product module and the bf16-storage emulation of the oracle module against the
    fp32 oracle module, for one seeded upstream gradient.  DMA-YOLO-l @1536 (config 3) and config 5 @1920 -- there
    C3TR's global attention runs over 60 x 60 = 3,600 tokens per image, as in the bench.  The emulation is 'bf16_sink'
    with the layer's input gradient rounded as the product stores it (module_parity).  Bounds per layer: output, input
    and parameter gradient relative L2 <= 1.25 x the emulation's + 5e-4, norm ratios within 1e-3 of 1 or of 1.5 x the
    emulation's own deviation + 2e-3.
    Round 5's C3TR rows (0.423 for product, bf16 AND fp16 emulation alike) compared three different dropout masks:
    TransformerLayer's nn.Dropout(0.1) (common.py:328) was on in all three runs.  With dropout off (module_parity) the
    row is a real check; config 5 then re-runs its C3TR layers with the product's attention output scaled by 1.1 (a
    10 % kernel error) and requires the bound to FAIL there."""
    from module_parity import layer_parity
    rows = _collect(layer_parity(yml, img, bs))
    assert len(rows) >= 15
    bad = _layer_bounds(rows)
    assert not bad, bad
    c3tr = [i for i, name, row in rows if name == 'C3TR']
    if 'xs-tr' in yml:
        assert c3tr
        import dmayolo.functional as Fn
        real = Fn.MHAFn

        class Off10:  # the attention core, 10 % off (forward and, through autograd, backward)
            @staticmethod
            def apply(q, k, v, nh):
                return real.apply(q, k, v, nh) * 1.1

        monkeypatch.setattr(Fn, 'MHAFn', Off10)
        sab = _collect(layer_parity(yml, img, bs, only=c3tr))
        monkeypatch.setattr(Fn, 'MHAFn', real)
        for i, name, row in sab:
            assert _layer_bounds([(i, name, row)]), (i, 'a 10 % attention error passed the per-layer bound')


def test_c5_layers_fp32_product_vs_oracle():
    """Config 5 @1920 bs2 per layer in fp32 storage (act_dtype float32: the fp32 kernels, fp32 generic attention over
    3,600 tokens) against the fp32 oracle module on the same inputs and upstream gradient -- the config-5 counterpart of
    test_bench_shape_fp32_product_vs_oracle, per layer so that CBAM / SPP argmax near-ties do not chain.  No storage
    rounding on either side: outputs <= 1e-4, input and parameter gradients <= 1e-3 relative L2, norms within 1e-3.
    SPP's input gradient gets 2e-3: its cv1 output is summed in another fp32 order by the product and the oracle, and
    the k = 5 / 9 / 13 max-pools route each window's gradient to whichever input wins on those last bits (round 6
    measured 3.4e-4 .. 9.6e-4 on the four SPP layers, every other layer <= 4.3e-4, profiles/r06/c5_layers_1920.log)."""
    from module_parity import layer_parity
    rows = _collect(layer_parity('yolov5l-xs-tr-cbam-spp-bifpn.yaml', 1920, 2, prod='fp32'))
    assert len(rows) >= 15 and any(name == 'C3TR' for _, name, _ in rows)
    bad = []
    for i, name, row in rows:
        if isinstance(row, Exception):
            if i != 0:
                bad.append((i, name, repr(row)))
            continue
        if row['y'][0] > 1e-4:
            bad.append((i, name, 'y', row['y'][0]))
        for kd in ('dx', 'w'):
            lim = 2e-3 if (kd == 'dx' and name in ('SPP', 'SPPF')) else 1e-3
            if kd in row and row[kd][0] > lim:
                bad.append((i, name, kd, row[kd][0]))
        for kd in ('dxn', 'wn'):
            if kd in row and abs(row[kd][0] - 1) > 1e-3:
                bad.append((i, name, kd, row[kd][0]))
    assert not bad, bad


def test_c5_layers_fp8_vs_emulation():
    """Config 5's fp8 leg (functional.set_fp8: e4m3 forward of every 3x3 conv with C % 128 == 0, bf16 backward) per
    layer at its bench resolution 1920 bs2 against the 'fp8_sink' emulation (precision_emu: the same e4m3 quantisation
    of input and weights, per tensor / per output channel, on top of 'bf16_sink'), both against the fp32 oracle.  The
    layers' first call quantises just in time with the current amax, as the emulation does.  Bounds as the bf16 layer
    test: 1.25 x the emulation's error + 5e-4 on outputs and gradients."""
    from module_parity import layer_parity
    rows = _collect(layer_parity('yolov5l-xs-tr-cbam-spp-bifpn.yaml', 1920, 2, prod='fp8'))
    assert len(rows) >= 15
    bad = _layer_bounds(rows)
    assert not bad, bad
