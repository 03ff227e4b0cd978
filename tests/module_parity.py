"""Layer-by-layer parity at a bench shape (test infrastructure, used by test_gpu_bench_shape.py and
tools/gpu/diag_modules.py): every top-level layer of a bench model alone, at the bench shape, on the inputs the fp32 oracle sees
there -- the bf16 product module and the bf16-storage emulation of the oracle module (tests/precision_emu.py 'bf16')
against the fp32 oracle module, for one seeded upstream gradient with per-channel means.  Per layer: relative L2 and
norm ratio of the input gradient and of the layer's concatenated parameter gradient, product | emulation.  A layer
whose product error or norm ratio sits well outside the emulation's is where the whole-model gradient picks up more
than storage noise.

The emulation is 'bf16_sink' with the layer's INPUT gradient rounded to bf16 once more as it leaves the layer: the
product stores dx in bf16 (its storage), and each of several consumers' contributions is rounded before it is summed
(functional.GradSink).  Round 4 compared against plain 'bf16' with an fp32 dx, i.e. one bf16 rounding short: every
plain Conv's dx measured 1.13x the emulation's -- sqrt(3.1^2 + 1.66^2) = 3.5e-3, exactly one extra round-to-nearest
(1.66e-3 relative, test_gpu_conv_bench_shapes.py) -- and the multi-consumer layers (CoorAttention, SCConv) more.
`fp16=True` also runs the reference's own autocast precision ('fp16', train.py:434) per layer, reported as dx16 / w16.

layer_parity() returns one row per layer; tools/gpu/diag_modules.py prints them.
"""
import copy
import os

import torch
import yaml
from dmayolo.models.yolo import Model
from dmayolo.synthetic import images, CONFIGS
from oracle import nn as onn
from precision_emu import emulate, RoundGrad

CL = torch.channels_last


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def nr(a, b):
    return float(a.double().norm() / b.double().norm().clamp_min(1e-30))


def run_layer(res, xs, xin, g, mods):
    """mods: (kind, module, storage dtype of its input gradient or None)"""
    for kind, mod, dt in mods:
        mod.zero_grad(set_to_none=True)
        if kind == 'prod':
            xi = [x.bfloat16().contiguous(memory_format=CL).requires_grad_(True) for x in xs]
            xf = xi
        else:
            xi = [x.clone().requires_grad_(True) for x in xs]
            xf = [RoundGrad.apply(x, dt) for x in xi] if dt is not None else xi
        y = mod(xf if isinstance(xin, (list, tuple)) else xf[0])
        if 'gup' not in res:
            C = y.shape[1]
            res['gup'] = torch.randn(y.shape, generator=g, device='cuda') + \
                torch.linspace(-0.5, 0.5, C, device='cuda').view(1, -1, 1, 1)
        # the product's output is bf16, so autograd hands it the upstream gradient rounded to bf16: the emulation gets
        # the same rounded gradient (fp16 emulation: rounded to fp16), the fp32 oracle the exact one
        gup = res['gup'].to(dt).float() if dt is not None else res['gup']
        (y.float() * gup).sum().backward()
        res[kind] = (torch.cat([x.grad.float().flatten() for x in xi]),
                     {k: p.grad.detach().float().flatten() for k, p in mod.named_parameters() if p.grad is not None})


def layer_parity(yml, img, bs, only=None, fp16=False, mode='bf16_sink'):
    """yields (layer id, type name, row) with row = dict(dx=(prod rel, emu rel), dxn=(prod norm ratio, emu norm
    ratio), w=(...), wn=(...), worst=(param, prod rel, emu rel)) -- w / wn / worst absent for parameter-free layers --
    or (layer id, type name, exception) when the layer could not run"""
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    with open(os.path.join(CONFIGS, yml)) as f:
        cfg = yaml.safe_load(f)
    nc = 10
    torch.manual_seed(0)
    m = Model(cfg, nc=nc, act_dtype=torch.bfloat16)
    ref = onn.bn_defaults(onn.Model(cfg, nc=nc))
    ref.load_state_dict(m.state_dict())
    for mod in list(m.modules()) + list(ref.modules()):
        if hasattr(mod, 'drop_prob'):
            mod.drop_prob = 0.0
        if type(mod).__name__ == 'SwinTransformerLayer' and hasattr(mod, 'drop_path'):
            mod.drop_path = torch.nn.Identity()
    m, ref = m.cuda().train(), ref.cuda().train()
    inputs = {}
    hooks = [mod.register_forward_pre_hook(lambda mod, a, i=i: inputs.__setitem__(i, a[0]))
             for i, mod in enumerate(ref.model)]
    with torch.no_grad():
        ref(images(bs, img, seed=1).cuda().float() / 255)
    for h in hooks:
        h.remove()
    for i, (pm, om) in enumerate(zip(m.model, ref.model)):
        name = type(pm).__name__
        if name in ('Detect', 'Upsample') or (only is not None and i not in only):
            continue
        xin = inputs[i]
        xs = list(xin) if isinstance(xin, (list, tuple)) else [xin]
        xs = [x.detach().bfloat16().float() for x in xs]  # the product's bf16 inputs, shared by all three
        g = torch.Generator(device='cuda').manual_seed(100 + i)
        res = {}
        em = emulate(copy.deepcopy(om), mode)
        mods = [('prod', pm, None), ('fp32', om, None), ('emu', em, torch.bfloat16)]
        if fp16:
            mods.append(('f16', emulate(copy.deepcopy(om), 'fp16'), torch.float16))
        try:
            run_layer(res, xs, xin, g, mods)
        except Exception as e:  # noqa: BLE001 (reported per layer)
            yield i, name, e
            continue
        dxp, dxf, dxe = res['prod'][0], res['fp32'][0], res['emu'][0]
        ks = [k for k in res['fp32'][1] if k in res['prod'][1] and k in res['emu'][1]]
        row = dict(dx=(rel(dxp, dxf), rel(dxe, dxf)), dxn=(nr(dxp, dxf), nr(dxe, dxf)))
        if 'f16' in res:
            row['dx16'] = rel(res['f16'][0], dxf)
            k16 = [k for k in ks if k in res['f16'][1]]
            if k16:
                row['w16'] = rel(torch.cat([res['f16'][1][k] for k in k16]), torch.cat([res['fp32'][1][k] for k in k16]))
        if ks:
            cat = lambda d: torch.cat([d[k] for k in ks])  # noqa: E731
            pp, pf, pe = cat(res['prod'][1]), cat(res['fp32'][1]), cat(res['emu'][1])
            worst = max(ks, key=lambda k: rel(res['prod'][1][k], res['fp32'][1][k]) /
                        max(rel(res['emu'][1][k], res['fp32'][1][k]), 1e-12))
            row.update(w=(rel(pp, pf), rel(pe, pf)), wn=(nr(pp, pf), nr(pe, pf)),
                       worst=(worst, rel(res['prod'][1][worst], res['fp32'][1][worst]),
                              rel(res['emu'][1][worst], res['fp32'][1][worst])))
        del res, em
        torch.cuda.empty_cache()
        yield i, name, row


def fmt(i, name, row):
    if isinstance(row, Exception):
        return f'{i:2d} {name:10s} | failed: {type(row).__name__}: {str(row)[:200]}'
    s = (f'{i:2d} {name:10s} | dx {row["dx"][0]:.2e} {row["dx"][1]:.2e} ({row["dx"][0] / max(row["dx"][1], 1e-30):.2f}x) '
         f'| {row["dxn"][0]:.4f} {row["dxn"][1]:.4f}')
    if 'dx16' in row:
        s += f' | fp16 emu dx {row["dx16"]:.2e}' + (f' W {row["w16"]:.2e}' if 'w16' in row else '')
    if 'w' in row:
        w = row['worst']
        s += (f' | W {row["w"][0]:.2e} {row["w"][1]:.2e} ({row["w"][0] / max(row["w"][1], 1e-30):.2f}x) | {row["wn"][0]:.4f} '
              f'{row["wn"][1]:.4f} | {w[0]} {w[1]:.2e} / '
              f'{w[2]:.2e}')
    return s
