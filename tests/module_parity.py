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
    """mods: (kind, module, storage dtype of its input gradient or None, product input dtype or None)"""
    for kind, mod, dt, pdt in mods:
        mod.zero_grad(set_to_none=True)
        if kind == 'prod':
            xi = [x.to(pdt).contiguous(memory_format=CL).requires_grad_(True) for x in xs]
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
        # the same rounded gradient (fp16 emulation: rounded to fp16), the fp32 oracle (and an fp32 product) the exact
        gup = res['gup'].to(dt).float() if dt is not None else res['gup']
        (y.float() * gup).sum().backward()
        res[kind] = (torch.cat([x.grad.float().flatten() for x in xi]),
                     {k: p.grad.detach().float().flatten() for k, p in mod.named_parameters() if p.grad is not None},
                     y.detach().float().flatten())


PROD = {  # product storage -> (act_dtype, emulation mode of the oracle, rounding of the product's upstream gradient)
    'bf16': (torch.bfloat16, 'bf16_sink', torch.bfloat16),
    'fp8': (torch.bfloat16, 'fp8_sink', torch.bfloat16),  # functional.set_fp8: e4m3 forward of the eligible convs
    'fp32': (torch.float32, None, None),  # the fp32 kernels against the fp32 oracle: no emulation
}


def layer_parity(yml, img, bs, only=None, fp16=False, prod='bf16'):
    """yields (layer id, type name, row) with row = dict(y=(prod rel, emu rel) of the layer output, dx=(prod rel, emu
    rel), dxn=(prod norm ratio, emu norm ratio), w=(...), wn=(...), worst=(param, prod rel, emu rel)) -- w / wn / worst
    absent for parameter-free layers, the emu entries None when prod='fp32' -- or (layer id, type name, exception) when
    the layer could not run.  Dropout is off in all three (nn.Dropout(0.1) of config 5's TransformerLayer,
    common.py:328: in train mode each run would draw its own mask; round 5's C3TR rows compared three different masks)"""
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    act_dtype, mode, gdt = PROD[prod]
    with open(os.path.join(CONFIGS, yml)) as f:
        cfg = yaml.safe_load(f)
    nc = 10
    torch.manual_seed(0)
    m = Model(cfg, nc=nc, act_dtype=act_dtype)
    ref = onn.bn_defaults(onn.Model(cfg, nc=nc))
    ref.load_state_dict(m.state_dict())
    for mod in list(m.modules()) + list(ref.modules()):
        if hasattr(mod, 'drop_prob'):
            mod.drop_prob = 0.0
        if type(mod).__name__ == 'SwinTransformerLayer' and hasattr(mod, 'drop_path'):
            mod.drop_path = torch.nn.Identity()
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    if prod == 'fp8':
        from dmayolo.functional import set_fp8
        assert set_fp8(m, True) > 0
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
        mods = [('prod', pm, gdt, act_dtype), ('fp32', om, None, None)]
        if mode is not None:
            mods.append(('emu', emulate(copy.deepcopy(om), mode), torch.bfloat16, None))
        if fp16:
            mods.append(('f16', emulate(copy.deepcopy(om), 'fp16'), torch.float16, None))
        try:
            run_layer(res, xs, xin, g, mods)
        except Exception as e:  # noqa: BLE001 (reported per layer)
            yield i, name, e
            continue
        emu = res.get('emu')
        opt = lambda f, k: f(emu[k], res['fp32'][k]) if emu is not None else None  # noqa: E731
        dxp, dxf = res['prod'][0], res['fp32'][0]
        ks = [k for k in res['fp32'][1] if k in res['prod'][1] and (emu is None or k in emu[1])]
        row = dict(y=(rel(res['prod'][2], res['fp32'][2]), opt(rel, 2)),
                   dx=(rel(dxp, dxf), opt(rel, 0)), dxn=(nr(dxp, dxf), opt(nr, 0)))
        if 'f16' in res:
            row['dx16'] = rel(res['f16'][0], dxf)
            k16 = [k for k in ks if k in res['f16'][1]]
            if k16:
                row['w16'] = rel(torch.cat([res['f16'][1][k] for k in k16]), torch.cat([res['fp32'][1][k] for k in k16]))
        if ks:
            cat = lambda d: torch.cat([d[k] for k in ks])  # noqa: E731
            pp, pf = cat(res['prod'][1]), cat(res['fp32'][1])
            pe = cat(emu[1]) if emu is not None else None
            erel = lambda k: rel(emu[1][k], res['fp32'][1][k]) if emu is not None else 1.0  # noqa: E731
            worst = max(ks, key=lambda k: rel(res['prod'][1][k], res['fp32'][1][k]) / max(erel(k), 1e-12))
            row.update(w=(rel(pp, pf), rel(pe, pf) if pe is not None else None),
                       wn=(nr(pp, pf), nr(pe, pf) if pe is not None else None),
                       worst=(worst, rel(res['prod'][1][worst], res['fp32'][1][worst]),
                              erel(worst) if emu is not None else None))
        del res
        torch.cuda.empty_cache()
        yield i, name, row


def fmt(i, name, row):
    if isinstance(row, Exception):
        return f'{i:2d} {name:10s} | failed: {type(row).__name__}: {str(row)[:200]}'
    e = lambda v: '-' if v is None else f'{v:.2e}'  # noqa: E731
    r = lambda a, b: '' if b is None else f' ({a / max(b, 1e-30):.2f}x)'  # noqa: E731
    n = lambda v: '-' if v is None else f'{v:.4f}'  # noqa: E731
    s = (f'{i:2d} {name:10s} | y {e(row["y"][0])} {e(row["y"][1])}{r(*row["y"])} '
         f'| dx {e(row["dx"][0])} {e(row["dx"][1])}{r(*row["dx"])} | {n(row["dxn"][0])} {n(row["dxn"][1])}')
    if 'dx16' in row:
        s += f' | fp16 emu dx {row["dx16"]:.2e}' + (f' W {row["w16"]:.2e}' if 'w16' in row else '')
    if 'w' in row:
        w = row['worst']
        s += (f' | W {e(row["w"][0])} {e(row["w"][1])}{r(*row["w"])} | {n(row["wn"][0])} {n(row["wn"][1])} | '
              f'{w[0]} {e(w[1])} / {e(w[2])}')
    return s
