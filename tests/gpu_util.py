"""Shared helpers for the GPU parity tests (product modules vs reference golden vectors / oracle)."""
import torch

from golden_util import Fixture, load_sd
from oracle import nn as onn


def product_modules():
    from dmayolo.models import common as P
    import torch.nn as nn
    return {
        'Conv': P.Conv, 'Bottleneck': P.Bottleneck, 'C3': P.C3, 'SCConv': P.SCConv,
        'CoorAttention': P.CoorAttention, 'C3CA': P.C3CA, 'SPPF': P.SPPF, 'SPPFCSPC': P.SPPFCSPC,
        'Upsample': P.Upsample, 'AdConcat2': P.AdConcat2, 'AdConcat3': P.AdConcat3, 'Concat': P.Concat,
        'SwinTransformerLayer': lambda c, h, ws, sh: P.SwinTransformerLayer(c, h, ws, sh), 'C3STR': P.C3STR,
        'SPP': lambda c1, c2, k: P.SPP(c1, c2, tuple(k)), 'CBAM': P.CBAM, 'C3TR': P.C3TR,
    }


def run_case(name, mods, device, dtype=torch.float32, inputs=None, sd=None):
    """Train fwd+bwd and eval fwd of a module on the golden fixture `name` (optionally new inputs)."""
    fx = Fixture(name)
    meta = fx.meta
    mod = mods[meta['module']](*meta['args'])
    onn.bn_defaults(mod)
    for m in mod.modules():
        if hasattr(m, 'drop_prob'):
            m.drop_prob = 0.0
        if type(m).__name__ == 'SwinTransformerLayer':
            m.drop_path = torch.nn.Identity()
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0  # fixtures were captured with the TransformerLayer dropout off
    load_sd(mod, sd if sd is not None else fx.group('sd'))
    mod = mod.to(device)
    xs = inputs if inputs is not None else fx.seq('in')
    ins = [x.to(device=device, dtype=dtype).requires_grad_(True) for x in xs]
    listin = meta['module'] in ('AdConcat2', 'AdConcat3', 'Concat')
    mod.train()
    out = mod(ins if listin else ins[0])
    outs = list(out) if isinstance(out, (list, tuple)) else [out]
    gen = torch.Generator().manual_seed(1000)
    if inputs is None:
        gups = [g.to(device, dtype) for g in fx.seq('gup')]
    else:
        gups = [torch.randn(o.shape, generator=gen).to(device, dtype) for o in outs]
    loss = sum((o.float() * g.float()).sum() for o, g in zip(outs, gups))
    loss.backward()
    res = dict(out=[o.detach().float().cpu() for o in outs], gin=[x.grad.float().cpu() for x in ins],
               gp={k: p.grad.float().cpu() for k, p in mod.named_parameters() if p.grad is not None},
               buf={k: v.float().cpu().clone() for k, v in mod.state_dict().items() if 'running' in k},
               gups=[g.float().cpu() for g in gups])
    load_sd(mod, sd if sd is not None else fx.group('sd'))
    mod.eval()
    with torch.no_grad():
        eo = mod([x.detach() for x in ins] if listin else ins[0].detach())
    res['eout'] = [o.float().cpu() for o in (eo if isinstance(eo, (list, tuple)) else [eo])]
    return fx, res


def rel_err(a, b):
    """relative L2 error (robust to the few max-pool argmax swaps bf16 rounding causes)"""
    # absolute floor: grads that are pure rounding noise in the reference (a bias feeding a
    # train-mode BN has an exactly-zero gradient) must not count as 100 % error
    return float((a.double() - b.double()).norm() / max(b.double().norm(), 1e-4 * b.numel() ** 0.5))
