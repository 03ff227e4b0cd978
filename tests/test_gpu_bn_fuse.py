"""GPU: SCConv's k3 BatchNorm folded into its gate (functional.SCGateFn, dmy_scgate_bn_fwd / _bwd): the gate applies
k3's BN to z and its backward writes k3's backward-reduce partials, handed over through the BnLink, against the unfused
path (bn_act_fwd + dmy_scgate_fwd, bn_bwd_reduce).

(Round 2's data-grad-epilogue form of the producer-BN reduce, dmy_conv_dgrad_bn, was measured slower end to end and
removed in round 6 with its tests.)
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize('N,C,H,W', [(2, 64, 96, 128), (3, 128, 40, 56), (1, 256, 24, 24)])
def test_scconv_gate_applies_k3_bn(N, C, H, W):
    """SCConv with k3's BatchNorm folded into the gate (conv_bn_act(defer=True) + dmy_scgate_bn_fwd / _bwd, whose
    backward hands k3 its BN reduce partials through the BnLink) against the unfused path (DMY_DEFER_AFFINE off:
    bn_act_fwd + dmy_scgate_fwd, bn_bwd_reduce): the forward output, every parameter gradient, the input gradient and
    the running statistics agree (same value contract: u3 = bf16(z * scale + shift), the reduce over du3 as stored)"""
    import dmayolo.functional as Fn
    from dmayolo.models.common import SCConv
    torch.manual_seed(0)
    m = SCConv(C, 2 * C, 2).cuda()
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.2, 0.2)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x0 = torch.randn(N, C, H, W, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
    gup = torch.randn(N, 2 * C, H // 2, W // 2, device='cuda')
    res = []
    for on in (False, True):
        m.load_state_dict(sd)
        m.zero_grad(set_to_none=True)
        Fn.DEFER_AFFINE[0] = on
        try:
            x = x0.clone().requires_grad_(True)
            y = m(x)
            (y.float() * gup).sum().backward()
        finally:
            Fn.DEFER_AFFINE[0] = True
        torch.cuda.synchronize()
        res.append((y.float(), x.grad.float(), {k: p.grad.clone() for k, p in m.named_parameters()},
                    {k: v.clone() for k, v in m.state_dict().items() if 'running' in k}))
    (y0, gx0, gp0, rs0), (y1, gx1, gp1, rs1) = res
    rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))  # noqa: E731
    assert torch.equal(y0, y1), rel(y1, y0)
    assert rel(gx1, gx0) < 1e-6, rel(gx1, gx0)
    for k in gp0:
        assert rel(gp1[k], gp0[k]) < 1e-5 or float((gp1[k] - gp0[k]).abs().max()) < 1e-6, (k, rel(gp1[k], gp0[k]))
    for k in rs0:
        assert torch.equal(rs0[k], rs1[k]), k
