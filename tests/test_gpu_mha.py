"""GPU: the C3TR attention core (csrc/mha.hip) and the TransformerLayer dropout.

* generic (fp32-math) kernel vs a plain PyTorch fp32 reference of softmax(q k^T / sqrt(d)) v and its
  autograd gradients (fp32 storage, tolerance 1e-4);
* bf16 MFMA kernels vs the generic kernel on the same bf16-representable inputs (head dim 32/64/128,
  ragged token counts): relative L2 error < 2e-2 forward, < 4e-2 backward;
* C3TR at head dim 128 (the config-5 width) in bf16 vs the CPU oracle;
* dropout: keep rate, exact 1/(1-p) scaling, identical mask in the backward."""
import pytest
import torch

from gpu_util import rel_err

pytestmark = pytest.mark.gpu


def _call(name, *a):
    from dmayolo.functional import call
    return call(name, *a)


def _attn_ref(q, k, v, nh):
    """plain PyTorch fp32: q, k, v [B, L, C] -> [B, L, C]"""
    B, L, C = q.shape
    d = C // nh
    sp = lambda t: t.view(B, L, nh, d).transpose(1, 2)
    a = torch.softmax((sp(q) * d ** -0.5) @ sp(k).transpose(-1, -2), -1)
    return (a @ sp(v)).transpose(1, 2).reshape(B, L, C)


def _run(dtype, q, k, v, do, nh, ref=False):
    from dmayolo.functional import ptr, stream
    B, L, C = q.shape
    d = C // nh
    dt = 1 if dtype == torch.bfloat16 else 0
    q, k, v, do = (t.to(dtype).contiguous().cuda() for t in (q, k, v, do))
    o = torch.empty_like(q)
    lse = torch.empty(B * nh * L, device='cuda')
    _call('dmy_mha_fwd_ref' if ref else 'dmy_mha_fwd', dt, ptr(q), C, ptr(k), C, ptr(v), C, ptr(o), C, ptr(lse), B, L,
          nh, d, d ** -0.5, stream())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    Dq = torch.empty(B * nh * L, device='cuda')
    _call('dmy_mha_bwd', dt, ptr(q), C, ptr(k), C, ptr(v), C, ptr(o), ptr(do), C, ptr(lse), ptr(Dq), ptr(dq), ptr(dk),
          ptr(dv), B, L, nh, d, d ** -0.5, stream())
    torch.cuda.synchronize()
    return [t.float().cpu() for t in (o, dq, dk, dv)] + [lse.cpu()]


def _inputs(B, L, C, seed):
    g = torch.Generator().manual_seed(seed)
    q, k, v, do = (torch.randn(B, L, C, generator=g) for _ in range(4))
    return q * 1.5, k * 1.5, v, do


@pytest.mark.parametrize('B,L,C,nh', [(2, 35, 16, 4), (1, 64, 64, 2), (2, 90, 128, 4), (1, 200, 256, 2),
                                      (1, 3600, 512, 4)])
def test_mha_generic_fp32_vs_torch(B, L, C, nh):
    """the fp32 generic kernels against plain PyTorch in float64 (the reference's math, no reordering error of its
    own), up to config 5's C3TR at 1920: 3,600 tokens, 512 channels, 4 heads of 128"""
    q, k, v, do = _inputs(B, L, C, 3)
    o, dq, dk, dv, _ = _run(torch.float32, q, k, v, do, nh)
    qq, kk, vv = (t.double().requires_grad_(True) for t in (q, k, v))
    ro = _attn_ref(qq, kk, vv, nh)
    ro.backward(do.double())
    torch.testing.assert_close(o.double(), ro.detach(), rtol=1e-4, atol=1e-5)
    assert rel_err(o.double(), ro.detach()) < 1e-5
    for a, b in ((dq, qq.grad), (dk, kk.grad), (dv, vv.grad)):
        torch.testing.assert_close(a.double(), b, rtol=1e-4, atol=1e-4)
        assert rel_err(a.double(), b) < 5e-5, rel_err(a.double(), b)


@pytest.mark.parametrize('B,L,C,nh', [(2, 90, 128, 4), (1, 400, 256, 4), (2, 130, 512, 4), (1, 64, 256, 2),
                                      (3, 17, 128, 2), (1, 3600, 512, 4)])
def test_mha_mfma_vs_generic(B, L, C, nh):
    q, k, v, do = _inputs(B, L, C, 4)
    q, k, v, do = (t.bfloat16().float() for t in (q, k, v, do))  # bf16-representable
    got = _run(torch.bfloat16, q, k, v, do, nh)
    ref = _run(torch.float32, q, k, v, do, nh)  # fp32 storage -> generic kernels
    names = ('o', 'dq', 'dk', 'dv')
    for n, a, b in zip(names, got[:4], ref[:4]):
        tol = 2e-2 if n == 'o' else 4e-2
        assert rel_err(a, b) < tol, (n, rel_err(a, b))
    torch.testing.assert_close(got[4], ref[4], rtol=1e-3, atol=2e-3)


def test_mha_mfma_matches_generic_bf16_forward():
    """MFMA forward vs the generic kernel on bf16 storage (identical inputs and output rounding)."""
    q, k, v, do = (t.bfloat16().float() for t in _inputs(2, 150, 256, 6))
    a = _run(torch.bfloat16, q, k, v, do, 4)
    b = _run(torch.bfloat16, q, k, v, do, 4, ref=True)
    assert rel_err(a[0], b[0]) < 1e-2, rel_err(a[0], b[0])


def test_dropout_kernel():
    from dmayolo.functional import DropoutFn
    torch.manual_seed(0)
    x = torch.randn(4, 64, 20, 30, device='cuda').contiguous(memory_format=torch.channels_last).requires_grad_(True)
    p = 0.1
    y = DropoutFn.apply(x, p)
    keep = y != 0
    frac = float(keep.float().mean())
    assert abs(frac - (1 - p)) < 5e-3, frac
    torch.testing.assert_close(y[keep], (x / (1 - p))[keep], rtol=0, atol=0)
    g = torch.randn_like(x)
    y.backward(g)
    torch.testing.assert_close(x.grad, torch.where(keep, g / (1 - p), torch.zeros_like(g)), rtol=0, atol=0)
    y2 = DropoutFn.apply(x.detach(), p)
    assert not torch.equal(y2 != 0, keep)  # a fresh seed per call


@pytest.mark.parametrize('c,hw', [(1024, (12, 10)), (512, (9, 7))])
def test_c3tr_bf16_vs_oracle(c, hw):
    """C3TR(c, c, 1) (head dim c/8: 128 at the config-5 width) in bf16 on the GPU vs the CPU oracle."""
    from dmayolo.models import common as P
    from oracle import nn as onn
    torch.manual_seed(31)
    pm = onn.bn_defaults(P.C3TR(c, c, 1, False))
    om = onn.bn_defaults(onn.C3TR(c, c, 1, False))
    om.load_state_dict(pm.state_dict())
    for m in list(pm.modules()) + list(om.modules()):
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    x = torch.randn(2, c, *hw, generator=torch.Generator().manual_seed(32)) * 0.5
    gup = torch.randn(2, c, *hw, generator=torch.Generator().manual_seed(33))
    pm = pm.cuda().train()
    xg = x.cuda().bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    yg = pm(xg)
    (yg.float() * gup.cuda()).sum().backward()
    xc = x.clone().requires_grad_(True)
    yc = om.train()(xc)
    (yc * gup).sum().backward()
    assert rel_err(yg.float().cpu(), yc.detach()) < 3e-2
    assert rel_err(xg.grad.float().cpu(), xc.grad) < 8e-2, rel_err(xg.grad.float().cpu(), xc.grad)
    gp = dict(pm.named_parameters())
    gmax = max(float(p.grad.norm()) for p in om.parameters() if p.grad is not None)
    for k, p in om.named_parameters():
        if p.grad is None:
            continue
        err = float((gp[k].grad.float().cpu() - p.grad).norm()) / max(float(p.grad.norm()), 1e-2 * gmax)
        assert err < 8e-2, (k, err)


def test_dropout_mask_redrawn_on_graph_replay():
    """DropoutFn's seed is drawn on the device (dmy_dropout_seed), so a HIP graph that captured forward +
    backward draws a fresh mask on every replay, and the backward of each replay uses that replay's mask."""
    import dmayolo.functional as Fn
    x = torch.randn(2, 64, 8, 8, device='cuda').contiguous(memory_format=torch.channels_last).requires_grad_(True)
    gup = torch.ones_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up off the default stream (creates the generator state outside the capture)
        Fn.DropoutFn.apply(x, 0.5).backward(gup)
    torch.cuda.current_stream().wait_stream(s)
    x.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):  # the same capture pattern as train_graph.GraphedTrainStep
        sy = Fn.DropoutFn.apply(x, 0.5)
        sy.backward(gup)
    masks = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        keep = sy.detach() != 0
        assert torch.equal(keep, x.grad != 0)  # backward regenerated this replay's mask
        torch.testing.assert_close(sy.detach()[keep], (x.detach() * 2)[keep])
        masks.append(keep.clone())
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])
    frac = float(torch.stack(masks).float().mean())
    assert 0.45 < frac < 0.55, frac
