"""Reduced-precision storage emulation of the CPU oracle (test infrastructure, used by test_gpu_bench_shape.py and
tools/gpu/diag_precision.py).

The oracle (oracle/nn.py) computes in fp32.  To say how far the bf16 HIP product may sit from it, the same oracle is
run again with the roundings a reduced-precision run performs, and the product is held to that run's error:

  mode 'bf16_act' (round 2's emulation): every leaf module output (Conv2d, Linear, SiLU, pools, LayerNorm, GELU, ...)
                   and the gradient flowing back into it rounded to bf16;
  mode 'bf16'     the product's storage model: 'bf16_act' + the conv / linear weights rounded to bf16 in the forward
                   and data-gradient (the kernels read bf16 OHWI / IHWO copies of the fp32 master weights; the weight
                   gradient itself stays fp32) + the outputs of the composite modules whose result the product stores
                   in bf16 (Bottleneck / Swin residual sums, CoorAttention's pooled means and x * a_w * a_h, the
                   AdConcat weighted copies, SCConv's gate product, CBAM's ca, ca * x, pooled map, spatial gate and output);
  mode 'bf16_sink' 'bf16' + each leaf's INPUT gradient rounded to bf16 as it leaves the leaf: the product's data-grad
                   kernels store every contribution to an input gradient in bf16 and accumulate the next one into that
                   bf16 buffer (functional.GradSink; autograd's own sums of bf16 gradients), where 'bf16' sums the
                   fp32 contributions first and rounds once at the producer's output.  A tensor with one consumer
                   rounds the same value twice (no change); one with k consumers gets the k roundings the product has;
  mode 'fp16'     the reference's own training precision, CUDA autocast (train.py:434): the same roundings to fp16
                   (conv / linear / activation outputs and weights fp16, BatchNorm statistics and the loss fp32),
                   backward seeded with a 2^16 loss scale as GradScaler does, so that fp16 gradients do not underflow;
  (round 6: also C3TR's stored tensors -- in-projected q / k / v, the attention probabilities, the attention output and
  the residual sums, which the oracle's functional projections had hidden from the leaf hooks -- and CoorAttention's
  pooled means)
  mode 'fp8_sink' 'fp8' with 'bf16_sink's input-gradient roundings (the per-layer comparison of the fp8 product);
  mode 'fp8'      config 5's storage: 'bf16', and every conv the product runs on the e4m3 kernel (functional.set_fp8:
                   k >= 3, C % 128 == 0, K % 8 == 0, K >= 32) computes its FORWARD from e4m3 operands -- the input
                   scaled per tensor by 448 / max|x|, the fp32 weight per output channel by 448 / max|w_k| -- while its
                   data and weight gradients use the bf16 input and weight copy, as the product's backward does.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

DTYPES = {'bf16_act': torch.bfloat16, 'bf16': torch.bfloat16, 'bf16_sink': torch.bfloat16, 'fp16': torch.float16,
          'fp8': torch.bfloat16, 'fp8_sink': torch.bfloat16}
LOSS_SCALE = {'bf16_act': 1.0, 'bf16': 1.0, 'bf16_sink': 1.0, 'fp16': 2.0 ** 16, 'fp8': 1.0, 'fp8_sink': 1.0}

LEAVES = (nn.Conv2d, nn.BatchNorm2d, nn.SiLU, nn.Upsample, nn.MaxPool2d, nn.Linear, nn.LayerNorm, nn.GELU, nn.Hardswish,
          nn.Sigmoid, nn.AvgPool2d, nn.AdaptiveAvgPool2d, nn.AdaptiveMaxPool2d, nn.ReLU)


class RoundAct(torch.autograd.Function):
    """storage rounding of an activation: forward value and the gradient flowing back through it"""

    @staticmethod
    def forward(ctx, x, dt):
        ctx.dt = dt
        return x.to(dt).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dt).float(), None


class RoundGrad(torch.autograd.Function):
    """identity forward; the gradient flowing back through it rounded (a leaf's input-gradient contribution)"""

    @staticmethod
    def forward(ctx, x, dt):
        ctx.dt = dt
        # a copy, not x.view_as(x): a module that updates its input in place (the C3TR transformer's residual adds)
        # may not modify a view created inside a custom Function
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dt).float(), None


class RoundWeight(torch.autograd.Function):
    """the low-precision weight copy a conv reads; its gradient reaches the fp32 master weight unrounded"""

    @staticmethod
    def forward(ctx, w, dt):
        return w.to(dt).float()

    @staticmethod
    def backward(ctx, g):
        return g, None


def _e4m3(v, amax):
    """quantise-dequantise with the product's convention: v * 448 / amax rounded to OCP e4m3fn (saturated), times
    amax / 448; amax broadcasts (per tensor or per output channel)"""
    inv = torch.where(amax > 0, 448.0 / amax, torch.ones_like(amax))
    q = (v * inv).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float()
    return q * torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))


class F8Conv(torch.autograd.Function):
    """e4m3 forward, bf16 backward (dmy_conv_fwd_fp8 + the bf16 data / weight gradient kernels)"""

    @staticmethod
    def forward(ctx, x, w, stride, padding):
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, padding)
        xq = _e4m3(x, x.abs().amax())
        wq = _e4m3(w, w.abs().flatten(1).amax(1).view(-1, 1, 1, 1))
        return F.conv2d(xq, wq, None, stride, padding)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        s, p = ctx.conf
        wb = w.bfloat16().float()
        gx = torch.nn.grad.conv2d_input(x.shape, wb, g, stride=s, padding=p)
        gw = torch.nn.grad.conv2d_weight(x, w.shape, g, stride=s, padding=p)
        return gx, gw, None, None


def fp8_eligible(m):
    k = m.kernel_size[0]
    return type(m) is nn.Conv2d and m.groups == 1 and k >= 3 and m.in_channels % 128 == 0 and \
        m.out_channels % 8 == 0 and m.out_channels >= 32 and m.bias is None


def _stored_types():
    from oracle import nn as onn
    return tuple(getattr(onn, n) for n in ('Bottleneck', 'CoorAttention', 'AdConcat2', 'AdConcat3',
                                             'SwinTransformerLayer', 'CABottleneck') if hasattr(onn, n))


def emulate(model, mode):
    """install the roundings of `mode` on an oracle model (forward hooks / per-instance forwards); returns it"""
    dt = DTYPES[mode]
    hook = lambda m, i, o: RoundAct.apply(o, dt) if torch.is_tensor(o) else o  # noqa: E731
    for mod in model.modules():
        if isinstance(mod, LEAVES):
            mod.register_forward_hook(hook)
    if mode == 'bf16_act':
        return model
    if mode in ('bf16_sink', 'fp8_sink'):
        pre = lambda m, i: tuple(RoundGrad.apply(a, dt) if torch.is_tensor(a) and a.requires_grad else a  # noqa: E731
                                 for a in i)
        for mod in model.modules():
            if isinstance(mod, LEAVES):
                mod.register_forward_pre_hook(pre)
    for mod in model.modules():
        if isinstance(mod, _stored_types()):
            mod.register_forward_hook(hook)
        if mode in ('fp8', 'fp8_sink') and type(mod) is nn.Conv2d and fp8_eligible(mod):
            mod.forward = (lambda m: lambda x: F8Conv.apply(x, m.weight, m.stride, m.padding))(mod)
        elif type(mod) is nn.Conv2d:
            mod.forward = (lambda m: lambda x: F.conv2d(x, RoundWeight.apply(m.weight, dt), m.bias, m.stride, m.padding,
                                                        m.dilation, m.groups))(mod)
        elif type(mod) is nn.Linear:
            mod.forward = (lambda m: lambda x: F.linear(x, RoundWeight.apply(m.weight, dt), m.bias))(mod)
    from oracle import nn as onn
    if hasattr(onn, 'CBAM'):
        for mod in model.modules():
            if isinstance(mod, onn.ChannelAttentionModule):
                mod.register_forward_hook(hook)  # ca, the sigmoid of the summed MLP branches, is stored
            if isinstance(mod, onn.CBAM):
                def cbam_fwd(x, m=mod):  # the product stores out1 = ca * x, the pooled map, sa and the output
                    out1 = RoundAct.apply(m.channel_attention(x) * x, dt)
                    s2 = RoundAct.apply(torch.cat([out1.mean(1, keepdim=True), out1.max(1, keepdim=True)[0]], 1), dt)
                    sa = RoundAct.apply(torch.sigmoid(m.spatial_attention.conv2d(s2)), dt)
                    return RoundAct.apply(sa * out1, dt)
                mod.forward = cbam_fwd
    if hasattr(onn, 'TransformerLayer'):
        # C3TR (config 5) as the product stores it: the in-projected q / k / v, the attention probabilities P (the
        # flash kernel's bf16 P . V MFMA operand), the attention output o and the two residual sums (out-projection and
        # fc2 with the residual fused into their conv epilogues: one rounding of the sum) -- the oracle calls the
        # projections functionally, so the leaf hooks saw none of them
        rw = lambda w: RoundWeight.apply(w, dt)  # noqa: E731
        ra = lambda t: RoundAct.apply(t, dt)  # noqa: E731
        for mod in model.modules():
            if isinstance(mod, onn.TransformerLayer):
                def tl_fwd(x, m=mod):
                    c = x.shape[-1]
                    x_ = m.ln1(x)
                    q_, k_, v_ = m.q(x_), m.k(x_), m.v(x_)
                    L, B, _ = q_.shape
                    h = m.num_heads
                    d = c // h
                    W, b = m.ma.in_proj_weight, m.ma.in_proj_bias
                    q = ra(F.linear(q_, rw(W[:c]), b[:c])).reshape(L, B * h, d).transpose(0, 1)
                    k = ra(F.linear(k_, rw(W[c:2 * c]), b[c:2 * c])).reshape(L, B * h, d).transpose(0, 1)
                    v = ra(F.linear(v_, rw(W[2 * c:]), b[2 * c:])).reshape(L, B * h, d).transpose(0, 1)
                    a = ra(torch.softmax((q * (1.0 / d ** 0.5)) @ k.transpose(1, 2), dim=-1))
                    o = ra((a @ v).transpose(0, 1).reshape(L, B, c))
                    x = ra(m.dropout(F.linear(o, rw(m.ma.out_proj.weight), m.ma.out_proj.bias)) + x)
                    hd = m.act(m.fc1(m.ln2(x)))
                    return ra(x + m.dropout(F.linear(m.dropout(hd), rw(m.fc2.weight))))
                mod.forward = tl_fwd
            if isinstance(mod, onn.TransformerBlock):
                def tb_fwd(x, m=mod):
                    if m.conv is not None:
                        x = m.conv(x)
                    bsz, _, hh, ww = x.shape
                    p_ = x.flatten(2).permute(2, 0, 1)
                    t = ra(F.linear(p_, rw(m.linear.weight), m.linear.bias) + p_)
                    return m.tr(t).permute(1, 2, 0).reshape(bsz, m.c2, hh, ww)
                mod.forward = tb_fwd
    if hasattr(onn, 'CoorAttention'):
        for mod in model.modules():
            if isinstance(mod, onn.CoorAttention):
                def ca_fwd(x, m=mod):  # the product stores the pooled row / column means (CAPoolFn) in bf16
                    _, _, H, W = x.shape
                    pooled = RoundAct.apply(torch.cat([x.mean(3, keepdim=True), x.mean(2, keepdim=True).transpose(2, 3)],
                                                      2), dt)
                    y = m.act(onn._bn_train_or_eval(m.bn1, m.conv1(pooled)))
                    ah = torch.sigmoid(m.conv_h(y[:, :, :H]))
                    aw = torch.sigmoid(m.conv_w(y[:, :, H:].transpose(2, 3)))
                    return x * aw * ah
                mod.forward = ca_fwd
    if hasattr(onn, 'SCConv'):
        for mod in model.modules():
            if isinstance(mod, onn.SCConv):
                def fwd(x, m=mod):  # oracle SCConv.forward with its gate product stored (scgate_fwd writes it)
                    g = F.interpolate(m.k2(x), size=x.shape[2:], mode='nearest')
                    return m.k4(RoundAct.apply(m.k3(x) * torch.sigmoid(x + g), dt))
                mod.forward = fwd
    return model


def input_round(x, mode):
    return x if mode is None else RoundAct.apply(x, DTYPES[mode])


def oracle_run(cfg, nc, sd, x, t, anchors, hyp, mode, dev='cpu'):
    """the CPU oracle (fp32, or under emulation `mode`) on a product state_dict: train-mode forward of the uint8
    images x, ComputeLoss against targets t, backward.  Returns (model, outputs, loss, items); cfg is a yaml path or
    dict.  DropPath is off (a random draw, not a rounding).  dev='cuda' runs the same torch ops on the GPU (TF32 off):
    another fp32 summation order, i.e. another realization of the emulation's rounding decisions; the loss (CPU
    restatement) then runs over the outputs copied back."""
    import yaml
    from oracle import nn as onn
    from oracle.loss import compute_loss
    if isinstance(cfg, str):
        with open(cfg) as f:
            cfg = yaml.safe_load(f)
    ref = onn.bn_defaults(onn.Model(cfg, nc=nc))
    ref.load_state_dict(sd)
    for mod in ref.modules():
        if hasattr(mod, 'drop_prob'):
            mod.drop_prob = 0.0
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    if mode is not None:
        emulate(ref, mode)
    if dev != 'cpu':
        torch.backends.cudnn.allow_tf32 = False
        torch.backends.cuda.matmul.allow_tf32 = False
        ref = ref.to(dev)
    ref.train()
    pr = ref(input_round(x.to(dev).float() / 255, mode))
    lo, it = compute_loss([p.cpu() for p in pr] if dev != 'cpu' else pr, t, anchors, hyp, nc)
    sc = LOSS_SCALE[mode] if mode else 1.0
    (lo * sc).backward()
    if sc != 1.0:
        for p in ref.parameters():
            if p.grad is not None:
                p.grad.div_(sc)
    if dev != 'cpu':
        ref = ref.cpu()
        pr = [p.detach().cpu() for p in pr]
    return ref, pr, lo, it


def grad_metrics(pg, rg, names):
    """(relative L2 of the per-tensor gradient-norm vector, cosine of the whole gradient) of grads pg vs rg"""
    gn = torch.tensor([float(pg[k].grad.norm()) if pg[k].grad is not None else 0.0 for k in names], dtype=torch.float64)
    gr = torch.tensor([float(rg[k].grad.norm()) for k in names], dtype=torch.float64)
    a = torch.cat([pg[k].grad.double().cpu().flatten() for k in names])
    b = torch.cat([rg[k].grad.double().flatten() for k in names])
    return float((gn - gr).norm() / gr.norm()), float(a @ b / (a.norm() * b.norm()))
