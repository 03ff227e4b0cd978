"""Swin (C3STR) modules — models/common.py:97-117, 191-196, 386-654.  Kernels: csrc/swin.hip."""
import torch
import torch.nn as nn

from .. import functional as Fn


class DropPath(nn.Module):
    """models/common.py:386-413 (stochastic depth, per-sample)."""

    def __init__(self, drop_prob=None):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        """Per-sample stochastic depth on the HIP path (the keep mask is drawn with torch's RNG)."""
        if self.drop_prob == 0. or not self.training or not self.drop_prob:
            return x
        keep = 1 - self.drop_prob
        s = (keep + torch.rand((x.shape[0],), dtype=torch.float32, device=x.device)).floor_().div_(keep)
        return Fn.SampleScaleFn.apply(x, s)

    def add(self, x, f, xsink=None):
        """x + self(f) in one pass (functional.DropPathAddFn): the same uniforms and keep rule as forward"""
        u = torch.rand((f.shape[0],), dtype=torch.float32, device=f.device)
        return Fn.DropPathAddFn.apply(x, f, u, 1 - self.drop_prob, xsink)


class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.drop1 = nn.Dropout(drop)
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop2 = nn.Dropout(drop)


class WindowAttention(nn.Module):
    def __init__(self, dim, window_size, num_heads, qkv_bias=True, attn_drop=0., proj_drop=0.):
        super().__init__()
        self.dim, self.window_size, self.num_heads = dim, window_size, num_heads
        self.scale = (dim // num_heads) ** -0.5
        ws = window_size[0]
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) * (2 * window_size[1] - 1),
                                                                     num_heads))
        r = torch.arange(ws).repeat_interleave(window_size[1])
        c = torch.arange(window_size[1]).repeat(ws)
        idx = (r[:, None] - r[None, :] + ws - 1) * (2 * window_size[1] - 1) + (c[:, None] - c[None, :] +
                                                                               window_size[1] - 1)
        self.register_buffer('relative_position_index', idx)
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=.02)


class SwinTransformerLayer(nn.Module):
    def __init__(self, c, num_heads, window_size=7, shift_size=0, mlp_ratio=4, qkv_bias=False, drop=0.,
                 attn_drop=0., drop_path=0., act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        if num_heads > 10:
            drop_path = 0.1
        self.window_size, self.shift_size, self.mlp_ratio = window_size, shift_size, mlp_ratio
        self.norm1 = norm_layer(c)
        self.attn = WindowAttention(c, window_size=(window_size, window_size), num_heads=num_heads,
                                    qkv_bias=qkv_bias, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = DropPath(drop_path) if drop_path > 0. else nn.Identity()
        self.norm2 = norm_layer(c)
        self.mlp = Mlp(in_features=c, hidden_features=int(c * mlp_ratio), act_layer=act_layer, drop=drop)

    def forward(self, x, out=None):
        """common.py:595-637 on NHWC tokens: LN -> qkv -> shifted-window attention (pad/roll/partition
        folded into the kernel's addressing) -> proj (+ residual) -> LN -> MLP(GELU) (+ residual).
        out: a concat_buffer slice the final residual sum is written into (C3STR; not with an active DropPath)."""
        c = x.shape[1]
        a = self.attn
        s1, s2 = Fn.GradSink(2), Fn.GradSink(2)  # x -> norm1 + residual; x2 -> norm2 + residual
        u = Fn.LayerNormFn.apply(x, self.norm1.weight, self.norm1.bias, self.norm1.eps, s1)
        qkv = Fn.conv_bn_act(u, a.qkv.weight.view(3 * c, c, 1, 1), a.qkv.bias, None, 1, 0, Fn.ACT_NONE)
        o = Fn.WinAttnFn.apply(qkv, a.relative_position_bias_table, a.num_heads, self.shift_size, a.scale)
        dp = isinstance(self.drop_path, DropPath) and self.training and self.drop_path.drop_prob
        if dp:
            x = self.drop_path.add(x, Fn.conv_bn_act(o, a.proj.weight.view(c, c, 1, 1), a.proj.bias, None, 1, 0,
                                                     Fn.ACT_NONE), s1)
        else:
            x = Fn.conv_bn_act(o, a.proj.weight.view(c, c, 1, 1), a.proj.bias, None, 1, 0, Fn.ACT_NONE, res=x,
                               rsink=s1)
        m = self.mlp
        u2 = Fn.LayerNormFn.apply(x, self.norm2.weight, self.norm2.bias, self.norm2.eps, s2)
        hd = m.fc1.weight.shape[0]
        h = Fn.conv_bn_act(u2, m.fc1.weight.view(hd, c, 1, 1), m.fc1.bias, None, 1, 0, Fn.ACT_GELU)
        if dp:
            return self.drop_path.add(x, Fn.conv_bn_act(h, m.fc2.weight.view(c, hd, 1, 1), m.fc2.bias, None, 1, 0,
                                                        Fn.ACT_NONE), s2)
        return Fn.conv_bn_act(h, m.fc2.weight.view(c, hd, 1, 1), m.fc2.bias, None, 1, 0, Fn.ACT_NONE, res=x,
                              rsink=s2, out=out)


class SwinTransformerBlock(nn.Module):
    def __init__(self, c1, c2, num_heads, num_layers, window_size=8):
        super().__init__()
        from .common import Conv
        self.conv = Conv(c1, c2) if c1 != c2 else None
        self.window_size = window_size
        self.shift_size = window_size // 2
        self.tr = nn.Sequential(*(SwinTransformerLayer(c2, num_heads=num_heads, window_size=window_size,
                                                       shift_size=0 if (i % 2 == 0) else self.shift_size)
                                  for i in range(num_layers)))

    dmy_out = True  # forward(x, out=view) writes its result into a concat_buffer slice when it can (C3.forward)

    def forward(self, x, out=None):
        if self.conv is not None:
            x = self.conv(x)
        layers = list(self.tr)
        for layer in layers[:-1]:
            x = layer(x)
        return layers[-1](x, out=out) if layers else x


