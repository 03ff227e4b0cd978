"""CPU fp32 restatement of the DMA-YOLO module zoo (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Parameter/buffer names follow the reference's state_dict layout so golden state_dicts load
unchanged; the arithmetic is restated, not copied.  Reference anchors (file:line) per class.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def same_pad(k, p=None):
    """models/common.py:33-48 (autopad)."""
    return (k // 2) if p is None else p


def _bn_train_or_eval(bn, z):
    return F.batch_norm(z, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training,
                        bn.momentum, bn.eps)


class Conv(nn.Module):
    """conv -> BN -> SiLU.  models/cspcm.py:11-23 (YAML Conv) == models/common.py:50-77."""

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, same_pad(k, p), groups=g, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.act = nn.SiLU() if act is True else (act if isinstance(act, nn.Module) else nn.Identity())

    def forward(self, x):
        return self.act(_bn_train_or_eval(self.bn, self.conv(x)))

    def forward_fuse(self, x):
        return self.act(self.conv(x))


class Bottleneck(nn.Module):
    """models/common.py:119-137."""

    def __init__(self, c1, c2, shortcut=True, g=1, e=0.5):
        super().__init__()
        h = int(c2 * e)
        self.cv1, self.cv2 = Conv(c1, h, 1, 1), Conv(h, c2, 3, 1, g=g)
        self.add = bool(shortcut and c1 == c2)

    def forward(self, x):
        y = self.cv2(self.cv1(x))
        return x + y if self.add else y


class C3(nn.Module):
    """models/common.py:159-182: cv3(cat(m(cv1 x), cv2 x))."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        h = int(c2 * e)
        self.cv1, self.cv2, self.cv3 = Conv(c1, h, 1, 1), Conv(c1, h, 1, 1), Conv(2 * h, c2, 1)
        self.m = nn.Sequential(*[Bottleneck(h, h, shortcut, g, e=1.0) for _ in range(n)])

    def forward(self, x):
        return self.cv3(torch.cat([self.m(self.cv1(x)), self.cv2(x)], 1))


class SPPF(nn.Module):
    """models/common.py:243-258 (three chained k5 max-pools)."""

    def __init__(self, c1, c2, k=5):
        super().__init__()
        h = c1 // 2
        self.cv1, self.cv2 = Conv(c1, h, 1, 1), Conv(4 * h, c2, 1, 1)
        self.m = nn.MaxPool2d(k, 1, k // 2)

    def forward(self, x):
        a = self.cv1(x)
        b = self.m(a)
        c = self.m(b)
        return self.cv2(torch.cat([a, b, c, self.m(c)], 1))


class SPP(nn.Module):
    """models/common.py:212-227: parallel max-pools (k odd, stride 1, pad k//2) of cv1(x), concat, cv2."""

    def __init__(self, c1, c2, k=(5, 9, 13)):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * (len(k) + 1), c2, 1, 1)
        self.m = nn.ModuleList([nn.MaxPool2d(kernel_size=x, stride=1, padding=x // 2) for x in k])

    def forward(self, x):
        x = self.cv1(x)
        return self.cv2(torch.cat([x] + [m(x) for m in self.m], 1))


class ChannelAttentionModule(nn.Module):
    """models/common.py:260-285: sigmoid(MLP(avgpool x) + MLP(maxpool x)), MLP = Linear-ReLU-Linear, r = 16."""

    def __init__(self, c1, reduction=16):
        super().__init__()
        mid = c1 // reduction
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.shared_MLP = nn.Sequential(nn.Linear(c1, mid), nn.ReLU(), nn.Linear(mid, c1))

    def forward(self, x):
        b = x.shape[0]
        a = self.shared_MLP(self.avg_pool(x).view(b, -1))
        m = self.shared_MLP(self.max_pool(x).view(b, -1))
        return torch.sigmoid(a + m)[:, :, None, None]


class SpatialAttentionModule(nn.Module):
    """models/common.py:287-300: sigmoid(conv7x7(cat(mean_c x, max_c x)))."""

    def __init__(self):
        super().__init__()
        self.conv2d = nn.Conv2d(2, 1, kernel_size=7, stride=1, padding=3)

    def forward(self, x):
        s = torch.cat([x.mean(1, keepdim=True), x.max(1, keepdim=True)[0]], 1)
        return torch.sigmoid(self.conv2d(s))


class CBAM(nn.Module):
    """models/common.py:302-310."""

    def __init__(self, c1, c2):
        super().__init__()
        self.channel_attention = ChannelAttentionModule(c1)
        self.spatial_attention = SpatialAttentionModule()

    def forward(self, x):
        out = self.channel_attention(x) * x
        return self.spatial_attention(out) * out


class SPPFCSPC(nn.Module):
    """models/common.py:1257-1276."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5, k=5):
        super().__init__()
        h = int(2 * c2 * e)
        self.cv1, self.cv2 = Conv(c1, h, 1, 1), Conv(c1, h, 1, 1)
        self.cv3, self.cv4 = Conv(h, h, 3, 1), Conv(h, h, 1, 1)
        self.m = nn.MaxPool2d(k, 1, k // 2)
        self.cv5, self.cv6 = Conv(4 * h, h, 1, 1), Conv(h, h, 3, 1)
        self.cv7 = Conv(2 * h, c2, 1, 1)

    def forward(self, x):
        p0 = self.cv4(self.cv3(self.cv1(x)))
        p1 = self.m(p0)
        p2 = self.m(p1)
        y1 = self.cv6(self.cv5(torch.cat([p0, p1, p2, self.m(p2)], 1)))
        return self.cv7(torch.cat([y1, self.cv2(x)], 1))


class SCConv(nn.Module):
    """Self-calibrated conv, models/common.py:1279-1316: k4(k3(x) * sigmoid(x + nearest(k2(x))))."""

    def __init__(self, c1, c2, stride, groups=1, dilation=1, pooling_r=4):
        super().__init__()
        conv = lambda ci, co, s: nn.Conv2d(ci, co, 3, s, 1, dilation=dilation, groups=groups, bias=False)
        self.k2 = nn.Sequential(nn.AvgPool2d(pooling_r, pooling_r), conv(c1, c1, 1), nn.BatchNorm2d(c1))
        self.k3 = nn.Sequential(conv(c1, c1, 1), nn.BatchNorm2d(c1))
        self.k4 = nn.Sequential(conv(c1, c2, stride), nn.BatchNorm2d(c2))

    def forward(self, x):
        g = F.interpolate(self.k2(x), size=x.shape[2:], mode='nearest')
        return self.k4(self.k3(x) * torch.sigmoid(x + g))


class CoorAttention(nn.Module):
    """Coordinate attention, models/common.py:1158-1207 (YAML token CA)."""

    def __init__(self, c1, c2, reduction=32):
        super().__init__()
        mid = max(8, c1 // reduction)
        self.conv1 = nn.Conv2d(c1, mid, 1, 1, 0)
        self.bn1 = nn.BatchNorm2d(mid)
        self.act = nn.Hardswish()
        self.conv_w = nn.Conv2d(mid, c2, 1, 1, 0)
        self.conv_h = nn.Conv2d(mid, c2, 1, 1, 0)

    def forward(self, x):
        _, _, H, W = x.shape
        rows = x.mean(3, keepdim=True)                      # [N,C,H,1]
        cols = x.mean(2, keepdim=True).transpose(2, 3)      # [N,C,W,1]
        y = self.act(_bn_train_or_eval(self.bn1, self.conv1(torch.cat([rows, cols], 2))))
        yh, yw = y[:, :, :H], y[:, :, H:]
        ah = torch.sigmoid(self.conv_h(yh))                 # [N,C,H,1]
        aw = torch.sigmoid(self.conv_w(yw.transpose(2, 3)))  # [N,C,1,W]
        return x * aw * ah


CA = CoorAttention


class CABottleneck(nn.Module):
    """models/common.py:1209-1227."""

    def __init__(self, c1, c2, shortcut=True, g=1, e=0.5, reduction=32):
        super().__init__()
        h = int(c2 * e)
        self.cv1, self.cv2 = Conv(c1, h, 1, 1), Conv(h, c2, 3, 1, g=g)
        self.ca = CoorAttention(c2, c2, reduction)
        self.add = bool(shortcut and c1 == c2)

    def forward(self, x):
        y = self.ca(self.cv2(self.cv1(x)))
        return x + y if self.add else y


class C3CA(C3):
    """models/common.py:1229-1235."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__(c1, c2, n, shortcut, g, e)
        h = int(c2 * e)
        self.m = nn.Sequential(*[CABottleneck(h, h, shortcut, g, e=1.0) for _ in range(n)])


class Concat(nn.Module):
    """models/common.py:656-664."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def forward(self, x):
        return torch.cat(x, self.d)


class _AdConcat(nn.Module):
    """BiFPN fast-normalised weighted concat, models/common.py:994-1026."""
    K = 2

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension
        self.w = nn.Parameter(torch.ones(self.K, dtype=torch.float32))
        self.epsilon = 1e-4

    def forward(self, x):
        wn = self.w / (self.w.sum(0) + self.epsilon)
        return torch.cat([wn[i] * x[i] for i in range(self.K)], self.d)


class AdConcat2(_AdConcat):
    K = 2


class AdConcat3(_AdConcat):
    K = 3


# ---------------------------------------------------------------- Swin (C3STR)

def swin_region_labels(R, Cc, ws, shift):
    """Label map of create_mask() INCLUDING the reference bug (models/common.py:569-593).

    h_slices[0] is the tuple (0, -ws): only rows 0 and R-ws receive the first label row, later
    slices overwrite in order.  Returns int tensor [R, Cc] in Swin space (rows = image W axis).
    """
    lab = torch.zeros(R, Cc, dtype=torch.int64)
    col = torch.zeros(Cc, dtype=torch.int64)
    cidx = torch.arange(Cc)
    col[(cidx >= Cc - ws) & (cidx < Cc - shift)] = 1
    col[cidx >= Cc - shift] = 2
    if Cc - ws <= 0:  # slice(0, -ws) empty
        pass
    for r in {0, R - ws}:
        lab[r] = col
    ridx = torch.arange(R)
    sel = (ridx >= R - ws) & (ridx < R - shift)
    lab[sel] = 3 + col
    lab[ridx >= R - shift] = 6 + col
    return lab


def swin_mask(R, Cc, ws, shift):
    lab = swin_region_labels(R, Cc, ws, shift)
    win = lab.view(R // ws, ws, Cc // ws, ws).permute(0, 2, 1, 3).reshape(-1, ws * ws)
    d = win[:, None, :] - win[:, :, None]
    return torch.where(d != 0, torch.tensor(-100.0), torch.tensor(0.0))  # [nW, N, N]


def rel_pos_index(ws):
    """models/common.py:479-490: (dr + ws-1) * (2ws-1) + (dc + ws-1)."""
    r = torch.arange(ws).repeat_interleave(ws)
    c = torch.arange(ws).repeat(ws)
    return (r[:, None] - r[None, :] + ws - 1) * (2 * ws - 1) + (c[:, None] - c[None, :] + ws - 1)


class Mlp(nn.Module):
    """models/common.py:97-117."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden_features or in_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features or in_features, out_features or in_features)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class WindowAttention(nn.Module):
    """models/common.py:452-545."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, attn_drop=0., proj_drop=0.):
        super().__init__()
        self.dim, self.window_size, self.num_heads = dim, window_size, num_heads
        self.scale = (dim // num_heads) ** -0.5
        ws = window_size[0]
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) ** 2, num_heads))
        self.register_buffer('relative_position_index', rel_pos_index(ws))
        self.qkv = nn.Linear(dim, 3 * dim, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x, mask=None):
        Bw, N, C = x.shape
        h = self.num_heads
        q, k, v = self.qkv(x).view(Bw, N, 3, h, C // h).permute(2, 0, 3, 1, 4)
        s = (q * self.scale) @ k.transpose(-1, -2)
        bias = self.relative_position_bias_table[self.relative_position_index.reshape(-1)].view(N, N, h)
        s = s + bias.permute(2, 0, 1)[None]
        if mask is not None:
            nW = mask.shape[0]
            s = (s.view(Bw // nW, nW, h, N, N) + mask[None, :, None]).view(Bw, h, N, N)
        a = torch.softmax(s, -1)
        return self.proj((a @ v).transpose(1, 2).reshape(Bw, N, C))


class SwinTransformerLayer(nn.Module):
    """models/common.py:547-637.  Operates on x.permute(0,3,2,1) = [B, W, H, C]."""

    def __init__(self, c, num_heads, window_size=7, shift_size=0, mlp_ratio=4, qkv_bias=False, drop=0.,
                 attn_drop=0., drop_path=0., act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.window_size, self.shift_size = window_size, shift_size
        self.drop_prob = 0.1 if num_heads > 10 else drop_path  # common.py:553-554 (forced 0 in parity tests)
        self.norm1 = norm_layer(c)
        self.attn = WindowAttention(c, (window_size, window_size), num_heads, qkv_bias=qkv_bias)
        self.norm2 = norm_layer(c)
        self.mlp = Mlp(c, int(c * mlp_ratio), act_layer=act_layer)

    def forward(self, x):
        B, C, Hi, Wi = x.shape
        ws, sh = self.window_size, self.shift_size
        t = x.permute(0, 3, 2, 1)                           # [B, R=Wi, Cc=Hi, C]
        R, Cc = Wi, Hi
        u = self.norm1(t)
        Rp, Cp = -(-R // ws) * ws, -(-Cc // ws) * ws
        u = F.pad(u, (0, 0, 0, Cp - Cc, 0, Rp - R))
        if sh > 0:
            u = torch.roll(u, (-sh, -sh), (1, 2))
            mask = swin_mask(Rp, Cp, ws, sh).to(u.device)
        else:
            mask = None
        win = u.view(B, Rp // ws, ws, Cp // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, C)
        o = self.attn(win, mask)
        o = o.view(B, Rp // ws, Cp // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, Rp, Cp, C)
        if sh > 0:
            o = torch.roll(o, (sh, sh), (1, 2))
        t = t + o[:, :R, :Cc]
        t = t + self.mlp(self.norm2(t))
        return t.permute(0, 3, 2, 1)


class SwinTransformerBlock(nn.Module):
    """models/common.py:639-654."""

    def __init__(self, c1, c2, num_heads, num_layers, window_size=8):
        super().__init__()
        self.conv = Conv(c1, c2) if c1 != c2 else None
        self.tr = nn.Sequential(*[SwinTransformerLayer(c2, num_heads, window_size,
                                                       0 if i % 2 == 0 else window_size // 2)
                                  for i in range(num_layers)])

    def forward(self, x):
        return self.tr(self.conv(x) if self.conv is not None else x)


class C3STR(C3):
    """models/common.py:191-196."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__(c1, c2, n, shortcut, g, e)
        h = int(c2 * e)
        self.m = SwinTransformerBlock(h, h, h // 32, n)


# ---------------------------------------------------------------- C3TR (config 5: global MHSA over P5 tokens)

class TransformerLayer(nn.Module):
    """models/common.py:312-336: x + Dropout(MHA(q(LN1 x), k(LN1 x), v(LN1 x))), then
    x + Dropout(fc2(Dropout(ReLU(fc1(LN2 x))))).  The nn.MultiheadAttention (common.py:323) is
    restated with explicit math (torch/nn/functional.py multi_head_attention_forward, need_weights
    path: in-projection, q scaled by head_dim^-1/2, softmax(q k^T), @ v, out-projection); the module
    is kept only as the holder of in_proj_weight / in_proj_bias / out_proj (state_dict keys)."""

    def __init__(self, c, num_heads):
        super().__init__()
        self.ln1 = nn.LayerNorm(c)
        self.q = nn.Linear(c, c, bias=False)
        self.k = nn.Linear(c, c, bias=False)
        self.v = nn.Linear(c, c, bias=False)
        self.ma = nn.MultiheadAttention(embed_dim=c, num_heads=num_heads)
        self.ln2 = nn.LayerNorm(c)
        self.fc1 = nn.Linear(c, 4 * c, bias=False)
        self.fc2 = nn.Linear(4 * c, c, bias=False)
        self.dropout = nn.Dropout(0.1)
        self.act = nn.ReLU(True)
        self.num_heads = num_heads

    def mha(self, q, k, v):
        """[L, B, c] sequence-first in, [L, B, c] out."""
        L, B, c = q.shape
        h = self.num_heads
        d = c // h
        W, b = self.ma.in_proj_weight, self.ma.in_proj_bias
        q = F.linear(q, W[:c], b[:c])
        k = F.linear(k, W[c:2 * c], b[c:2 * c])
        v = F.linear(v, W[2 * c:], b[2 * c:])
        q = q.reshape(L, B * h, d).transpose(0, 1) * (1.0 / math.sqrt(d))
        k = k.reshape(L, B * h, d).transpose(0, 1)
        v = v.reshape(L, B * h, d).transpose(0, 1)
        a = torch.softmax(q @ k.transpose(1, 2), dim=-1)
        o = (a @ v).transpose(0, 1).reshape(L, B, c)
        return F.linear(o, self.ma.out_proj.weight, self.ma.out_proj.bias)

    def forward(self, x):
        x_ = self.ln1(x)
        x = self.dropout(self.mha(self.q(x_), self.k(x_), self.v(x_))) + x
        x_ = self.ln2(x)
        x_ = self.fc2(self.dropout(self.act(self.fc1(x_))))
        return x + self.dropout(x_)


class TransformerBlock(nn.Module):
    """models/common.py:338-355: tokens = pixels in (H, W) row-major order, sequence-first [HW, B, c];
    learned position term p + linear(p); output back to [B, c, H, W]."""

    def __init__(self, c1, c2, num_heads, num_layers):
        super().__init__()
        self.conv = Conv(c1, c2) if c1 != c2 else None
        self.linear = nn.Linear(c2, c2)
        self.tr = nn.Sequential(*(TransformerLayer(c2, num_heads) for _ in range(num_layers)))
        self.c2 = c2

    def forward(self, x):
        if self.conv is not None:
            x = self.conv(x)
        b, _, h, w = x.shape
        p = x.flatten(2).permute(2, 0, 1)
        return self.tr(p + self.linear(p)).permute(1, 2, 0).reshape(b, self.c2, h, w)


class C3TR(C3):
    """models/common.py:184-189: C3 whose bottleneck stack is a TransformerBlock(c_, c_, 4 heads, n)."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__(c1, c2, n, shortcut, g, e)
        h = int(c2 * e)
        self.m = TransformerBlock(h, h, 4, n)


# ---------------------------------------------------------------- Detect / Model

class Detect(nn.Module):
    """models/yolo.py:40-114."""
    stride = None

    def __init__(self, nc=80, anchors=(), ch=(), inplace=True):
        super().__init__()
        self.nc, self.no, self.nl, self.na = nc, nc + 5, len(anchors), len(anchors[0]) // 2
        self.register_buffer('anchors', torch.tensor(anchors).float().view(self.nl, -1, 2))
        self.m = nn.ModuleList(nn.Conv2d(c, self.no * self.na, 1) for c in ch)
        self.inplace = inplace

    def forward(self, xs):
        outs, z = [], []
        for i in range(self.nl):
            y = self.m[i](xs[i])
            b, _, ny, nx = y.shape
            y = y.view(b, self.na, self.no, ny, nx).permute(0, 1, 3, 4, 2).contiguous()
            outs.append(y)
            if not self.training:
                gy, gx = torch.meshgrid(torch.arange(ny), torch.arange(nx), indexing='ij')
                grid = torch.stack((gx, gy), 2).view(1, 1, ny, nx, 2).float()
                ag = (self.anchors[i] * self.stride[i]).view(1, self.na, 1, 1, 2)
                s = y.sigmoid()
                xy = (s[..., :2] * 2 - 0.5 + grid) * self.stride[i]
                wh = (s[..., 2:4] * 2) ** 2 * ag
                z.append(torch.cat([xy, wh, s[..., 4:]], -1).view(b, -1, self.no))
        return outs if self.training else (torch.cat(z, 1), outs)


def make_divisible(x, d):
    return math.ceil(x / d) * d


_CHANNEL_MODS = ('Conv', 'Bottleneck', 'SPPF', 'C3', 'C3TR', 'C3STR', 'CoorAttention', 'CA', 'CABottleneck', 'C3CA',
                 'SPPFCSPC', 'SCConv', 'SPP', 'CBAM')
_REPEAT_MODS = ('C3', 'C3TR', 'C3STR', 'C3CA')


def _eval_arg(a, env):
    if not isinstance(a, str):
        return a
    try:
        return eval(a, env)
    except NameError:
        return a


def parse_model(d, ch):
    """models/yolo.py:353-478 restricted to the hot-path module set."""
    anchors, nc, gd, gw = d['anchors'], d['nc'], d['depth_multiple'], d['width_multiple']
    na = (len(anchors[0]) // 2) if isinstance(anchors, list) else anchors
    no = na * (nc + 5)
    layers, save, c2 = [], [], ch[-1]
    env = dict(globals(), nc=nc, anchors=anchors, nn=nn)
    for i, (f, n, mname, args) in enumerate(d['backbone'] + d['head']):
        m = eval(mname, env) if isinstance(mname, str) else mname
        args = [_eval_arg(a, env) for a in args]
        n_ = n = max(round(n * gd), 1) if n > 1 else n
        name = mname.split('.')[-1]
        if name in _CHANNEL_MODS:
            c1, c2 = ch[f], args[0]
            if c2 != no:
                c2 = make_divisible(c2 * gw, 8)
            args = [c1, c2, *args[1:]]
            if name == 'CA':
                m = CoorAttention
            if name in _REPEAT_MODS:
                args.insert(2, n)
                n = 1
        elif name in ('Concat', 'AdConcat2', 'AdConcat3'):
            c2 = sum(ch[x] for x in f)
        elif name == 'Detect':
            args.append([ch[x] for x in f])
            if isinstance(args[1], int):
                args[1] = [list(range(args[1] * 2))] * len(f)
        else:
            c2 = ch[f]
        mod = nn.Sequential(*[m(*args) for _ in range(n)]) if n > 1 else m(*args)
        mod.i, mod.f = i, f
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(mod)
        if i == 0:
            ch = []
        ch.append(c2)
    return nn.Sequential(*layers), sorted(save)


class Model(nn.Module):
    """models/yolo.py:117-239 (forward path only; weights come from state_dict transfer)."""

    def __init__(self, cfg, ch=3, nc=None, stride=None):
        super().__init__()
        import copy
        self.yaml = copy.deepcopy(cfg)
        if nc:
            self.yaml['nc'] = nc
        self.model, self.save = parse_model(copy.deepcopy(self.yaml), [ch])
        det = self.model[-1]
        if stride is None:  # P3-P5 heads (8, 16, 32); the config-5 head adds P2 (4)
            stride = (4., 8., 16., 32.)[-det.nl:]
        det.stride = torch.tensor(stride)
        self.stride = det.stride

    def forward(self, x):
        ys = []
        for m in self.model:
            if m.f != -1:
                x = ys[m.f] if isinstance(m.f, int) else [x if j == -1 else ys[j] for j in m.f]
            x = m(x)
            ys.append(x if m.i in self.save else None)
        return x


def bn_defaults(model):
    """utils/torch_utils.py:161-170 (initialize_weights): BN eps 1e-3, momentum 0.03."""
    for m in model.modules():
        if type(m) is nn.BatchNorm2d:
            m.eps, m.momentum = 1e-3, 0.03
    return model
