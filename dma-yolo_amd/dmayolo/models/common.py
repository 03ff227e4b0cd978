"""Drop-in replacements for the reference's YAML modules (models/common.py, models/cspcm.py).

Same class names, constructor signatures, parameter/buffer names (state_dict keys) and the
attributes other reference code reads (`Conv.conv/.bn/.forward_fuse`, `AdConcat*.w`, real
nn.BatchNorm2d / nn.Conv2d instances for optimizer grouping and initialize_weights).
forward() runs the gfx950 kernels through dmayolo.functional; there is no CPU path.

Activation tensors are NHWC (torch.channels_last) in the model's storage dtype.
"""
import math
import os
import weakref

import torch
import torch.nn as nn

from .. import functional as Fn
from ..functional import ACT_NONE, ACT_SILU, ACT_HARDSWISH, ACT_SIGMOID, ACT_GELU, ACT_RELU

__all__ = ['autopad', 'Conv', 'Bottleneck', 'C3', 'SPPF', 'SPPFCSPC', 'SCConv', 'CoorAttention', 'CA',
           'CABottleneck', 'C3CA', 'Concat', 'AdConcat2', 'AdConcat3', 'Upsample', 'C3STR', 'SwinTransformerBlock',
           'SwinTransformerLayer', 'WindowAttention', 'Mlp', 'DropPath', 'space_to_depth', 'SPP', 'CBAM',
           'ChannelAttentionModule', 'SpatialAttentionModule', 'C3TR', 'TransformerBlock', 'TransformerLayer']


def autopad(k, p=None):
    """models/common.py:33-48."""
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


def act_code(m):
    if m is None or isinstance(m, nn.Identity):
        return ACT_NONE
    if isinstance(m, nn.SiLU):
        return ACT_SILU
    if isinstance(m, nn.Hardswish):
        return ACT_HARDSWISH
    if isinstance(m, nn.Sigmoid):
        return ACT_SIGMOID
    if isinstance(m, nn.GELU):
        return ACT_GELU
    if isinstance(m, nn.ReLU):
        return ACT_RELU
    raise NotImplementedError(f'activation {type(m).__name__} has no gfx950 kernel')


def _pad_int(p):
    return p if isinstance(p, int) else p[0]


def conv_forward(conv, bn, act, x, res=None, xsink=None, rsink=None, out=None, defer=False):
    """conv (nn.Conv2d, groups=1, dilation=1) -> optional BN -> act (+ residual) on the HIP path.
    xsink / rsink: Fn.GradSink for the gradients of x / res when they have other consumers.  defer: a train-mode BN
    layer without activation returns its pre-BN output for a consumer that applies the BN itself (SCConv's gate)"""
    assert conv.groups == 1 and conv.dilation in (1, (1, 1)), 'grouped/dilated conv not on the DMA-YOLO path'
    s = conv.stride if isinstance(conv.stride, int) else conv.stride[0]
    pad, a = _pad_int(conv.padding), act_code(act)
    return Fn.conv_bn_act(x, conv.weight, conv.bias, bn, s, pad, a, res=res, spec=Fn.spec_for(conv, s, pad, a, bn),
                          xsink=xsink, rsink=rsink, out=out, defer=defer)


class Conv(nn.Module):
    """conv + BN + SiLU: models/cspcm.py:11-23 (YAML-level Conv) == models/common.py:50-77."""

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p), groups=g, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.act = nn.SiLU() if act is True else (act if isinstance(act, nn.Module) else nn.Identity())

    def forward(self, x, res=None, xsink=None, rsink=None, out=None):
        return conv_forward(self.conv, self.bn, self.act, x, res, xsink, rsink, out)

    def forward_fuse(self, x, res=None, xsink=None, rsink=None, out=None):
        return conv_forward(self.conv, None, self.act, x, res, xsink, rsink, out)


class Bottleneck(nn.Module):
    """models/common.py:119-137; the residual add is fused into cv2's BN/act epilogue."""

    def __init__(self, c1, c2, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_, c2, 3, 1, g=g)
        self.add = shortcut and c1 == c2

    def forward(self, x, out=None):
        if not self.add:
            return self.cv2(self.cv1(x), out=out)
        sk = Fn.GradSink(2)  # x -> cv1 and the residual
        return self.cv2(self.cv1(x, xsink=sk), res=x, rsink=sk, out=out)


# in-place C3 concat (C3.forward): 0 off (copy), 1 Bottleneck stacks, 2 also Swin blocks (C3STR); DMY_INPLACE_CAT
_INPLACE_CAT = int(os.environ.get('DMY_INPLACE_CAT', '2'))


# inference: C3's cv1 and cv2 (both 1x1 over x) as ONE conv with their weights / BN stacked; DMY_C3_PAIR (default on)
_C3_PAIR = os.environ.get('DMY_C3_PAIR', '1') == '1'
_PAIRS = weakref.WeakKeyDictionary()  # C3 module -> (source key, weight, bias, bn, act); not module state, so no
# state_dict / checkpoint entry


class _PairBN:
    """two eval-mode BatchNorm2d side by side (the stacked cv1 | cv2 of C3._pair), as conv_bn_act reads one"""
    training, track_running_stats, momentum = False, True, None

    def __init__(self, a, b):
        self.eps = a.eps
        self.weight, self.bias, self.running_mean, self.running_var = (
            torch.cat([getattr(a, n).detach(), getattr(b, n).detach()])
            for n in ('weight', 'bias', 'running_mean', 'running_var'))


class C3(nn.Module):
    """models/common.py:159-182."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, e=1.0) for _ in range(n)))

    def _pair(self):
        """(weight, bias, bn, act) of cv1 | cv2 stacked along the output channels, rebuilt when a source parameter or
        BN buffer changes (torch _version / Fn.PARAM_GEN); None when the two layers cannot share a launch"""
        c1, c2 = self.cv1, self.cv2
        b1, b2 = getattr(c1, 'bn', None), getattr(c2, 'bn', None)
        w1, w2 = c1.conv.weight, c2.conv.weight
        if (b1 is None) != (b2 is None) or type(c1.act) is not type(c2.act) or w1.shape[1:] != w2.shape[1:] or \
                tuple(w1.shape[2:]) != (1, 1) or tuple(c1.conv.stride) != (1, 1) or tuple(c2.conv.stride) != (1, 1) or \
                (b1 is not None and (b1.eps != b2.eps or b1.training or b2.training)) or \
                (c1.conv.bias is None) != (c2.conv.bias is None):
            return None
        srcs = [w1, w2, c1.conv.bias, c2.conv.bias] + ([b1.weight, b1.bias, b1.running_mean, b1.running_var, b2.weight,
                                                        b2.bias, b2.running_mean, b2.running_var] if b1 is not None else [])
        key = (Fn.PARAM_GEN[0],) + tuple((t.data_ptr(), t._version) if t is not None else None for t in srcs)
        ent = _PAIRS.get(self)
        if ent is None or ent[0] != key:
            w = torch.cat([w1.detach(), w2.detach()])
            b = torch.cat([c1.conv.bias.detach(), c2.conv.bias.detach()]) if c1.conv.bias is not None else None
            ent = _PAIRS[self] = (key, w, b, _PairBN(b1, b2) if b1 is not None else None, act_code(c1.act))
        return ent[1:]

    def forward(self, x, out=None):
        """out: a concat_buffer slice cv3 writes the block's output into (Model's concat plan)"""
        blocks = list(self.m) if isinstance(self.m, nn.Sequential) else []
        seq = bool(blocks) and type(blocks[-1]) is Bottleneck and _INPLACE_CAT >= 1
        pair = self._pair() if seq and _C3_PAIR and not self.training and not torch.is_grad_enabled() else None
        if pair is not None:
            # inference: one 1x1 launch writes cv1's and cv2's activations into the two halves of the concat buffer;
            # the Bottleneck stack starts from the first half and its last block writes its output back over it (for
            # one block that is its own residual input: each output element is read as the residual, then written, by
            # the epilogue that owns it), so cv3 reads the buffer as the concat
            w, b, bn, act = pair
            c_ = w.shape[0] // 2
            cat = Fn.concat_buffer(x.shape[0], 2 * c_, x.shape[2], x.shape[3], x)
            Fn.conv_bn_act(x, w, b, bn, 1, 0, act, out=cat)
            a = cat[:, :c_]
            for blk in blocks[:-1]:
                a = blk(a)
            a = blocks[-1](a, out=cat[:, :c_])
            return self.cv3(Fn.ConcatFn.apply(None, 0.0, None, a, cat[:, c_:]), out=out)
        sk = Fn.GradSink(2)  # x -> cv1 and cv2
        a = self.cv1(x, xsink=sk)
        if not seq and not (getattr(self.m, 'dmy_out', False) and _INPLACE_CAT >= 2):
            return self.cv3(Fn.ConcatFn.apply(None, 0.0, None, self.m(a), self.cv2(x, xsink=sk)), out=out)
        # the last Bottleneck (or the Swin block) and cv2 write their activations straight into the two halves of the
        # concat buffer; a producer that cannot (e.g. an active DropPath) returns its own tensor and ConcatFn copies
        c_ = a.shape[1]
        cat = Fn.concat_buffer(a.shape[0], 2 * c_, a.shape[2], a.shape[3], a)
        if seq:
            for b in blocks[:-1]:
                a = b(a)
            a = blocks[-1](a, out=cat[:, :c_])
        else:
            a = self.m(a, out=cat[:, :c_])
        return self.cv3(Fn.ConcatFn.apply(None, 0.0, None, a, self.cv2(x, xsink=sk, out=cat[:, c_:])), out=out)


class SPPF(nn.Module):
    """models/common.py:243-258."""

    def __init__(self, c1, c2, k=5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * 4, c2, 1, 1)
        self.m = nn.MaxPool2d(kernel_size=k, stride=1, padding=k // 2)

    def forward(self, x):
        k = self.m.kernel_size
        c_ = self.cv1.conv.out_channels
        if _INPLACE_CAT >= 1:  # cv1 and the three pools write straight into the concat buffer's slices: no copies
            cat = Fn.concat_buffer(x.shape[0], 4 * c_, x.shape[2], x.shape[3], x)
            sl = [cat[:, i * c_:(i + 1) * c_] for i in range(4)]
        else:
            sl = [None] * 4
        x = self.cv1(x, out=sl[0])
        ys = Fn.maxpool_chain3(x, k, sl[1:])  # inference: the three pools in one launch
        if ys is not None:
            return self.cv2(Fn.ConcatFn.apply(None, 0.0, None, x, *ys))
        s0, s1, s2 = Fn.GradSink(2), Fn.GradSink(2), Fn.GradSink(2)  # each pool input -> next pool + concat
        y1 = Fn.MaxPoolFn.apply(x, k, s0, sl[1:2])
        y2 = Fn.MaxPoolFn.apply(y1, k, s1, sl[2:3])
        return self.cv2(Fn.ConcatFn.apply(None, 0.0, (s0, s1, s2, None), x, y1, y2,
                                          Fn.MaxPoolFn.apply(y2, k, s2, sl[3:4])))


class SPPFCSPC(nn.Module):
    """models/common.py:1257-1276."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5, k=5):
        super().__init__()
        c_ = int(2 * c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(c_, c_, 3, 1)
        self.cv4 = Conv(c_, c_, 1, 1)
        self.m = nn.MaxPool2d(kernel_size=k, stride=1, padding=k // 2)
        self.cv5 = Conv(4 * c_, c_, 1, 1)
        self.cv6 = Conv(c_, c_, 3, 1)
        self.cv7 = Conv(2 * c_, c2, 1, 1)

    def forward(self, x):
        k = self.m.kernel_size
        c_ = self.cv1.conv.out_channels
        N, H, W = x.shape[0], x.shape[2], x.shape[3]
        if _INPLACE_CAT >= 1:  # every concat input written straight into its slice (cv4 + the pools, cv6 + cv2)
            cat = Fn.concat_buffer(N, 4 * c_, H, W, x)
            sl = [cat[:, i * c_:(i + 1) * c_] for i in range(4)]
            cat2 = Fn.concat_buffer(N, 2 * c_, H, W, x)
            s2l = [cat2[:, :c_], cat2[:, c_:]]
        else:
            sl, s2l = [None] * 4, [None] * 2
        sx = Fn.GradSink(2)  # x -> cv1 and cv2
        x1 = self.cv4(self.cv3(self.cv1(x, xsink=sx)), out=sl[0])
        ys = Fn.maxpool_chain3(x1, k, sl[1:])  # inference: the three pools in one launch
        if ys is not None:
            y1 = self.cv6(self.cv5(Fn.ConcatFn.apply(None, 0.0, None, x1, *ys)), out=s2l[0])
        else:
            s1, s2, s3 = Fn.GradSink(2), Fn.GradSink(2), Fn.GradSink(2)
            x2 = Fn.MaxPoolFn.apply(x1, k, s1, sl[1:2])
            x3 = Fn.MaxPoolFn.apply(x2, k, s2, sl[2:3])
            y1 = self.cv6(self.cv5(Fn.ConcatFn.apply(None, 0.0, (s1, s2, s3, None), x1, x2, x3,
                                                     Fn.MaxPoolFn.apply(x3, k, s3, sl[3:4]))), out=s2l[0])
        y2 = self.cv2(x, xsink=sx, out=s2l[1])
        return self.cv7(Fn.ConcatFn.apply(None, 0.0, None, y1, y2))


class SCConv(nn.Module):
    """Self-calibrated convolution, models/common.py:1279-1316: k4(k3(x) * sigmoid(x + up(k2(x))))."""

    def __init__(self, c1, c2, stride, groups=1, dilation=1, pooling_r=4):
        super().__init__()
        self.k2 = nn.Sequential(nn.AvgPool2d(kernel_size=pooling_r, stride=pooling_r),
                                nn.Conv2d(c1, c1, 3, 1, autopad(3, None), dilation=dilation, groups=groups,
                                          bias=False),
                                nn.BatchNorm2d(c1))
        self.k3 = nn.Sequential(nn.Conv2d(c1, c1, 3, 1, autopad(3, None), dilation=dilation, groups=groups,
                                          bias=False),
                                nn.BatchNorm2d(c1))
        self.k4 = nn.Sequential(nn.Conv2d(c1, c2, 3, stride, autopad(3, None), dilation=dilation, groups=groups,
                                          bias=False),
                                nn.BatchNorm2d(c2))

    def forward(self, x, xsink=None):
        """xsink: the caller's GradSink for x (Model fan-out); this module's three contributions join it"""
        r = self.k2[0].kernel_size
        r = r if isinstance(r, int) else r[0]
        sk = Fn.GradSink(3) if xsink is None else xsink.expect(3)  # x -> avg-pool (k2), k3, the gate
        g = conv_forward(self.k2[1], self.k2[2], None, Fn.AvgPoolFn.apply(x, r, sk))
        u3 = conv_forward(self.k3[0], self.k3[1], None, x, xsink=sk, defer=True)  # BN applied by the gate
        return conv_forward(self.k4[0], self.k4[1], None, Fn.SCGateFn.apply(x, u3, g, sk))


class CoorAttention(nn.Module):
    """Coordinate attention, models/common.py:1158-1207 (YAML token `CA`)."""

    def __init__(self, c1, c2, reduction=32):
        super().__init__()
        self.pool_h = nn.AdaptiveAvgPool2d((None, 1))
        self.pool_w = nn.AdaptiveAvgPool2d((1, None))
        c_ = max(8, c1 // reduction)
        self.conv1 = nn.Conv2d(c1, c_, kernel_size=1, stride=1, padding=0)
        self.bn1 = nn.BatchNorm2d(c_)
        self.act = nn.Hardswish()
        self.conv_w = nn.Conv2d(c_, c2, kernel_size=1, stride=1, padding=0)
        self.conv_h = nn.Conv2d(c_, c2, kernel_size=1, stride=1, padding=0)

    def forward(self, x):
        y = conv_forward(self.conv1, self.bn1, self.act, Fn.CAPoolFn.apply(x))   # [N, c_, H+W, 1]
        lh = conv_forward(self.conv_h, None, None, y)                           # logits over all H+W rows
        lw = conv_forward(self.conv_w, None, None, y)
        return Fn.CAApplyFn.apply(x, lh, lw)


CA = CoorAttention  # the north-star YAML's undefined `CA` token binds to CoorAttention


class CABottleneck(nn.Module):
    """models/common.py:1209-1227."""

    def __init__(self, c1, c2, shortcut=True, g=1, e=0.5, reduction=32):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_, c2, 3, 1, g=g)
        self.ca = CoorAttention(c2, c2, reduction)
        self.add = shortcut and c1 == c2

    def forward(self, x):
        if not self.add:
            return self.ca(self.cv2(self.cv1(x)))
        sk = Fn.GradSink(2)  # x -> cv1 and the residual
        return Fn.AddFn.apply(x, self.ca(self.cv2(self.cv1(x, xsink=sk))), sk)


class C3CA(C3):
    """models/common.py:1229-1235."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = nn.Sequential(*(CABottleneck(c_, c_, shortcut, g, e=1.0) for _ in range(n)))


class Concat(nn.Module):
    """models/common.py:656-664 (channel concat only: the YAML always passes dimension 1)."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def forward(self, x):
        assert self.d == 1
        return Fn.ConcatFn.apply(None, 0.0, None, *x)


def _join(sinks):
    """register one contribution with each given sink; None when there are none"""
    if sinks is None or all(sk is None for sk in sinks):
        return None
    return tuple(sk.expect(1) if sk is not None else None for sk in sinks)


class AdConcat2(nn.Module):
    """BiFPN weighted concat, models/common.py:994-1008."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension
        self.w = nn.Parameter(torch.ones(2, dtype=torch.float32), requires_grad=True)
        self.epsilon = 0.0001

    def forward(self, x, sinks=None):
        """sinks: None or one GradSink-or-None per input (Model fan-out); each joins with one contribution"""
        assert self.d == 1 and len(x) == 2
        return Fn.ConcatFn.apply(self.w, self.epsilon, _join(sinks), *x)


class AdConcat3(AdConcat2):
    """models/common.py:1010-1026."""

    def __init__(self, dimension=1):
        super().__init__(dimension)
        self.w = nn.Parameter(torch.ones(3, dtype=torch.float32), requires_grad=True)

    def forward(self, x, sinks=None):
        assert self.d == 1 and len(x) == 3
        return Fn.ConcatFn.apply(self.w, self.epsilon, _join(sinks), *x)


class SPP(nn.Module):
    """models/common.py:212-227: parallel max-pools (k = 5/9/13, 3/7/11, 3/5/7 in the config-5 YAML)."""

    def __init__(self, c1, c2, k=(5, 9, 13)):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * (len(k) + 1), c2, 1, 1)
        self.m = nn.ModuleList([nn.MaxPool2d(kernel_size=x, stride=1, padding=x // 2) for x in k])

    def forward(self, x):
        c_, n = self.cv1.conv.out_channels, len(self.m)
        if _INPLACE_CAT >= 1:  # cv1 and every pool write straight into the concat buffer's slices: no copies
            cat = Fn.concat_buffer(x.shape[0], (n + 1) * c_, x.shape[2], x.shape[3], x)
            sl = [cat[:, i * c_:(i + 1) * c_] for i in range(n + 1)]
        else:
            sl = [None] * (n + 1)
        x = self.cv1(x, out=sl[0])
        sk = Fn.GradSink(n + 1)  # x -> every pool and the concat
        ys = [Fn.MaxPoolFn.apply(x, m.kernel_size, sk, sl[i + 1:i + 2]) for i, m in enumerate(self.m)]
        return self.cv2(Fn.ConcatFn.apply(None, 0.0, (sk,) + (None,) * len(ys), x, *ys))


class ChannelAttentionModule(nn.Module):
    """models/common.py:260-285: sigmoid(MLP(avgpool x) + MLP(maxpool x)); both branches go through the
    shared MLP in one [2N]-row pass (1x1 conv kernels), the halves are summed in the sigmoid kernel."""

    def __init__(self, c1, reduction=16):
        super().__init__()
        mid = c1 // reduction
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.shared_MLP = nn.Sequential(nn.Linear(c1, mid), nn.ReLU(), nn.Linear(mid, c1))
        self.sigmoid = nn.Sigmoid()

    def forward(self, x, sink=None):
        l1, l2 = self.shared_MLP[0], self.shared_MLP[2]
        mid, c1 = l1.weight.shape
        z = Fn.GPoolFn.apply(x, sink)
        h = Fn.conv_bn_act(z, l1.weight.view(mid, c1, 1, 1), l1.bias, None, 1, 0, ACT_RELU)
        z2 = Fn.conv_bn_act(h, l2.weight.view(c1, mid, 1, 1), l2.bias, None, 1, 0, ACT_NONE)
        return Fn.HalvesSigmoidFn.apply(z2)


class SpatialAttentionModule(nn.Module):
    """models/common.py:287-300."""

    def __init__(self):
        super().__init__()
        self.conv2d = nn.Conv2d(in_channels=2, out_channels=1, kernel_size=7, stride=1, padding=3)
        self.sigmoid = nn.Sigmoid()

    def forward(self, s2):
        return conv_forward(self.conv2d, None, self.sigmoid, s2)


class CBAM(nn.Module):
    """models/common.py:302-310: out = ca(x) * x;  out = sa(out) * out."""

    def __init__(self, c1, c2):
        super().__init__()
        self.channel_attention = ChannelAttentionModule(c1)
        self.spatial_attention = SpatialAttentionModule()

    def forward(self, x):
        sk = Fn.GradSink(2)  # x -> the pools and the channel scaling
        ca = self.channel_attention(x, sk)
        out1, s2 = Fn.CBAMInFn.apply(x, ca, sk)
        return Fn.PixScaleFn.apply(out1, self.spatial_attention(s2))


class space_to_depth(nn.Module):
    """models/common.py:1451-1458 (SPD: stride-free 2x downsampling into channels)."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def forward(self, x):
        return Fn.SpaceToDepthFn.apply(x)


class Upsample(nn.Upsample):
    """nn.Upsample(None, 2, 'nearest') as used by the YAML heads; nearest only.  out: a concat_buffer slice to write
    the result into (Model's concat plan)."""

    def forward(self, x, out=None):
        assert self.mode == 'nearest'
        H, W = x.shape[2:]
        if self.size is not None:
            OH, OW = (self.size, self.size) if isinstance(self.size, int) else self.size
        else:
            sf = self.scale_factor if isinstance(self.scale_factor, (tuple, list)) else (self.scale_factor,) * 2
            OH, OW = int(math.floor(H * sf[0])), int(math.floor(W * sf[1]))
        return Fn.ResizeFn.apply(x, OH, OW, [out] if out is not None else None)


# ------------------------------------------------------------------ Swin (C3STR) — layers in swin.py
from .swin import SwinTransformerBlock, SwinTransformerLayer, WindowAttention, Mlp, DropPath  # noqa: E402


class C3STR(C3):
    """models/common.py:191-196: C3 whose bottleneck stack is a 3-layer Swin block (heads = c_ // 32)."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = SwinTransformerBlock(c_, c_, c_ // 32, n)


# ------------------------------------------------------------------ C3TR (config 5: global MHSA over P5 tokens)

class TransformerLayer(nn.Module):
    """models/common.py:312-336: x + Dropout(MHA(q(LN1 x), k(LN1 x), v(LN1 x))); x + Dropout(fc2(Dropout(
    ReLU(fc1(LN2 x))))).  `ma` is the real nn.MultiheadAttention (state_dict keys ma.in_proj_weight /
    in_proj_bias / out_proj.*; train.py's optimizer grouping skips in_proj_*); its
    projections run on the implicit-GEMM kernels and the attention core on csrc/mha.hip.  Tokens are
    the pixels of the NHWC activation, so the reference's [HW, b, c] sequence-first transposes are free."""

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

    @staticmethod
    def _lin(x, w, b=None, act=ACT_NONE, **kw):
        return Fn.conv_bn_act(x, w.view(w.shape[0], w.shape[1], 1, 1), b, None, 1, 0, act, **kw)

    def forward(self, x):
        c = x.shape[1]
        ma = self.ma
        drop = self.training and self.dropout.p > 0
        p = self.dropout.p
        s1, su, s2 = Fn.GradSink(2), Fn.GradSink(3), Fn.GradSink(2)  # x -> ln1 + residual; u -> q/k/v; x2 -> ln2 + residual
        u = Fn.LayerNormFn.apply(x, self.ln1.weight, self.ln1.bias, self.ln1.eps, s1)
        W, bi = ma.in_proj_weight, ma.in_proj_bias
        q = self._lin(self._lin(u, self.q.weight, xsink=su), W[:c], bi[:c])
        k = self._lin(self._lin(u, self.k.weight, xsink=su), W[c:2 * c], bi[c:2 * c])
        v = self._lin(self._lin(u, self.v.weight, xsink=su), W[2 * c:], bi[2 * c:])
        o = Fn.MHAFn.apply(q, k, v, ma.num_heads)
        if drop:
            x = Fn.AddFn.apply(x, Fn.DropoutFn.apply(self._lin(o, ma.out_proj.weight, ma.out_proj.bias), p), s1)
        else:
            x = self._lin(o, ma.out_proj.weight, ma.out_proj.bias, res=x, rsink=s1)
        u2 = Fn.LayerNormFn.apply(x, self.ln2.weight, self.ln2.bias, self.ln2.eps, s2)
        h = self._lin(u2, self.fc1.weight, act=ACT_RELU)
        if drop:
            return Fn.AddFn.apply(x, Fn.DropoutFn.apply(self._lin(Fn.DropoutFn.apply(h, p), self.fc2.weight), p), s2)
        return self._lin(h, self.fc2.weight, res=x, rsink=s2)


class TransformerBlock(nn.Module):
    """models/common.py:338-355: (optional Conv) -> p + linear(p) (learned position term, residual fused
    into the GEMM epilogue) -> n TransformerLayers; tokens stay in the NHWC activation."""

    def __init__(self, c1, c2, num_heads, num_layers):
        super().__init__()
        self.conv = None
        if c1 != c2:
            self.conv = Conv(c1, c2)
        self.linear = nn.Linear(c2, c2)
        self.tr = nn.Sequential(*(TransformerLayer(c2, num_heads) for _ in range(num_layers)))
        self.c2 = c2

    def forward(self, x):
        if self.conv is not None:
            x = self.conv(x)
        sk = Fn.GradSink(2)  # p -> linear + residual
        w = self.linear.weight
        p = Fn.conv_bn_act(x, w.view(self.c2, self.c2, 1, 1), self.linear.bias, None, 1, 0, ACT_NONE, res=x,
                           xsink=sk, rsink=sk)
        return self.tr(p)


class C3TR(C3):
    """models/common.py:184-189: C3 whose bottleneck stack is TransformerBlock(c_, c_, 4 heads, n)."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = TransformerBlock(c_, c_, 4, n)
