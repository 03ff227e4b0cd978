"""Anchor-free TDetect head (models/detect_t.py:23-101) on the gfx950 kernels.

Training returns (x, box, cls) like the reference: x = per-level [B, 64 + nc, H, W] outputs (NHWC
storage), box [B, 64, A] / cls [B, nc, A] = channel slices of one anchor-major [B, A, 64 + nc]
buffer (permuted views, no copy).  Inference returns (y [B, 4 + nc, A] fp32, (x, box, cls)) with y =
DFL-decoded xywh in pixels and sigmoid scores (csrc/tal.hip).
"""
import ctypes
import math

import torch
import torch.nn as nn

from .. import functional as Fn
from ..functional import call, ptr, stream, dcode

REG_MAX = 16


class DFL(nn.Module):
    """models/detect_t.py:92-101: the fixed bin-value conv is kept for state_dict compatibility;
    the decode itself runs inside the TAL kernels."""

    def __init__(self, c1=REG_MAX):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        self.conv.weight.data[:] = torch.arange(c1, dtype=torch.float).view(1, c1, 1, 1)
        self.c1 = c1


def _seq(seq, x, xsink=None):
    """Sequential(Conv, Conv, nn.Conv2d) on the HIP path."""
    from .common import conv_forward
    x = seq[0](x, xsink=xsink)
    x = seq[1](x)
    return conv_forward(seq[2], None, None, x)


def level_arrays(hw, strides):
    nl = len(hw)
    H = (ctypes.c_int * nl)(*[int(h) for h, _ in hw])
    W = (ctypes.c_int * nl)(*[int(w) for _, w in hw])
    S = (ctypes.c_float * nl)(*[float(s) for s in strides])
    return nl, ctypes.cast(H, ctypes.c_void_p), ctypes.cast(W, ctypes.c_void_p), ctypes.cast(S, ctypes.c_void_p), (H, W, S)


class TDetect(nn.Module):
    """models/detect_t.py:23-59."""
    shape = None
    anchors = torch.empty(0)
    strides = torch.empty(0)
    dynamic = False
    export = False

    def __init__(self, nc=80, ch=(), inplace=True):
        super().__init__()
        from .common import Conv
        self.nc = nc
        self.reg_max = REG_MAX
        self.nl = len(ch)
        self.no = nc + self.reg_max * 4
        self.inplace = inplace
        self.stride = torch.zeros(self.nl)
        c2, c3 = max(ch[0] // 4, 16), max(ch[0], self.no - 4)
        self.cv2 = nn.ModuleList(
            nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 4 * self.reg_max, 1)) for x in ch)
        self.cv3 = nn.ModuleList(
            nn.Sequential(Conv(x, c3, 3), Conv(c3, c3, 3), nn.Conv2d(c3, self.nc, 1)) for x in ch)
        self.dfl = DFL(self.reg_max)

    def forward(self, x):
        for i in range(self.nl):
            sk = Fn.GradSink(2)  # x[i] -> cv2[i] and cv3[i]
            x[i] = Fn.ConcatFn.apply(None, 0.0, None, _seq(self.cv2[i], x[i], sk), _seq(self.cv3[i], x[i], sk))
        flat = Fn.FlattenLevelsFn.apply(*x)
        box = flat[..., :self.reg_max * 4].permute(0, 2, 1)
        cls = flat[..., self.reg_max * 4:].permute(0, 2, 1)
        if self.training:
            return x, box, cls
        y = self.decode(flat, [xi.shape[2:] for xi in x])
        return y if self.export else (y, (x, box, cls))

    @torch.no_grad()
    def decode(self, flat, hw):
        B, A, _ = flat.shape
        y = torch.empty((B, 4 + self.nc, A), dtype=torch.float32, device=flat.device)
        sl = getattr(self, 'stride_list', None) or [float(v) for v in self.stride.cpu()]
        nl, H, W, S, keep = level_arrays(hw, sl)
        call('dmy_tal_detect_out', dcode(flat), ptr(flat.contiguous()), B, self.nc, nl, H, W, S, ptr(y), stream())
        return y

    def bias_init(self):
        """models/detect_t.py:53-59."""
        for a, b, s in zip(self.cv2, self.cv3, self.stride):
            a[-1].bias.data[:] = 1.0
            b[-1].bias.data[:self.nc] = math.log(5 / self.nc / (640 / s) ** 2)
