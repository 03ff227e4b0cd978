"""Drop-in Model / parse_model / Detect (models/yolo.py:40-478) on the gfx950 kernels.

Differences from the reference that do not change results:
  * strides come from a shape-only walk of the parsed graph instead of a probe forward
    (models/yolo.py:159-170); the probe's side effect on BN running stats is not reproduced
    (parity is anchored on state_dict transfer);
  * activations are NHWC in `Model.act_dtype` (float32 parity / bfloat16 throughput).
"""
import ctypes
import math
import os
import weakref
from copy import deepcopy
from pathlib import Path
from typing import List

import torch
import torch.nn as nn

from .. import functional as Fn
from ..functional import call, ptr, stream, dcode
from .common import *  # noqa: F401,F403  (the YAML namespace)
from .common import Conv, Upsample, SCConv, autopad, space_to_depth
from .tdetect import TDetect
from ..utils.general import make_divisible
from ..utils.torch_utils import initialize_weights, fuse_conv_and_bn

_CAT_PLAN = os.environ.get('DMY_CAT_PLAN', '1') == '1'  # see Model._make_cat_plan
_MODEL_SINKS = os.environ.get('DMY_MODEL_SINKS', '1') != '0'  # Model-level gradient fan-out sinks


class Detect(nn.Module):
    """models/yolo.py:40-114."""
    stride = None
    onnx_dynamic = False

    def __init__(self, nc=80, anchors=(), ch=(), inplace=True):
        super().__init__()
        self.nc = nc
        self.no = nc + 5
        self.nl = len(anchors)
        self.na = len(anchors[0]) // 2
        self.grid = [torch.zeros(1)] * self.nl
        self.anchor_grid = [torch.zeros(1)] * self.nl
        self.register_buffer('anchors', torch.tensor(anchors).float().view(self.nl, -1, 2))
        self.m = nn.ModuleList(nn.Conv2d(x, self.no * self.na, 1) for x in ch)
        self.inplace = inplace

    def forward(self, x, sinks=None):
        """sinks: None or one GradSink-or-None per level input (Model fan-out), one contribution each"""
        out = []
        for i in range(self.nl):
            sk = sinks[i].expect(1) if sinks is not None and sinks[i] is not None else None
            y = Fn.conv_bn_act(x[i], self.m[i].weight, self.m[i].bias, None, 1, 0, Fn.ACT_NONE, xsink=sk)
            bs, _, ny, nx = y.shape
            # NHWC [bs, ny, nx, na*no] -> [bs, na, ny, nx, no] view (no copy)
            out.append(y.permute(0, 2, 3, 1).view(bs, ny, nx, self.na, self.no).permute(0, 3, 1, 2, 4))
        if self.training:
            return out
        return self.decode(out), out

    @torch.no_grad()
    def decode(self, out):
        bs = out[0].shape[0]
        total = sum(self.na * p.shape[2] * p.shape[3] for p in out)
        z = torch.empty((bs, total, self.no), dtype=torch.float32, device=out[0].device)
        off = 0
        anchors = self.anchors.float().contiguous()
        sl = getattr(self, 'stride_list', None)
        if not sl or len(sl) != len(out):  # host copy of the strides: no device sync per forward (graph-capturable)
            sl = self.stride_list = [float(v) for v in self.stride.cpu()]
        if len(out) <= 4 and len({p.dtype for p in out}) == 1:  # every level in one launch
            nl, (_, na, _, _, no) = len(out), out[0].shape
            ys = (ctypes.c_void_p * nl)(*[p.data_ptr() for p in out])
            st = (ctypes.c_long * (3 * nl))(*[v for p in out for v in (p.stride(0), p.stride(2), p.stride(3))])
            hw = (ctypes.c_int * (2 * nl))(*[v for p in out for v in (p.shape[2], p.shape[3])])
            ls = (ctypes.c_float * nl)(*sl)
            call('dmy_detect_decode_levels', dcode(out[0]), nl, ys, st, hw, ls, bs, na, no, ptr(anchors), ptr(z), total,
                 stream())
            return z
        for i, p in enumerate(out):
            _, na, ny, nx, no = p.shape
            s = p.stride()
            call('dmy_detect_decode', dcode(p), ptr(p), s[0], s[2], s[3], bs, ny, nx, na, no, sl[i],
                 ptr(anchors[i]), ptr(z), off, total, stream())
            off += na * ny * nx
        return z

    def _make_grid(self, nx=20, ny=20, i=0):
        d = self.anchors[i].device
        yv, xv = torch.meshgrid([torch.arange(ny, device=d), torch.arange(nx, device=d)], indexing='ij')
        grid = torch.stack((xv, yv), 2).expand((1, self.na, ny, nx, 2)).float()
        anchor_grid = (self.anchors[i].clone() * self.stride[i]).view((1, self.na, 1, 1, 2)).expand(
            (1, self.na, ny, nx, 2)).float()
        return grid, anchor_grid


def check_anchor_order(m):
    """utils/autoanchor.py:16-23."""
    a = m.anchors.prod(-1).view(-1)
    da = a[-1] - a[0]
    ds = m.stride[-1] - m.stride[0]
    if da.sign() != ds.sign():
        m.anchors[:] = m.anchors.flip(0)


def _out_hw(m, hw):
    """Shape-only walk used for the stride probe (models/yolo.py:159-170)."""
    if isinstance(m, nn.Sequential) and not isinstance(m[0], nn.AvgPool2d):
        for mm in m:
            hw = _out_hw(mm, hw)
        return hw
    if isinstance(m, Conv):
        c = m.conv
        k, s, p = c.kernel_size[0], c.stride[0], c.padding[0]
        return ((hw[0] + 2 * p - k) // s + 1, (hw[1] + 2 * p - k) // s + 1)
    if isinstance(m, SCConv):
        s = m.k4[0].stride[0]
        return ((hw[0] - 1) // s + 1, (hw[1] - 1) // s + 1)
    if isinstance(m, nn.Upsample):
        sf = m.scale_factor if isinstance(m.scale_factor, (int, float)) else m.scale_factor[0]
        return (int(hw[0] * sf), int(hw[1] * sf))
    if isinstance(m, space_to_depth):
        return (hw[0] // 2, hw[1] // 2)
    return hw


class Model(nn.Module):
    """models/yolo.py:117-350."""

    def __init__(self, cfg='yolov5s.yaml', ch=3, nc=None, anchors=None, act_dtype=torch.float32):
        super().__init__()
        if isinstance(cfg, dict):
            self.yaml = deepcopy(cfg)
        else:
            import yaml
            self.yaml_file = Path(cfg).name
            with open(cfg, errors='ignore') as f:
                self.yaml = yaml.safe_load(f)
        ch = self.yaml['ch'] = self.yaml.get('ch', ch)
        if nc and nc != self.yaml['nc']:
            self.yaml['nc'] = nc
        if anchors:
            self.yaml['anchors'] = round(anchors)
        self.model, self.save = parse_model(deepcopy(self.yaml), ch=[ch])
        self.names = [str(i) for i in range(self.yaml['nc'])]
        self.inplace = self.yaml.get('inplace', True)
        self.act_dtype = act_dtype
        m = self.model[-1]
        if isinstance(m, Detect):
            s = 256
            m.inplace = self.inplace
            hw = self._probe_hw(s)
            m.stride = torch.tensor([s / h for h, _ in hw], dtype=torch.float32)
            m.anchors /= m.stride.view(-1, 1, 1)
            check_anchor_order(m)
            self.stride = m.stride
            self._initialize_biases()
        elif isinstance(m, TDetect):  # models/yolo.py:173-180
            s = 256
            m.inplace = self.inplace
            hw = self._probe_hw(s)
            m.stride = torch.tensor([s / h for h, _ in hw], dtype=torch.float32)
            self.stride = m.stride
            m.bias_init()
        initialize_weights(self)

    def _probe_hw(self, s):
        ys, hw = [], (s, s)
        for m in self.model:
            if m.f != -1:
                hw = ys[m.f] if isinstance(m.f, int) else [hw if j == -1 else ys[j] for j in m.f]
            if isinstance(m, (Detect, TDetect)):
                return hw
            if isinstance(hw, list):
                hw = hw[0]
            hw = _out_hw(m, hw)
            ys.append(hw)
        raise AssertionError('no Detect layer')

    def forward(self, x, augment=False, profile=False, visualize=False):
        if augment:
            raise NotImplementedError('test-time augmentation is outside the DMA-YOLO hot path')
        if torch.jit.is_tracing():
            return _traced_forward(self, x)
        return self._forward_once(x)

    def _s2d_stem(self, x):
        """layer 0 is the k6 s2 p2 stem Conv (every yolov5* / DMA-YOLO yaml) and the image allows the
        space-to-depth form (even H, W; no input gradient)"""
        m0 = self.model[0]
        if type(m0) is not Conv or x.dim() != 4 or x.requires_grad or x.shape[2] % 2 or x.shape[3] % 2:
            return False
        c = m0.conv
        return (c.kernel_size == (6, 6) and c.stride == (2, 2) and c.padding == (2, 2) and c.in_channels == x.shape[1]
                and c.groups == 1 and getattr(self, 's2d_stem', True))

    def to_input(self, x):
        """uint8/float NCHW image batch -> NHWC act_dtype (train.py:402 `/255` for uint8).  With the k6 s2 p2
        stem the image is stored space-to-depth (Fn.image_s2d) and the stem runs as a k3 s1 p1 conv."""
        if x.dtype == self.act_dtype and x.dim() == 4 and (x.shape[1] == 1 or x.stride(1) == 1):
            return x
        if x.is_cuda and self._s2d_stem(x):
            return Fn.image_s2d(x, self.act_dtype)
        y = Fn.ToNHWC.apply(x, self.act_dtype)
        y._dmy_cpad = -(-x.shape[1] // Fn.VW[self.act_dtype]) * Fn.VW[self.act_dtype]  # zero-padded channels
        return y

    def _weight_prep(self, dev):
        """functional.WeightPrep over every groups-1 Conv2d except a 3-channel stem (space-to-depth /
        channel-padded, prepped by its own layout kernel); rebuilt when the parameters move or fuse() ran"""
        first = next(self.parameters())
        key = (first.data_ptr(), dev, self.act_dtype)
        c = getattr(self, '_prep', None)
        if c is None or c[0] != key:
            ws = [m.weight for m in self.modules() if isinstance(m, nn.Conv2d) and m.groups == 1 and
                  m.in_channels > 4 and m.dilation in (1, (1, 1)) and m.weight.requires_grad]
            c = self._prep = (key, Fn.WeightPrep(ws, self.act_dtype, dev))
        return c[1]

    def _wgrad_arena(self):
        """Fresh zeroed weight-gradient arena for this training forward (functional.WgradArena)."""
        lay = getattr(self, '_arena_layout', None)
        first = next(self.parameters())
        if lay is None or lay[0] != (first.data_ptr(), first.device):
            offs, n = Fn.WgradArena.layout(self.parameters())
            lay = self._arena_layout = ((first.data_ptr(), first.device), offs, n)
        return Fn.WgradArena(torch.zeros(lay[2], dtype=torch.float32, device=first.device), lay[1])

    def _forward_once(self, x, profile=False, visualize=False):
        x = self.to_input(x)
        if self._cat_plans is None:
            self._cat_plans = {}
        y = []
        arena = self.training and torch.is_grad_enabled() and x.is_cuda
        prev = Fn.WgradArena.current, Fn.WeightPrep.current
        if arena:
            Fn.WgradArena.current = self._wgrad_arena()
            self._last_arena = weakref.ref(Fn.WgradArena.current)  # ddp.ArenaDDP all-reduces slices of it
            Fn.WeightPrep.current = self._weight_prep(x.device).launch()
        fan = self._fanout() if _MODEL_SINKS and torch.is_grad_enabled() and self.training else {}
        sinks = {}
        skey = tuple(x.shape) + (x.dtype,)
        plan = self._cat_plans.get(skey) if _CAT_PLAN else None
        shapes = [] if _CAT_PLAN and plan is None else None
        bufs = {}
        try:
            for m in self.model:
                if m.f != -1:
                    x = y[m.f] if isinstance(m.f, int) else [x if j == -1 else y[j] for j in m.f]
                kw = self._sink_kw(m, sinks) if sinks else None
                if plan is not None and m.i in plan:  # write straight into a later plain Concat's channel slice
                    c, c0, C, shp = plan[m.i]
                    if c not in bufs:
                        bufs[c] = Fn.concat_buffer(*shp, x if torch.is_tensor(x) else x[0])
                    kw = dict(kw or {}, out=bufs[c][:, c0:c0 + C])
                x = m(x, **kw) if kw else m(x)
                y.append(x if m.i in self.save else None)
                if shapes is not None:
                    shapes.append(tuple(x.shape) if torch.is_tensor(x) else None)
                if m.i in fan:
                    sinks[m.i] = Fn.GradSink(0)
        finally:
            Fn.WgradArena.current, Fn.WeightPrep.current = prev
        if shapes is not None:
            self._cat_plans[skey] = self._make_cat_plan(shapes)
        return x

    # In-place plain Concat across layers (DMY_CAT_PLAN=0 turns it off): after a first forward at an input shape has
    # recorded every layer's output shape, each later forward at that shape allocates every plain Concat's buffer
    # ahead and hands its producers (Conv, C3, Upsample: the modules whose forward takes out=) their channel slice,
    # so ConcatFn recognises the in-place slices and copies nothing (yolov5s's head: 8 slice copies per forward).
    # The producers' other consumers read the slice through its pixel stride.  Only concats whose every input comes
    # from such a producer, each feeding no other concat.
    _cat_plans = None

    def _make_cat_plan(self, shapes):
        import inspect
        takes_out = lambda m: 'out' in inspect.signature(m.forward).parameters  # noqa: E731
        users = {}
        for m in self.model:
            if type(m).__name__ == 'Concat':
                for j in ([m.f] if isinstance(m.f, int) else m.f):
                    users.setdefault(m.i - 1 if j == -1 else j, []).append(m.i)
        plan = {}
        for m in self.model:
            if type(m).__name__ != 'Concat' or isinstance(m.f, int):
                continue
            src = [m.i - 1 if j == -1 else j for j in m.f]
            shp = [shapes[j] for j in src]
            if any(sh is None or len(sh) != 4 for sh in shp) or len(set(src)) != len(src):
                continue
            if any(len(users.get(j, [])) != 1 or not takes_out(self.model[j]) for j in src):
                continue
            if len({(sh[0], sh[2], sh[3]) for sh in shp}) != 1:
                continue
            Ct, c0 = sum(sh[1] for sh in shp), 0
            N, _, H, W = shp[0]
            for j, sh in zip(src, shp):
                plan[j] = (m.i, c0, sh[1], (N, Ct, H, W))
                c0 += sh[1]
        return plan

    # gradient fan-out: a layer output read by several layers (the BiFPN skips, the P3-P5 outputs read by a Conv and
    # Detect) gets one GradSink that the sink-aware consumers' backward kernels write / accumulate into, so autograd
    # does not sum their contributions with separate ATen add kernels (DMY_MODEL_SINKS=0 turns it off).  On by default
    # since round 6 (no ATen arithmetic on the hot path); same-box A/Bs (profiles/r02/ab_model_sinks.log,
    # profiles/r04/model_sinks_ab.log) put it within the +-0.5 % run-to-run noise -- DMA-1536 +0.35 % with Detect
    # included, -0.3 %..+0.05 % without; yolov5s -0.3 % with Detect (its only multi-consumer outputs are read by a Conv
    # and Detect, whose narrow-K data-grad then accumulates), so Detect joins only under DMY_SINK_DETECT=1.
    _SINK_TYPES = ('Conv', 'SCConv', 'AdConcat2', 'AdConcat3') + (('Detect',) if os.environ.get('DMY_SINK_DETECT') == '1'
                                                                  else ())

    def _fanout(self):
        """{layer index: consumer count} for outputs read by >= 2 layers, >= 1 of them sink-aware (cached)"""
        if getattr(self, '_fan', None) is None:
            cons = {}
            for m in self.model:
                for j in ([m.f] if isinstance(m.f, int) else m.f):
                    cons.setdefault(m.i - 1 if j == -1 else j, []).append(type(m).__name__)
            self._fan = {i: len(c) for i, c in cons.items() if len(c) >= 2 and any(t in self._SINK_TYPES for t in c)}
        return self._fan

    def _sink_kw(self, m, sinks):
        """keyword arguments handing layer m its inputs' fan-out sinks, or None"""
        name = type(m).__name__
        if name not in self._SINK_TYPES:
            return None
        src = [m.i - 1 if j == -1 else j for j in ([m.f] if isinstance(m.f, int) else m.f)]
        sk = [sinks.get(j) for j in src]
        if all(s is None for s in sk):
            return None
        if name == 'Conv':
            return {'xsink': sk[0].expect(1)}
        if name == 'SCConv':
            return {'xsink': sk[0]}
        return {'sinks': sk}

    def _initialize_biases(self, cf=None):
        """models/yolo.py:293-301."""
        m = self.model[-1]
        for mi, s in zip(m.m, m.stride):
            b = mi.bias.view(m.na, -1)
            b.data[:, 4] += math.log(8 / (640 / s) ** 2)
            b.data[:, 5:] += math.log(0.6 / (m.nc - 0.999999)) if cf is None else torch.log(cf / cf.sum())
            mi.bias = torch.nn.Parameter(b.view(-1), requires_grad=True)

    def fuse(self):
        """models/yolo.py:315-323: BN folded into YAML-level Conv layers only."""
        for m in self.model:
            if isinstance(m, Conv) and hasattr(m, 'bn'):
                m.conv = fuse_conv_and_bn(m.conv, m.bn)
                delattr(m, 'bn')
                m.forward = m.forward_fuse
        self._prep = None
        return self

    def _apply(self, fn):
        self = super()._apply(fn)
        m = self.model[-1]
        if isinstance(m, Detect):
            m.stride_list = [float(v) for v in m.stride.cpu()] if m.stride.numel() else []
            m.stride = fn(m.stride)
            m.grid = list(map(fn, m.grid))
            if isinstance(m.anchor_grid, list):
                m.anchor_grid = list(map(fn, m.anchor_grid))
        elif isinstance(m, TDetect):  # models/yolo.py:345-348; the stride list for the kernels stays on the host
            m.stride_list = [float(v) for v in m.stride.cpu()] if m.stride.numel() else []
            m.stride = fn(m.stride)
            m.anchors = fn(m.anchors)
            m.strides = fn(m.strides)
        return self

    def info(self, verbose=False, img_size=640):
        n_p = sum(x.numel() for x in self.parameters())
        return n_p


_CH_MODS = None


def _namespace():
    import types
    from . import common as C
    ns = {k: getattr(C, k) for k in C.__all__}
    ns['Detect'] = Detect
    ns['TDetect'] = TDetect
    ns['nn'] = types.SimpleNamespace(Upsample=Upsample, BatchNorm2d=nn.BatchNorm2d)
    return ns


def parse_model(d, ch):
    """models/yolo.py:353-478 for the hot-path module set (eval of YAML names in this namespace)."""
    from . import common as C
    ns = _namespace()
    anchors, nc, gd, gw = d['anchors'], d['nc'], d['depth_multiple'], d['width_multiple']
    na = (len(anchors[0]) // 2) if isinstance(anchors, list) else anchors
    no = na * (nc + 5)
    ev = dict(ns, nc=nc, anchors=anchors)
    chan_mods = (C.Conv, C.Bottleneck, C.SPPF, C.C3, C.C3TR, C.C3STR, C.CoorAttention, C.CABottleneck, C.C3CA,
                 C.SPPFCSPC, C.SCConv, C.SPP, C.CBAM)
    rep_mods = (C.C3, C.C3TR, C.C3STR, C.C3CA)
    layers, save, c2 = [], [], ch[-1]
    for i, (f, n, m, args) in enumerate(d['backbone'] + d['head']):
        m = eval(m, ev) if isinstance(m, str) else m
        for j, a in enumerate(args):
            try:
                args[j] = eval(a, ev) if isinstance(a, str) else a
            except NameError:
                pass
        n = n_ = max(round(n * gd), 1) if n > 1 else n
        if m in chan_mods:
            c1, c2 = ch[f], args[0]
            if c2 != no:
                c2 = make_divisible(c2 * gw, 8)
            args = [c1, c2, *args[1:]]
            if m in rep_mods:
                args.insert(2, n)
                n = 1
        elif m is nn.BatchNorm2d:
            args = [ch[f]]
        elif m in (C.Concat, C.AdConcat2, C.AdConcat3):
            c2 = sum(ch[x] for x in f)
        elif m is Detect:
            args.append([ch[x] for x in f])
            if isinstance(args[1], int):
                args[1] = [list(range(args[1] * 2))] * len(f)
        elif m is TDetect:
            args.append([ch[x] for x in f])
        elif m is space_to_depth:
            c2 = 4 * ch[f]
        elif m is Upsample:
            c2 = ch[f]
        else:
            raise NotImplementedError(f'YAML module {m} is outside the DMA-YOLO hot path')
        m_ = nn.Sequential(*(m(*args) for _ in range(n))) if n > 1 else m(*args)
        t = str(m)[8:-2].replace('__main__.', '')
        np_ = sum(x.numel() for x in m_.parameters())
        m_.i, m_.f, m_.type, m_.np = i, f, t, np_
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(m_)
        if i == 0:
            ch = []
        ch.append(c2)
    return nn.Sequential(*layers), sorted(save)


# ------------------------------------------------------------------ torch.jit.trace support
# The reference logs the model graph at the first batch (utils/loggers/__init__.py:86:
# tb.add_graph(torch.jit.trace(de_parallel(model), imgs[0:1], strict=False))).  The per-layer HIP launches go
# through ctypes, which the tracer cannot see, so under tracing the whole forward is ONE registered dispatcher op,
# dmayolo::model_forward (torch.library): the trace records that node (and can replay it), the op runs the
# ordinary HIP forward below the tracer.  Outputs are copies (a custom op may not return views of its
# intermediates); train mode returns the Detect maps, eval mode (decoded boxes, maps).
_TRACE_MODELS = weakref.WeakValueDictionary()


@torch.library.custom_op('dmayolo::model_forward', mutates_args=())
def _model_forward_op(x: torch.Tensor, key: int) -> List[torch.Tensor]:
    m = _TRACE_MODELS[key]
    with torch.no_grad():
        y = m._forward_once(x)
    if isinstance(y, tuple):
        return [y[0].clone()] + [o.clone() for o in y[1]]
    return [o.clone() for o in y]


def _traced_forward(model, x):
    _TRACE_MODELS[id(model)] = model
    res = torch.ops.dmayolo.model_forward(x, id(model))
    return list(res) if model.training else (res[0], list(res[1:]))
