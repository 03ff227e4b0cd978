"""Autograd Functions over the gfx950 C-ABI (dmayolo._lib).  Activations are NHWC
(torch channels_last, logical NCHW shape) in the storage dtype (float32 parity / bfloat16
throughput); master weights, BN statistics and reductions are fp32.

Every forward/backward here launches hand-written HIP kernels; no ATen compute op sits on the
hot path (torch is used for allocation and the current stream only).
"""
import os
import weakref

import torch

from . import _lib
from ._lib import call, ptr, stream, ACT_NONE, ACT_SILU, ACT_HARDSWISH, ACT_SIGMOID, ACT_GELU, ACT_RELU  # noqa: F401

DT = {torch.float32: 0, torch.bfloat16: 1}
CL = torch.channels_last


def dcode(t):
    try:
        return DT[t.dtype]
    except KeyError:
        raise TypeError(f'dmayolo kernels take float32 or bfloat16 activations, got {t.dtype}')


def pixel_stride(t):
    """Return (t', ps) with t' NHWC-addressable: addr(b,c,h,w) = b*H*W*ps + (h*W+w)*ps + c."""
    N, C, H, W = t.shape
    for attempt in range(2):
        s = t.stride()
        if C == 1 or s[1] == 1:
            ps = s[3] if W > 1 else (s[2] if H > 1 else (s[0] if N > 1 else C))
            if (W == 1 or s[3] == ps) and (H == 1 or s[2] == W * ps) and (N == 1 or s[0] == H * W * ps) and ps >= C:
                return t, ps
        t = t.contiguous(memory_format=CL)
    raise AssertionError('layout')


def new_act(N, C, H, W, like):
    return torch.empty((N, C, H, W), dtype=like.dtype, device=like.device, memory_format=CL)


def f32(n, dev):
    return torch.empty(n, dtype=torch.float32, device=dev)


_CONST = {}


def const_vec(n, value, dev):
    """a cached fp32 vector of n copies of value on dev, for kernel arguments that are only read (the unit scale /
    zero shift of the activation-only passes): one fill per (n, value, device) instead of two per layer and step"""
    key = (int(n), float(value), str(dev))
    t = _CONST.get(key)
    if t is None:
        t = torch.full((int(n),), float(value), dtype=torch.float32, device=dev)
        # a fill recorded into a HIP graph only runs at replay: cache only what an eager fill has written
        if not torch.cuda.is_current_stream_capturing():
            _CONST[key] = t
    return t


# Output-into-slice side channel of conv_bn_act (see concat_buffer): the view is consumed by the ConvBNActFn.apply
# that conv_bn_act issues right after setting it, and only when its shape / dtype / device match the output.
_OUT = [None]


def _take_out(N, K, OH, OW, like):
    o, _OUT[0] = _OUT[0], None
    if o is None or tuple(o.shape) != (N, K, OH, OW) or o.dtype != like.dtype or o.device != like.device:
        return None
    if pixel_stride(o)[0] is not o:  # not NHWC-addressable in place (pixel_stride would copy): a fresh output instead
        return None
    return o


def concat_buffer(N, Ct, H, W, like):
    """the channels_last buffer of a plain Concat whose producers write their outputs straight into its channel
    slices (conv_bn_act(out=buf[:, c0:c1])); ConcatFn then recognises the in-place slices and copies nothing"""
    return new_act(N, Ct, H, W, like)


class GradSink:
    """Input-gradient accumulator for an activation with several consumers inside one module.

    Autograd would sum the consumers' gradient contributions with separate add kernels.  Here
    the consumers' backward kernels write (first contribution in backward order) or accumulate
    (the rest, through the kernels' accumulate flags) into one NHWC buffer, and only the LAST of
    the `n` contributions hands the finished buffer to autograd (the others return None).  The
    activation's producer runs only after all of its consumers' backwards, and any contribution
    from outside the module is added by autograd to the finished buffer.  The sink resets after
    the n-th contribution, so a retained graph can run backward again.
    """
    __slots__ = ('n', 'seen', 'buf', 'ps')

    def __init__(self, n):
        self.n, self.seen, self.buf, self.ps = n, 0, None, 0

    def expect(self, k):
        """register k more contributions (a consumer module taking this sink from its caller, in forward)"""
        self.n += k
        return self

    def _tick(self):
        self.seen += 1
        if self.seen < self.n:
            return None
        ret = self.buf
        self.buf, self.seen = None, 0
        return ret

    def target(self, N, C, H, W, like):
        """-> (buffer, pixel stride, accumulate flag, tensor to hand to autograd or None); call
        `done()` after the kernel has been launched"""
        if self.buf is None:
            self.buf, self.ps = new_act(N, C, H, W, like), C
            return self.buf, C, 0
        return self.buf, self.ps, 1

    def peek(self, N, C, H, W):
        """(buffer, pixel stride) a target() call would return now without allocating, or None when it would
        allocate a fresh dense buffer"""
        return (self.buf, self.ps) if self.buf is not None else None

    def done(self):
        return self._tick()

    def passthrough(self, g):
        """identity contribution (a residual / concat slice): adopt g as the buffer, or add it in.
        Adoption is safe for the residual pattern: every other reader of g lies inside the branch,
        whose backwards all finish before the branch's first consumer accumulates into g."""
        g, gps = pixel_stride(g)
        if self.buf is None:
            self.buf, self.ps = g, gps
        else:
            N, C, H, W = g.shape
            call('dmy_slice_copy', dcode(g), ptr(g), gps, ptr(self.buf), self.ps, N * H * W, C, None, 0, 0, 0.0, 1,
                 stream())
        return self._tick()


def sink_target(sink, N, C, H, W, like):
    """-> (buffer, pixel stride, accumulate flag) for an input gradient; see sink_result"""
    if sink is None:
        return new_act(N, C, H, W, like), C, 0
    return sink.target(N, C, H, W, like)


def sink_result(sink, buf):
    """what the backward returns for that input: its own buffer, or the sink's verdict"""
    return buf if sink is None else sink.done()


# ------------------------------------------------------------------ convolution (+BN +act)

WGRAD_OIHW, WGRAD_ZEROED = 1, 2  # dmy_conv_wgrad_ex flags
DETERMINISTIC = [False]  # set_deterministic(): split-K weight-grads through a workspace, reduced in split order


def set_deterministic(on=True):
    """Run-to-run bit-identical training steps on the conv / loss path: weight-gradient split-K partials go to a
    workspace reduced in split order (dmy_conv_wgrad_det) instead of fp32 atomics.  The loss kernels are always
    deterministic.  Costs one workspace write + read per split-K weight-grad launch."""
    DETERMINISTIC[0] = bool(on)


def _wgrad(dt, x, dz, dw, N, H, W, C, xps, K, k, s, p, OH, OW, dzps, flags, fl, **kw):
    """one weight-gradient launch (atomic split-K, or the deterministic workspace form)"""
    if DETERMINISTIC[0]:
        ne = call('dmy_conv_wgrad_ws_elems', dt, ptr(x), ptr(dz), N, H, W, C, xps, K, k, k, s, p, OH, OW, dzps, flags)
        ws = f32(ne, dz.device) if ne else None
        KernelTimer.run('conv_wgrad', fl, 'dmy_conv_wgrad_det', dt, ptr(x), ptr(dz), ptr(dw), N, H, W, C, xps, K, k, k,
                        s, p, OH, OW, dzps, flags, ptr(ws), ne, stream(), **kw)
    else:
        KernelTimer.run('conv_wgrad', fl, 'dmy_conv_wgrad_ex', dt, ptr(x), ptr(dz), ptr(dw), N, H, W, C, xps, K, k, k,
                        s, p, OH, OW, dzps, flags, stream(), **kw)


class WgradArena:
    """Per-training-forward fp32 buffer holding every conv / linear weight gradient of a Model in
    torch OIHW order.  Model.forward clears it with ONE fill; each weight-grad launch then
    accumulates straight into its slice (no per-launch memset, no layout pass), and the slice is
    handed to autograd as the parameter's gradient.  A new buffer per forward, so the previous
    step's .grad views are never overwritten (gradient accumulation stays correct); a weight used
    twice in one forward gets a fresh tensor the second time."""
    current = None
    ALIGN = 64  # elements (256 B): slices stay 16-B aligned for the vectorised optimizer kernels

    def __init__(self, buf, offsets):
        self.buf, self.offsets, self.taken = buf, offsets, set()

    @classmethod
    def layout(cls, params):
        """data_ptr -> (offset, numel) for every fp32 parameter that requires a gradient (conv / linear weights,
        BN gamma / beta, conv biases: every tensor the conv backward produces comes from here, so the
        optimizer's pointer tables see the same gradient addresses every step); total size"""
        offs, n = {}, 0
        for q in params:
            if q.dim() >= 1 and q.dtype == torch.float32 and q.requires_grad:
                offs[q.data_ptr()] = (n, q.numel())
                n += -(-q.numel() // cls.ALIGN) * cls.ALIGN
        return offs, n

    def take(self, key, shape):
        o = self.offsets.get(key)
        numel = 1
        for d in shape:
            numel *= d
        if o is None or o[1] != numel or key in self.taken:
            return None
        self.taken.add(key)
        return self.buf[o[0]:o[0] + numel].view(shape)


# Bumped whenever our kernels write parameters or BN buffers through raw pointers (fused optimizers, EMA,
# train-mode BN running statistics): torch's _version does not see those writes, so the inference caches
# (prepped weights, eval BN coefficients) key on this as well.
PARAM_GEN = [0]


class WeightPrep:
    """Training forward: the activation-dtype copies of every conv weight of a Model (OHWI forward operand,
    IHWO data-grad operand) written by ONE dmy_conv_wprep_multi launch per forward instead of one
    dmy_conv_wprep per layer.  Buffer, operand views and the 40-byte device descriptor table are built once
    per model (host work per step: one launch).  Reusing the buffer is safe: its content is a pure function
    of the current weights, which change only at optimizer.step, between a backward and the next forward."""
    current = None
    ALIGN = 64  # elements: every operand 16-B aligned (v3 loaders)

    def __init__(self, weights, dtype, dev):
        import numpy as np
        sizes = [-(-w.numel() // self.ALIGN) * self.ALIGN for w in weights]
        self.buf = torch.empty(2 * sum(sizes), dtype=dtype, device=dev)
        self.map, recs, off = {}, [], 0
        for w, n in zip(weights, sizes):
            K, C, KH, KW = w.shape
            wf = self.buf[off:off + w.numel()].view(K, KH * KW * C)
            wt = self.buf[off + n:off + n + w.numel()].view(C, KH * KW * K)
            self.map[w.data_ptr()] = (wf, wt)
            recs.append((w.data_ptr(), wf.data_ptr(), wt.data_ptr(), K, C, KH, KW))
            off += 2 * n
        rec = np.dtype([('w', '<u8'), ('wf', '<u8'), ('wt', '<u8'), ('K', '<i4'), ('C', '<i4'), ('KH', '<i4'),
                        ('KW', '<i4')])
        self.table = torch.from_numpy(np.array(recs, dtype=rec).view(np.uint8)).to(dev)
        self.n, self.dtype = len(recs), dtype

    def launch(self):
        call('dmy_conv_wprep_multi', DT[self.dtype], ptr(self.table), self.n, stream())
        return self

    def get(self, weight, dtype):
        return self.map.get(weight.data_ptr()) if dtype == self.dtype else None


class ConvSpec:
    """Static description of one conv(+BN)(+act) layer; `bn` is the live nn.BatchNorm2d (or None).
    wcache / ecache: inference-only caches of the prepped weight and the eval BN coefficients."""
    __slots__ = ('stride', 'pad', 'act', 'bn', 'wcache', 'ecache', 'fp8', 'f8cache', 'f8_emit', 'defer', '__weakref__')

    def __init__(self, stride, pad, act, bn=None):
        self.stride, self.pad, self.act, self.bn = int(stride), int(pad), int(act), bn
        self.wcache = self.ecache = self.f8cache = self.f8_emit = None
        self.fp8 = False
        self.defer = False  # deferred_affine(): the consumer applies this layer's BN (see SCGateFn)


_SPECS = weakref.WeakKeyDictionary()


def spec_for(owner, stride, pad, act, bn):
    """The persistent ConvSpec of a conv module (keyed weakly on the module, so deepcopies such as the EMA
    model get their own)."""
    sp = _SPECS.get(owner)
    if sp is None or (sp.stride, sp.pad, sp.act) != (int(stride), int(pad), int(act)) or sp.bn is not bn:
        sp = _SPECS[owner] = ConvSpec(stride, pad, act, bn)
    sp.fp8 = bool(getattr(owner, 'dmy_fp8', False))
    return sp


_PSPECS = {}  # id(weight parameter) -> (weakref, {(stride, pad, act, id(bn)): ConvSpec}); tensors cannot be
# WeakKeyDictionary keys (their == is elementwise)


def _param_spec(w, stride, pad, act, bn):
    k = id(w)
    ent = _PSPECS.get(k)
    if ent is None or ent[0]() is not w:
        ent = _PSPECS[k] = (weakref.ref(w, lambda _r, k=k: _PSPECS.pop(k, None)), {})
    key = (int(stride), int(pad), int(act), id(bn))
    sp = ent[1].get(key)
    if sp is None or sp.bn is not bn:
        sp = ent[1][key] = ConvSpec(stride, pad, act, bn)
    return sp


def fp8_eligible(C, K, dtype, rows):
    """layers the e4m3 forward kernel takes (dmy_conv_fwd_fp8): bf16 activations, C % 128 == 0 (one 128-wide
    K step per tap), K % 8 == 0, and byte offsets of the quantised input below the buffer-descriptor range"""
    return dtype == torch.bfloat16 and C % 128 == 0 and K % 8 == 0 and K >= 32 and rows * C < 0xFFFFFFF0


def set_fp8(model, on=True, min_k=3):
    """Config 5 (BASELINE configs[4]): run the forward of every eligible conv (input channels % 128 == 0, kernel
    >= min_k) on the fp8 e4m3 MFMA kernel; the backward stays bf16.  Default min_k = 3: a 1x1 layer is HBM /
    latency-bound, so its 2x MFMA rate does not pay for quantising its input (profiles/r02, c5 fp8 A/B).
    Returns the number of convs switched: those fp8_eligible's shape tests (C % 128, K % 8, K >= 32) admit; at run
    time the layer also needs bf16 activations and a quantised input under the descriptor range."""
    n = 0
    for m in model.modules():
        if isinstance(m, torch.nn.Conv2d) and m.groups == 1 and m.kernel_size[0] >= min_k \
                and fp8_eligible(m.in_channels, m.out_channels, torch.bfloat16, 0):
            m.dmy_fp8 = bool(on)
            n += 1
    PARAM_GEN[0] += 1  # drop cached inference weights / coefficients
    return n


_F8_WS = [0]


def _f8_ws():
    _F8_WS[0] = call('dmy_fp8_quant_ws_elems')
    return _F8_WS[0]


# delayed (previous-step) activation scaling for the fp8 convs: the producing layer emits the e4m3 copy of its
# output in its BN-act pass (dmy_bn_act_fwd_f8) instead of two quantisation passes over it (dmy_fp8_quant).
# DMY_F8_DELAYED=0 keeps the just-in-time quantisation with the current amax.
F8_DELAYED = [os.environ.get('DMY_F8_DELAYED', '1') == '1']


# headroom on the delayed amax (DMY_F8_HEADROOM, >= 1; 1 = none): a margin against an activation range that grows
# between steps, at the cost of log2(headroom) bits of e4m3 resolution
F8_HEADROOM = [float(os.environ.get('DMY_F8_HEADROOM', '1'))]


class F8Emit:
    """Per producer layer: two ping-pong arrays of block maxima (this step's |y| maxima become the next step's
    quantisation amax) and the last call's per-block saturation counts.  The first step only records maxima (its
    consumer quantises just in time)."""
    __slots__ = ('buf', 'p', 'valid', 'numel')

    def __init__(self, dev):
        nb = call('dmy_bn_act_f8_blocks')
        self.buf = torch.zeros(3, nb, dtype=torch.float32, device=dev)
        self.p, self.valid, self.numel = 0, False, 0

    def run(self, z, scale, shift, act, res, rps, y, yps, M, K):
        """BN-act of the producer with the e4m3 side output; returns (y8, used amax) or None on the first step"""
        y8 = torch.empty(M * K, dtype=torch.uint8, device=z.device)
        used = f32(1, z.device)
        call('dmy_bn_act_fwd_f8', ptr(z), K, ptr(scale), ptr(shift), act, ptr(res), rps, ptr(y), yps, M, K, ptr(y8),
             ptr(self.buf[self.p]), ptr(self.buf[1 - self.p]), ptr(used), F8_HEADROOM[0], ptr(self.buf[2]), stream())
        self.p ^= 1
        out = (y8, used) if self.valid else None
        self.valid, self.numel = True, M * K
        return out

    def saturated(self):
        """(count, fraction) of the last call's e4m3 elements clipped at +-448 (a device sync)"""
        n = float(self.buf[2].sum()) if self.valid else 0.0
        return n, n / max(1, self.numel)


def f8_saturation(model):
    """{module name: (saturated count, fraction)} of every delayed-scaling producer's last step"""
    out = {}
    for name, mod in model.named_modules():
        if not isinstance(mod, torch.nn.Conv2d):
            continue
        sps = [_SPECS[mod]] if mod in _SPECS else []  # module-held specs (common.conv_forward)
        ent = _PSPECS.get(id(mod.weight))
        if ent is not None and ent[0]() is mod.weight:
            sps += list(ent[1].values())
        for sp in sps:
            if isinstance(sp.f8_emit, F8Emit):
                out[name] = sp.f8_emit.saturated()
    return out


def _fp8_weight(weight, spec, wkey, dev):
    K, C, KH, KW = weight.shape
    fc = spec.f8cache
    if fc is not None and fc[0] == wkey:
        return fc[1], fc[2]
    w8 = torch.empty(weight.numel(), dtype=torch.uint8, device=dev)
    ws = f32(K, dev)
    call('dmy_conv_wprep_fp8', ptr(weight.detach().contiguous()), ptr(w8), ptr(ws), K, C, KH, KW, stream())
    spec.f8cache = (wkey, w8, ws)
    return w8, ws


def _fp8_operands(x, xps, weight, spec, wkey, f8in=None):
    """per-tensor e4m3 copy of the activation and the per-output-channel e4m3 weight (cached on the spec until the
    weight changes).  f8in = (x8, amax) emitted by the producer (delayed scaling), else dmy_fp8_quant with the
    current amax"""
    N, C, H, W = x.shape
    K, _, KH, KW = weight.shape
    rows = N * H * W
    if f8in is not None:
        w8, ws = _fp8_weight(weight, spec, wkey, x.device)
        return f8in[0], f8in[1], w8, ws
    x8 = torch.empty(rows * C, dtype=torch.uint8, device=x.device)
    amax = f32(_F8_WS[0] or _f8_ws(), x.device)  # [0] = the amax the quantisation used
    call('dmy_fp8_quant', ptr(x), rows, C, xps, ptr(x8), ptr(amax), stream())
    fc = spec.f8cache
    if fc is not None and fc[0] == wkey:
        w8, ws = fc[1], fc[2]
    else:
        w8 = torch.empty(weight.numel(), dtype=torch.uint8, device=x.device)
        ws = f32(K, x.device)
        call('dmy_conv_wprep_fp8', ptr(weight.detach().contiguous()), ptr(w8), ptr(ws), K, C, KH, KW, stream())
        spec.f8cache = (wkey, w8, ws)
    return x8, amax, w8, ws


def prep_weight(w, dtype, need_t, Cp=None):
    K, C, KH, KW = w.shape
    Cp = Cp or C
    wc = w.detach().contiguous()
    wf = torch.empty((K, KH * KW * Cp), dtype=dtype, device=w.device)
    wt = torch.empty((C, KH * KW * K), dtype=dtype, device=w.device) if need_t else None
    call('dmy_conv_wprep', DT[dtype], ptr(wc), ptr(wf), ptr(wt), K, C, Cp, KH, KW, stream())
    return wf, wt


VW = {torch.float32: 4, torch.bfloat16: 8}


def zero_padded_channels(x):
    """Channel count the storage of `x` is zero-padded to (set by ToNHWC for the 3-channel stem)."""
    cp = getattr(x, '_dmy_cpad', 0)
    return cp if cp and cp % VW[x.dtype] == 0 else 0


def conv_out_hw(H, W, k, s, p):
    return (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1


class KernelTimer:
    """Live per-launch timing of the implicit-GEMM conv kernels with HIP events on the launch
    stream (bench.py roofline).  Off by default; zero overhead when disabled."""
    enabled = False
    records = []  # (kind, algorithmic_flops, algorithmic_bytes, start_event, end_event, shape tag)

    @classmethod
    def run(cls, kind, flops, name, *args, tag=None, nbytes=0.0):
        """nbytes: algorithmic HBM bytes of the launch (operands read once, result written once)"""
        if not cls.enabled:
            return call(name, *args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call(name, *args)
        e1.record()
        cls.records.append((kind, flops, nbytes, e0, e1, tag))

    @classmethod
    def summary(cls, detail=None, peak_flops=2.5e15, peak_bw=8.0e12, peak_flops_f8=5.0e15, table=None):
        """Per-kind totals: launches, flops, seconds, bytes, and the roofline time sum_launches max(F / peak_flops,
        B / peak_bw) split by the binding resource (troof_mfma / troof_hbm).  When `detail` is a dict it also
        receives per-(kind, shape) [launches, flops, seconds, bytes]; when `table` is a list it receives one
        (kind, shape tag, flops, bytes, seconds, roofline seconds) tuple per launch, in launch order."""
        torch.cuda.synchronize()
        out = {}
        for kind, fl, nb, e0, e1, tag in cls.records:
            t = e0.elapsed_time(e1) * 1e-3
            tm, th = fl / (peak_flops_f8 if kind.endswith('_f8') else peak_flops), nb / peak_bw
            if table is not None:
                table.append((kind, tag, fl, nb, t, max(tm, th)))
            d = out.setdefault(kind, [0, 0.0, 0.0, 0.0, 0.0, 0.0])
            d[0] += 1
            d[1] += fl
            d[2] += t
            d[3] += nb
            d[4 if tm >= th else 5] += max(tm, th)
            if detail is not None:
                d = detail.setdefault((kind, tag), [0, 0.0, 0.0, 0.0])
                d[0] += 1
                d[1] += fl
                d[2] += t
                d[3] += nb
        cls.records = []
        return {k: dict(launches=v[0], flops=v[1], seconds=v[2], bytes=v[3], troof_mfma=v[4], troof_hbm=v[5])
                for k, v in out.items()}


def _launch_conv_fwd(x, xps, wf, bias, y, yps, psum, psq, K, k, s, p, OH, OW, Ca, ka, epi=None, f8=None):
    """(k, s, p) and x's shape are the launch geometry; Ca / ka the layer's real input channels and kernel
    (they differ for the space-to-depth stem and the channel-padded stem), used for the flop / byte count.
    epi = (scale, shift, act, res, rps): fused inference epilogue (dmy_conv_fwd_act)
    f8 = (x8, amax, w8, wscale): run on the e4m3 kernel (dmy_conv_fwd_fp8, timer kind conv_fwd_f8)"""
    N, C, H, W = x.shape
    es = x.element_size()
    Hi, Wi = (2 * H, 2 * W) if ka != k else (H, W)
    kw = dict(tag=(N, Ca, Hi, Wi, K, ka, s if ka == k else 2),
              nbytes=es * (N * H * W * C + K * C * k * k + N * OH * OW * K))
    fl = 2.0 * N * OH * OW * K * Ca * ka * ka
    if f8 is not None:
        x8, amax, w8, ws = f8
        sc, sh, act, res, rps = epi if epi is not None else (None, None, 0, None, 0)
        kw['nbytes'] = N * H * W * C + K * C * k * k + es * N * OH * OW * K
        KernelTimer.run('conv_fwd_f8', fl, 'dmy_conv_fwd_fp8', ptr(x8), ptr(w8), ptr(amax), ptr(ws), ptr(bias), ptr(y),
                        ptr(psum), ptr(psq), N, H, W, C, K, k, k, s, p, OH, OW, yps, ptr(sc), ptr(sh), act, ptr(res),
                        rps, stream(), **kw)
        return
    ne = call('dmy_conv_fwd_splitk_elems', dcode(x), ptr(x), ptr(wf), ptr(y), N, H, W, C, xps, K, k, k, s, p, OH, OW,
              yps) if psum is None else 0
    if ne > 0:  # small M (batch-1 inference): split-K over the chip, reduced with the epilogue
        sc, sh, act, res, rps = epi if epi is not None else (None, None, 0, None, 0)
        ws = f32(ne, x.device)
        KernelTimer.run('conv_fwd', fl, 'dmy_conv_fwd_act_ws', dcode(x), ptr(x), ptr(wf), ptr(bias), ptr(y), N, H, W,
                        C, xps, K, k, k, s, p, OH, OW, yps, ptr(sc), ptr(sh), act, ptr(res), rps, ptr(ws), ne, stream(),
                        **kw)
    elif epi is None:
        KernelTimer.run('conv_fwd', fl, 'dmy_conv_fwd', dcode(x), ptr(x), ptr(wf), ptr(bias), ptr(y), ptr(psum),
                        ptr(psq), N, H, W, C, xps, K, k, k, s, p, OH, OW, yps, stream(), **kw)
    else:
        sc, sh, act, res, rps = epi
        KernelTimer.run('conv_fwd', fl, 'dmy_conv_fwd_act', dcode(x), ptr(x), ptr(wf), ptr(bias), ptr(y), N, H, W, C,
                        xps, K, k, k, s, p, OH, OW, yps, ptr(sc), ptr(sh), act, ptr(res), rps, stream(), **kw)


def eval_coef(spec, dev):
    """eval-mode BN scale / shift from the running statistics (dmy_bn_eval_coef), cached on the spec until a
    parameter / buffer changes (torch _version, or PARAM_GEN for our in-place kernels)"""
    bn = spec.bn
    key = (PARAM_GEN[0],) + tuple((t.data_ptr(), t._version) if t is not None else None
                                  for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)) + (float(bn.eps),)
    if spec.ecache is not None and spec.ecache[0] == key:
        return spec.ecache[1], spec.ecache[2]
    K = bn.running_mean.numel()
    scale, shift = f32(K, dev), f32(K, dev)
    call('dmy_bn_eval_coef', ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean), ptr(bn.running_var),
         float(bn.eps), K, ptr(scale), ptr(shift), stream())
    spec.ecache = (key, scale, shift)
    return scale, shift


class BnLink:
    """A train-mode BN layer whose BN the consumer applies (SCConv's k3, applied by its gate: SCGateFn): the consumer's
    backward writes the layer's backward-reduce partials itself (dmy_scgate_bn_bwd), saving bn_bwd_reduce's pass over
    dy.  `ready` holds (the gradient buffer, its pixel stride, pdb, pdg, rows, its version); the producer's backward
    uses the partials only when the gradient it receives IS that buffer, unmodified, and falls back to
    dmy_bn_bwd_reduce otherwise.  (Round 2's data-grad-epilogue variant of the same partials, dmy_conv_dgrad_bn, measured
    slower end to end -- DMA-1536 140.8 -> 138.1 img/s, profiles/r02/ab_bnfuse.log -- and was removed in round 6.)"""
    __slots__ = ('scale', 'shift', 'mean', 'invstd', 'act', 'K', 'ready')

    def __init__(self, scale, shift, mean, invstd, act, K):
        self.scale, self.shift, self.mean, self.invstd, self.act, self.K = scale, shift, mean, invstd, act, K
        self.ready = None


# SCConv's k3 BatchNorm applied by its gate (SCGateFn, dmy_scgate_bn_*): DMY_DEFER_AFFINE=0 restores the separate
# bn_act_fwd / bn_bwd_reduce passes
DEFER_AFFINE = [os.environ.get('DMY_DEFER_AFFINE', '1') == '1']
# backward BN partials (> 256 rows) folded by the two-stage column sum before the finalize (DMY_BWD_COLSUM=0: off)
BWD_COLSUM = [os.environ.get('DMY_BWD_COLSUM', '1') == '1']


# fused 1x1 backward (bwd1x1.hip): BN apply + data-grad + weight-grad of a train-mode 1x1 Conv-BN-act layer in one
# launch, dz never stored.  DMY_BWD1X1=0 restores the three-pass path (A/B, parity tests)
BWD1X1 = [os.environ.get('DMY_BWD1X1', '1') == '1']


def _bwd1x1(ctx, dy, dps, x, xps, wt, z, scale, shift, mean, invstd, ca, cb, cc, N, C, H, W, K, k, s, p, M):
    """-> (dx, dw) when the fused kernel took the layer's apply + data-grad + weight-grad, else None.  Eligible: bf16
    storage, train-mode BN, 1x1 stride 1, both gradients wanted, a (K, C) pair the kernel
    is built for (dmy_conv1x1_bwd_bn_ok).  Deterministic mode: the weight-grad partials go through a workspace summed
    in block order instead of fp32 atomics."""
    if not (BWD1X1[0] and ctx.train_bn and k == 1 and s == 1 and p == 0 and not ctx.s2d and ctx.cp == C and
            dy.dtype == torch.bfloat16 and wt is not None and ctx.needs_input_grad[0] and ctx.needs_input_grad[1]):
        return None
    buf_probe = ctx.xsink.peek(N, C, H, W) if ctx.xsink is not None else None
    bps_probe = buf_probe[1] if buf_probe is not None else C
    if not call('dmy_conv1x1_bwd_bn_ok', M, K, C, dps, xps, bps_probe, ptr(dy), ptr(z), ptr(x),
                ptr(buf_probe[0]) if buf_probe is not None else ptr(z)):
        return None
    dev = dy.device
    buf, bps, acc = sink_target(ctx.xsink, N, C, H, W, z)
    dw = ctx.arena.take(ctx.wkey, (K, C, 1, 1)) if ctx.arena is not None else None
    if dw is None:
        dw = torch.zeros((K, C, 1, 1), dtype=torch.float32, device=dev)
    es = z.element_size()
    ne = call('dmy_conv1x1_bwd_bn_ws_elems', M, K, C) if DETERMINISTIC[0] else 0
    ws = f32(ne, dev) if ne else None
    KernelTimer.run('conv_bwd1x1', 4.0 * M * K * C, 'dmy_conv1x1_bwd_bn', ptr(dy), dps, ptr(z), ptr(x), xps, ptr(wt),
                    ptr(scale), ptr(shift), ptr(mean), ptr(invstd), ctx.spec.act, ptr(ca), ptr(cb), ptr(cc), ptr(buf),
                    bps, acc, ptr(dw), ptr(ws), ne, M, K, C, stream(), tag=(N, C, H, W, K, k, s),
                    nbytes=es * (2 * M * K + (2 + acc) * M * C + K * C) + 4 * K * C)
    return sink_result(ctx.xsink, buf), dw


class ConvBNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, res, spec, xsink=None, rsink=None, grad_on=True):
        s2d = getattr(x, '_dmy_s2d', 0)
        f8in, prod = getattr(x, '_dmy_f8', None), getattr(x, '_dmy_prod', None)
        out_req, _OUT[0] = _OUT[0], None  # conv_bn_act's out view, checked against the output geometry below
        K, C2, k, _ = weight.shape
        ctx.s2d = 0
        # ctx.needs_input_grad mirrors requires_grad even when the CALLER runs under torch.no_grad() (forward itself
        # always runs with grad disabled): `grad_on` is the caller's grad mode, so a no-grad call (detect / val with
        # parameters that require grad) takes the one-launch inference path
        need_grad = grad_on and any(ctx.needs_input_grad[:6])
        bn = spec.bn
        train_bn = bn is not None and (bn.training or not bn.track_running_stats)
        infer = not need_grad and not train_bn  # one fused launch: conv + eval-BN + act (+ residual)
        wkey = (PARAM_GEN[0], weight.data_ptr(), weight._version, x.dtype, s2d)
        cached = infer and spec.wcache is not None and spec.wcache[0] == wkey
        if s2d:
            # stem over the space-to-depth image (image_s2d): the k6 s2 p2 conv runs as k3 s1 p1 over Cs channels
            assert C2 == s2d and k == 6 and spec.stride == 2 and spec.pad == 2, 's2d input feeds only the k6 s2 p2 stem'
            x, xps = pixel_stride(x)
            N, Cs, H2, W2 = x.shape
            C, H, W = s2d, 2 * H2, 2 * W2
            OH, OW = H2, W2
            if cached:
                wf = spec.wcache[1]
            else:
                wf = torch.empty((K, 9 * Cs), dtype=x.dtype, device=x.device)
                call('dmy_conv_wprep_s2d', DT[x.dtype], ptr(weight.detach().contiguous()), ptr(wf), K, C, Cs, stream())
                if infer:
                    spec.wcache = (wkey, wf)
            wt = None
            ctx.s2d = Cs
            # from here on the launch geometry is the k3 s1 p1 view
            Cg, Hg, Wg, kg, sg, pg = Cs, H2, W2, 3, 1, 1
            Cp = C
        else:
            cpad = zero_padded_channels(x)
            x, xps = pixel_stride(x)
            N, C, H, W = x.shape
            assert C2 == C, (C2, C)
            # stem: read the zero-padded storage as Cp channels (16-byte vectors) with zero weights
            Cp = cpad if (cpad and C % VW[x.dtype] and xps >= cpad) else C
            OH, OW = conv_out_hw(H, W, k, spec.stride, spec.pad)
            pre = WeightPrep.current.get(weight, x.dtype) if WeightPrep.current is not None and Cp == C else None
            if cached:
                wf, wt = spec.wcache[1], None
            elif pre is not None:
                wf, wt = pre
            else:
                wf, wt = prep_weight(weight, x.dtype, need_grad and Cp == C, Cp)
                if infer:
                    spec.wcache = (wkey, wf)
            if Cp != C:
                x = x.as_strided((N, Cp, H, W), x.stride())
            Cg, Hg, Wg, kg, sg, pg = Cp, H, W, k, spec.stride, spec.pad
        s, p = spec.stride, spec.pad
        dev, dt = x.device, x.dtype
        M = N * OH * OW
        f8 = None
        if spec.fp8 and not s2d and Cp == C and fp8_eligible(C, K, dt, N * H * W):
            if f8in is not None and (f8in[0].numel() != N * H * W * C or not F8_DELAYED[0]):
                f8in = None
            f8 = _fp8_operands(x, xps, weight, spec, wkey, f8in)
            if f8in is None and prod is not None and prod.f8_emit is None and F8_DELAYED[0] and not infer:
                prod.f8_emit = F8Emit(dev)  # from the next step on, the producer emits this input's e4m3 copy
        if res is not None:
            res, rps = pixel_stride(res)
        else:
            rps = 0
        _OUT[0] = out_req
        out = _take_out(N, K, OH, OW, x) if (bn is not None or spec.act != ACT_NONE or res is not None) else None
        yps = pixel_stride(out)[1] if out is not None else K
        if infer:
            y = out if out is not None else new_act(N, K, OH, OW, x)
            scale, shift = eval_coef(spec, dev) if bn is not None else (None, None)
            if scale is None and spec.act == ACT_NONE and res is None:
                _launch_conv_fwd(x, xps, wf, bias, y, yps, None, None, K, kg, sg, pg, OH, OW, C, k, f8=f8)
            else:
                _launch_conv_fwd(x, xps, wf, bias, y, yps, None, None, K, kg, sg, pg, OH, OW, C, k,
                                 epi=(scale, shift, spec.act, res, rps), f8=f8)
            return y
        z = new_act(N, K, OH, OW, x)
        if bn is not None:
            scale, shift, mean, invstd = f32(K, dev), f32(K, dev), f32(K, dev), f32(K, dev)
            if train_bn:
                if f8 is not None:
                    P = call('dmy_conv_fwd_fp8_partial_rows', M, K)
                else:  # rows for any route; the launch reports the rows its kernel wrote (halo / LANE: per wave)
                    P = call('dmy_conv_fwd_bound_rows', M, K)
                psum, psq = f32(P * K, dev), f32(P * K, dev)
                _launch_conv_fwd(x, xps, wf, bias, z, K, psum, psq, K, kg, sg, pg, OH, OW, C, k, f8=f8)
                if f8 is None:
                    P = call('dmy_conv_fwd_last_rows')
                if P > 256:  # two-stage column reduction of the epilogue partials
                    S = call('dmy_colsum2_rows', P)
                    ps2, pq2 = f32(S * K, dev), f32(S * K, dev)
                    call('dmy_colsum2', ptr(psum), ptr(psq), P, K, ptr(ps2), ptr(pq2), stream())
                    psum, psq, P = ps2, pq2, S
                upd = int(bn.training and bn.track_running_stats)
                if upd:
                    PARAM_GEN[0] += 1  # running stats change behind torch's back: drop inference caches
                mom = bn.momentum if bn.momentum is not None else 0.0
                call('dmy_bn_finalize', ptr(psum), ptr(psq), P, K, float(M), ptr(bn.weight), ptr(bn.bias),
                     ptr(bn.running_mean) if upd else None, ptr(bn.running_var) if upd else None,
                     ptr(bn.num_batches_tracked) if upd else None, float(mom), float(bn.eps), upd,
                     ptr(mean), ptr(invstd), ptr(scale), ptr(shift), stream())
            else:
                _launch_conv_fwd(x, xps, wf, bias, z, K, None, None, K, kg, sg, pg, OH, OW, C, k, f8=f8)
                call('dmy_bn_eval_coef', ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean), ptr(bn.running_var),
                     float(bn.eps), K, ptr(scale), ptr(shift), stream())
            defer = (spec.defer and DEFER_AFFINE[0] and train_bn and need_grad and dt == torch.bfloat16 and
                     spec.act == ACT_NONE and res is None and out is None and K % 8 == 0 and f8 is None)
            if defer:
                # the consumer (SCGateFn) reads z and applies scale / shift itself, and hands this layer's backward the
                # reduce partials (BnLink): the tensor returned is z, valid only for that consumer
                ctx.save_for_backward(x, wt, z, scale, shift, mean, invstd, bn.weight if bn.weight is not None else None)
                # the link must NOT hold z here: z is this Function's OUTPUT, so ctx -> link -> z -> grad_fn -> ctx would
                # be a reference cycle through the C++ autograd node that Python's GC cannot break (round 4 leaked
                # every SCConv's z, ~4 GiB per DMA-1536 step).  The gate receives z as its own input.
                ctx.bnlink = BnLink(scale, shift, mean, invstd, spec.act, K)
                z._dmy_affine, z._dmy_bnlink = (scale, shift, mean, invstd), ctx.bnlink
                ctx.spec, ctx.train_bn, ctx.has_res = spec, train_bn, False
                ctx.geom = (N, C, H, W, xps, K, k, s, p, OH, OW)
                ctx.ggeom = (Hg, Wg, kg, sg, pg)
                ctx.cp = Cp
                ctx.has_bias = bias is not None
                ctx.xsink, ctx.rsink = xsink, rsink
                ctx.arena = WgradArena.current
                ctx.wkey = weight.data_ptr()
                ctx.pkeys = tuple(t.data_ptr() if t is not None else None for t in (bias, gamma, beta))
                return z
            y = out if out is not None else new_act(N, K, OH, OW, x)
            emit = spec.f8_emit if (F8_DELAYED[0] and dt == torch.bfloat16 and K % 8 == 0 and yps % 8 == 0 and
                                    (res is None or rps % 8 == 0)) else None
            if emit is not None and not torch.cuda.is_current_stream_capturing():
                e8 = emit.run(z, scale, shift, spec.act, res, rps, y, yps, M, K)
                if e8 is not None:
                    y._dmy_f8 = e8
            else:
                call('dmy_bn_act_fwd', dcode(x), ptr(z), K, ptr(scale), ptr(shift), spec.act, ptr(res), rps, ptr(y),
                     yps, M, K, stream())
            if dt == torch.bfloat16 and K % 128 == 0 and train_bn:
                y._dmy_prod = spec  # an fp8 consumer may ask this layer to emit its e4m3 copy (F8Emit)
            ctx.save_for_backward(x, wt, z, scale, shift, mean, invstd, bn.weight if bn.weight is not None else None)
            ctx.bnlink = None
        else:
            _launch_conv_fwd(x, xps, wf, bias, z, K, None, None, K, kg, sg, pg, OH, OW, C, k, f8=f8)
            if spec.act != ACT_NONE or res is not None:
                y = out if out is not None else new_act(N, K, OH, OW, x)
                one, zero = const_vec(K, 1.0, dev), const_vec(K, 0.0, dev)
                call('dmy_bn_act_fwd', dcode(x), ptr(z), K, ptr(one), ptr(zero), spec.act, ptr(res), rps, ptr(y), yps,
                     M, K, stream())
            else:
                y = z
            ctx.save_for_backward(x, wt, z)
        ctx.spec, ctx.train_bn, ctx.has_res = spec, train_bn, res is not None
        ctx.geom = (N, C, H, W, xps, K, k, s, p, OH, OW)
        ctx.ggeom = (Hg, Wg, kg, sg, pg)
        ctx.cp = Cp
        ctx.has_bias = bias is not None
        ctx.xsink, ctx.rsink = xsink, rsink
        ctx.arena = WgradArena.current
        ctx.wkey = weight.data_ptr()
        ctx.pkeys = tuple(t.data_ptr() if t is not None else None for t in (bias, gamma, beta))
        return y

    @staticmethod
    def backward(ctx, dy):
        spec = ctx.spec
        N, C, H, W, xps, K, k, s, p, OH, OW = ctx.geom
        dy, dps = pixel_stride(dy.to(ctx.saved_tensors[2].dtype))
        dev = dy.device
        M = N * OH * OW
        dt = dcode(dy)
        dbias = dgamma = dbeta = None
        arena = ctx.arena

        def pgrad(key, zero=False):
            """the parameter's gradient tensor: its (zeroed) arena slice, else a fresh one"""
            g = arena.take(key, (K,)) if (arena is not None and key is not None) else None
            if g is None:
                g = torch.zeros(K, dtype=torch.float32, device=dev) if zero else f32(K, dev)
            return g

        if spec.bn is not None:
            x, wt, z, scale, shift, mean, invstd, gamma = ctx.saved_tensors
            dz = new_act(N, K, OH, OW, z)
            ca, cb, cc = f32(K, dev), f32(K, dev), f32(K, dev)
            if ctx.train_bn:
                link = getattr(ctx, 'bnlink', None)
                rd = link.ready if link is not None else None
                if link is not None:
                    link.ready = None
                if rd is not None and rd[0].data_ptr() == dy.data_ptr() and rd[1] == dps and \
                        rd[0]._version == rd[5]:
                    _, _, pdb, pdg, P, _ = rd  # written by the consumer (data-grad epilogue / SCConv gate)
                else:
                    P = call('dmy_bn_reduce_rows', dt, ptr(z), K, ptr(dy), dps, M, K)
                    pdb, pdg = f32(P * K, dev), f32(P * K, dev)
                    call('dmy_bn_bwd_reduce', dt, ptr(z), K, ptr(dy), dps, ptr(scale), ptr(shift), ptr(mean),
                         ptr(invstd), spec.act, M, K, ptr(pdb), ptr(pdg), stream())
                if P > 256 and BWD_COLSUM[0]:
                    # up to 4096 block rows: the one-block-per-channel finalize read them with a stride of K floats in
                    # 20 us per layer (97 layers per DMA-1536 step); the two-stage column sum reads them coalesced
                    S = call('dmy_colsum2_rows', P)
                    pd2, pg2 = f32(S * K, dev), f32(S * K, dev)
                    call('dmy_colsum2', ptr(pdb), ptr(pdg), P, K, ptr(pd2), ptr(pg2), stream())
                    pdb, pdg, P = pd2, pg2, S
                dgamma, dbeta = pgrad(ctx.pkeys[1]), pgrad(ctx.pkeys[2])
                call('dmy_bn_bwd_finalize', ptr(pdb), ptr(pdg), P, K, float(M), ptr(gamma), ptr(invstd), ptr(dgamma),
                     ptr(dbeta), ptr(ca), ptr(cb), ptr(cc), stream())
            else:
                ca.copy_(scale)
                cb.zero_()
                cc.zero_()
            fused = _bwd1x1(ctx, dy, dps, x, xps, wt, z, scale, shift, mean, invstd, ca, cb, cc, N, C, H, W, K, k, s,
                            p, M)
            if fused is not None:
                dx, dw = fused
                dbias = pgrad(ctx.pkeys[0], zero=True) if ctx.has_bias else None  # sum(dz) == 0 behind train-mode BN
                dres = (dy if ctx.rsink is None else ctx.rsink.passthrough(dy)) if ctx.has_res else None
                return dx, dw, dbias, dgamma, dbeta, dres, None, None, None, None
            call('dmy_bn_bwd_apply', dt, ptr(z), K, ptr(dy), dps, ptr(scale), ptr(shift), ptr(mean), ptr(invstd),
                 spec.act, ptr(ca), ptr(cb), ptr(cc), ptr(dz), K, M, K, stream())
            dzps = K
        else:
            x, wt, z = ctx.saved_tensors
            if spec.act != ACT_NONE:
                dz = new_act(N, K, OH, OW, z)
                zero, one = const_vec(K, 0.0, dev), const_vec(K, 1.0, dev)
                call('dmy_bn_bwd_apply', dt, ptr(z), K, ptr(dy), dps, ptr(one), ptr(zero), ptr(zero), ptr(one),
                     spec.act, ptr(one), ptr(zero), ptr(zero), ptr(dz), K, M, K, stream())
                dzps = K
            else:
                dz, dzps = dy, dps
            if ctx.has_bias:
                P = call('dmy_bn_reduce_rows', dt, ptr(dz), dzps, None, 0, M, K)
                ps_, pq_ = f32(P * K, dev), f32(P * K, dev)
                call('dmy_bn_stats', dt, ptr(dz), dzps, M, K, ptr(ps_), ptr(pq_), stream())
                dbias = pgrad(ctx.pkeys[0])
                call('dmy_reduce_rows', ptr(ps_), P, K, ptr(dbias), 0, stream())
        if spec.bn is not None and ctx.has_bias and ctx.train_bn:
            dbias = pgrad(ctx.pkeys[0], zero=True)  # sum(dz) == 0 exactly behind train-mode BN
        dx = dw = None
        Cp = ctx.cp
        if ctx.needs_input_grad[0]:
            if Cp != C or ctx.s2d:
                raise NotImplementedError('input gradient of a channel-padded stem conv')
            buf, bps, acc = sink_target(ctx.xsink, N, C, H, W, z)
            kw = dict(tag=(N, C, H, W, K, k, s),
                      nbytes=z.element_size() * (M * K + K * C * k * k + (1 + acc) * N * H * W * C))
            fl = 2.0 * M * K * C * k * k
            KernelTimer.run('conv_dgrad', fl, 'dmy_conv_dgrad', dt, ptr(dz), ptr(wt), ptr(buf), acc, N, H, W, C, bps,
                            K, k, k, s, p, OH, OW, dzps, stream(), **kw)
            dx = sink_result(ctx.xsink, buf)
        if ctx.needs_input_grad[1] and ctx.s2d:
            Cs = ctx.s2d
            H2, W2 = ctx.ggeom[:2]
            dwo = f32(K * 9 * Cs, dev)
            _wgrad(dt, x, dz, dwo, N, H2, W2, Cs, xps, K, 3, 1, 1, OH, OW, dzps, 0, 2.0 * M * K * C * k * k,
                   tag=(N, C, H, W, K, k, s), nbytes=z.element_size() * (N * H2 * W2 * Cs + M * K) + 4 * K * Cs * 9)
            dw = ctx.arena.take(ctx.wkey, (K, C, k, k)) if ctx.arena is not None else None
            if dw is None:
                dw = torch.empty((K, C, k, k), dtype=torch.float32, device=dev)
            call('dmy_conv_wgrad_s2d_to_oihw', ptr(dwo), ptr(dw), K, C, Cs, stream())
        elif ctx.needs_input_grad[1]:
            wkw = dict(tag=(N, C, H, W, K, k, s), nbytes=z.element_size() * (N * H * W * Cp + M * K) + 4 * K * Cp * k * k)
            dw = ctx.arena.take(ctx.wkey, (K, C, k, k)) if ctx.arena is not None else None
            zeroed = dw is not None
            if dw is None:
                dw = torch.empty((K, C, k, k), dtype=torch.float32, device=dev)
            if k == 1 and Cp == C:
                # 1x1: the GEMM view IS torch OIHW -> accumulate straight into the step's zeroed arena slice
                flags = WGRAD_OIHW | (WGRAD_ZEROED if zeroed else 0)
                _wgrad(dt, x, dz, dw, N, H, W, C, xps, K, k, s, p, OH, OW, dzps, flags, 2.0 * M * K * C * k * k, **wkw)
            else:
                # k > 1: OIHW-order atomics would scatter every tile row with stride k*k (measured 1.5x slower
                # weight-grad on yolov5s); accumulate in GEMM order, then one layout pass (drops stem padding)
                dwo = f32(K * Cp * k * k, dev)
                _wgrad(dt, x, dz, dwo, N, H, W, Cp, xps, K, k, s, p, OH, OW, dzps, 0, 2.0 * M * K * C * k * k, **wkw)
                call('dmy_conv_wgrad_to_oihw', ptr(dwo), ptr(dw), K, C, Cp, k, k, stream())
        dres = None
        if ctx.has_res:
            dres = dy if ctx.rsink is None else ctx.rsink.passthrough(dy)
        return dx, dw, dbias, dgamma, dbeta, dres, None, None, None, None


def conv_bn_act(x, weight, bias, bn, stride, pad, act, res=None, spec=None, xsink=None, rsink=None, out=None,
                defer=False):
    """xsink / rsink: GradSinks collecting the gradient of x / of the residual (see GradSink).  out: an NHWC view
    (a concat_buffer channel slice) the activation is written into instead of a fresh tensor, when the layer has a
    separate activation pass (BN and / or act / residual); the returned tensor is then that view."""
    if spec is None:  # a persistent spec per weight PARAMETER (views made per call share their base), so the
        # inference caches (prepped weight, eval BN coefficients) hold across calls for the Detect / Swin / CBAM convs
        spec = _param_spec(weight._base if weight._base is not None else weight, stride, pad, act, bn)
    spec.defer = bool(defer)
    gamma = bn.weight if bn is not None else None
    beta = bn.bias if bn is not None else None
    _OUT[0] = out
    try:
        return ConvBNActFn.apply(x, weight, bias, gamma, beta, res, spec, xsink, rsink, torch.is_grad_enabled())
    finally:
        _OUT[0] = None


# ------------------------------------------------------------------ pooling / resize / concat

class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, sink=None, out=None):
        """out: None or [view] -- a concat_buffer channel slice the pooled map is written into (SPPF / SPPFCSPC), in a
        list so autograd does not treat the buffer as an input"""
        x, xps = pixel_stride(x)
        N, C, H, W = x.shape
        o = out[0] if out else None
        if o is not None and (tuple(o.shape) != (N, C, H, W) or o.dtype != x.dtype or pixel_stride(o)[0] is not o):
            o = None
        y, yps = (o, pixel_stride(o)[1]) if o is not None else (new_act(N, C, H, W, x), C)
        arg = torch.empty((N, H, W, C), dtype=torch.uint8, device=x.device)
        call('dmy_maxpool_fwd', dcode(x), ptr(x), xps, ptr(y), yps, ptr(arg), N, H, W, C, k, stream())
        ctx.save_for_backward(arg)
        ctx.k, ctx.shape, ctx.sink = k, (N, C, H, W), sink
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        dy, dps = pixel_stride(dy)
        buf, bps, acc = sink_target(ctx.sink, N, C, H, W, dy)
        call('dmy_maxpool_bwd', dcode(dy), ptr(dy), dps, ptr(arg), ptr(buf), bps, acc, N, H, W, C, ctx.k, stream())
        return sink_result(ctx.sink, buf), None, None, None


POOL3 = [os.environ.get('DMY_POOL3', '1') == '1']  # the one-launch pyramid (DMY_POOL3=0: three MaxPoolFn launches)


def maxpool_chain3(x, k, outs=(None, None, None)):
    """inference SPPF / SPPFCSPC pyramid: (pool(x), pool(pool(x)), pool(pool(pool(x)))) with the k x k stride-1 pool in
    ONE launch (dmy_maxpool_chain3_fwd, the bits of three MaxPoolFn launches), written into `outs` when they are three
    NHWC views with one pixel stride (concat_buffer slices), else into fresh tensors.  None when autograd is recording
    (the backward needs MaxPoolFn's argmax) or the kernel does not take the shape: the caller chains MaxPoolFn"""
    if torch.is_grad_enabled() or k not in (3, 5) or x.dtype not in (torch.bfloat16, torch.float32) or not POOL3[0]:
        return None
    x, xps = pixel_stride(x)
    N, C, H, W = x.shape
    vw = 8 if x.dtype == torch.bfloat16 else 4
    ys, yps = [], None
    for o in outs:
        if o is None or tuple(o.shape) != (N, C, H, W) or o.dtype != x.dtype or pixel_stride(o)[0] is not o or \
                (yps is not None and pixel_stride(o)[1] != yps):
            ys = None
            break
        yps = pixel_stride(o)[1]
        ys.append(o)
    if ys is None:
        ys, yps = [new_act(N, C, H, W, x) for _ in range(3)], C
    if C % vw or xps % vw or yps % vw or N * (C // vw) >= 65536 or any(t.data_ptr() % 16 for t in [x] + ys):
        return None
    call('dmy_maxpool_chain3_fwd', dcode(x), ptr(x), xps, ptr(ys[0]), ptr(ys[1]), ptr(ys[2]), yps, N, H, W, C, k,
         stream())
    return tuple(ys)


class AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, sink=None):
        x, xps = pixel_stride(x)
        N, C, H, W = x.shape
        y = new_act(N, C, H // r, W // r, x)
        call('dmy_avgpool_fwd', dcode(x), ptr(x), xps, ptr(y), N, H, W, C, r, stream())
        ctx.r, ctx.shape, ctx.sink = r, (N, C, H, W), sink
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.shape
        dy = dy.contiguous(memory_format=CL)
        buf, bps, acc = sink_target(ctx.sink, N, C, H, W, dy)
        call('dmy_avgpool_bwd', dcode(dy), ptr(dy), ptr(buf), bps, acc, N, H, W, C, ctx.r, stream())
        return sink_result(ctx.sink, buf), None, None


class ResizeFn(torch.autograd.Function):
    """nearest resize with ATen's index rule (F.interpolate(mode='nearest'), nn.Upsample)."""

    @staticmethod
    def forward(ctx, x, OH, OW, out=None):
        """out: None or [view] -- a concat_buffer channel slice the result is written into (Model's concat plan)"""
        x, xps = pixel_stride(x)
        N, C, H, W = x.shape
        o = out[0] if out else None
        if o is not None and (tuple(o.shape) != (N, C, OH, OW) or o.dtype != x.dtype or pixel_stride(o)[0] is not o):
            o = None
        y, yps = (o, pixel_stride(o)[1]) if o is not None else (new_act(N, C, OH, OW, x), C)
        call('dmy_resize_fwd', dcode(x), ptr(x), xps, ptr(y), yps, 1.0, N, H, W, OH, OW, C, stream())
        ctx.shape = (N, C, H, W, OH, OW)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W, OH, OW = ctx.shape
        dy, dps = pixel_stride(dy)
        dx = new_act(N, C, H, W, dy)
        call('dmy_resize_bwd', dcode(dy), ptr(dy), dps, ptr(dx), C, N, H, W, OH, OW, C, stream())
        return dx, None, None, None


CAT_DOT = [os.environ.get('DMY_CAT_DOT', '1') == '1']  # weighted-concat backward in one pass per input


class ConcatFn(torch.autograd.Function):
    """cat(w_i/(sum w + eps) * x_i) along channels (w=None: plain Concat)."""

    @staticmethod
    def forward(ctx, w, eps, sinks, *xs):
        """sinks: None or one GradSink-or-None per input (the slice gradient is handed to it)"""
        ctx.sinks = sinks
        base = _inplace_concat(xs) if w is None else None
        xs = [pixel_stride(x) for x in xs]
        N, _, H, W = xs[0][0].shape
        Ct = sum(x.shape[1] for x, _ in xs)
        y = base.detach() if base is not None else new_act(N, Ct, H, W, xs[0][0])
        c0 = 0
        M = N * H * W
        for i, (x, xps) in enumerate(xs):
            if base is not None:  # the producers wrote their slices in place (concat_buffer)
                break
            C = x.shape[1]
            call('dmy_slice_copy', dcode(x), ptr(x), xps, ctypes_off(y, c0), Ct, M, C, ptr(w), i,
                 len(xs) if w is not None else 0, float(eps), 0, stream())
            c0 += C
        ctx.chans = [x.shape[1] for x, _ in xs]
        ctx.eps = eps
        if w is not None:
            ctx.save_for_backward(w, *[x for x, _ in xs])
        else:
            ctx.save_for_backward()
        ctx.has_w = w is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        dy, dps = pixel_stride(dy)
        N, Ct, H, W = dy.shape
        M = N * H * W
        grads, c0 = [], 0
        sinks = ctx.sinks or [None] * len(ctx.chans)
        if not ctx.has_w:
            for C, sk in zip(ctx.chans, sinks):
                sl = dy[:, c0:c0 + C]
                grads.append(sl if sk is None else sk.passthrough(sl))
                c0 += C
            return (None, None, None, *grads)
        w, *xs = ctx.saved_tensors
        nb = call('dmy_dot_partial_blocks', M, max(ctx.chans))
        part = torch.zeros((len(xs), nb), dtype=torch.float32, device=dy.device)
        for i, (x, C) in enumerate(zip(xs, ctx.chans)):
            x, xps = pixel_stride(x)
            g, gps, acc = sink_target(sinks[i], N, C, H, W, dy)
            sl = dy[:, c0:c0 + C]
            vw = 8 if dy.dtype == torch.bfloat16 else 4
            if CAT_DOT[0] and C % vw == 0 and dps % vw == 0 and gps % vw == 0 and xps % vw == 0 and \
                    all(t.data_ptr() % 16 == 0 for t in (sl, g, x)):  # one pass over the dy slice
                call('dmy_slice_copy_dot', dcode(dy), ptr(sl), dps, ptr(g), gps, ptr(x), xps, M, C, ptr(w), i, len(xs),
                     float(ctx.eps), acc, ptr(part[i]), stream())
            else:
                call('dmy_slice_copy', dcode(dy), ptr(sl), dps, ptr(g), gps, M, C, ptr(w), i, len(xs), float(ctx.eps),
                     acc, stream())
                call('dmy_dot_partial', dcode(dy), ptr(sl), dps, ptr(x), xps, M, C, ptr(part[i]), stream())
            g = sink_result(sinks[i], g)
            nbi = call('dmy_dot_partial_blocks', M, C)
            if nbi < nb:
                part[i, nbi:].zero_()
            grads.append(g)
            c0 += C
        dw = torch.empty_like(w)
        call('dmy_bifpn_wgrad', ptr(part), nb, len(xs), ptr(w), float(ctx.eps), ptr(dw), stream())
        return (dw, None, None, *grads)


def _inplace_concat(xs):
    """the concat_buffer whose consecutive channel slices the inputs are, in order, or None"""
    b = xs[0]._base
    if b is None or b.dim() != 4 or not b.is_contiguous(memory_format=CL):
        return None
    N, Ct, H, W = b.shape
    c0, es = 0, b.element_size()
    for x in xs:
        if x._base is not b or x.shape[0] != N or x.shape[2:] != b.shape[2:] or \
                x.data_ptr() != b.data_ptr() + c0 * es or x.stride() != b.stride():
            return None
        c0 += x.shape[1]
    return b if c0 == Ct else None


def ctypes_off(t, c0):
    import ctypes
    return ctypes.c_void_p(t.data_ptr() + c0 * t.element_size())


# ------------------------------------------------------------------ SCConv gate / CoorAttention

class SCGateFn(torch.autograd.Function):
    """out = u3 * sigmoid(x + nearest(g))  (models/common.py:1311-1314).  When u3 is k3's deferred BN output (z with
    `_dmy_affine`, conv_bn_act(defer=True)), the gate applies k3's BN scale / shift to z itself and its backward writes
    k3's BN backward-reduce partials into k3's BnLink (dmy_scgate_bn_fwd / _bwd), so k3's bn_act_fwd and
    bn_bwd_reduce passes disappear."""

    @staticmethod
    def forward(ctx, x, u3, g, sink=None):
        ctx.sink = sink
        aff, link = getattr(u3, '_dmy_affine', None), getattr(u3, '_dmy_bnlink', None)
        x, xps = pixel_stride(x)
        g = g.contiguous(memory_format=CL)
        N, C, H, W = x.shape
        GH, GW = g.shape[2:]
        out = new_act(N, C, H, W, x)
        ctx.aff = ctx.link = None
        if aff is not None:
            assert pixel_stride(u3)[0] is u3 and u3.stride(1) == 1 and u3.stride(3) == C, 'deferred z must be dense NHWC'
            call('dmy_scgate_bn_fwd', ptr(x), xps, ptr(u3), ptr(aff[0]), ptr(aff[1]), ptr(g), ptr(out), N, H, W, C, GH,
                 GW, stream())
            ctx.aff, ctx.link = aff, link
        else:
            u3 = u3.contiguous(memory_format=CL)
            call('dmy_scgate_fwd', dcode(x), ptr(x), xps, ptr(u3), ptr(g), ptr(out), N, H, W, C, GH, GW, stream())
        ctx.save_for_backward(x, u3, g)
        ctx.xps = xps
        return out

    @staticmethod
    def backward(ctx, dout):
        x, u3, g = ctx.saved_tensors
        N, C, H, W = x.shape
        GH, GW = g.shape[2:]
        dout = dout.contiguous(memory_format=CL)
        du3 = new_act(N, C, H, W, x)
        # d(x + up(g)) -> x's gradient sink; the resize backward of g needs it on its own
        dpre = new_act(N, C, H, W, x)
        if ctx.aff is not None:
            sc, sh, mean, invstd = ctx.aff
            P = call('dmy_scgate_bn_rows', N, H, W, C)
            pdb, pdg = f32(P * C, x.device), f32(P * C, x.device)
            call('dmy_scgate_bn_bwd', ptr(x), ctx.xps, ptr(u3), ptr(sc), ptr(sh), ptr(mean), ptr(invstd), ptr(g),
                 ptr(dout), ptr(du3), ptr(dpre), N, H, W, C, GH, GW, ptr(pdb), ptr(pdg), stream())
            # k3's ConvBNActFn backward takes these partials iff the gradient it receives IS du3, unmodified
            ctx.link.ready = (du3, C, pdb, pdg, P, du3._version)
        else:
            call('dmy_scgate_bwd', dcode(x), ptr(x), ctx.xps, ptr(u3), ptr(g), ptr(dout), ptr(du3), ptr(dpre), C, 0,
                 N, H, W, C, GH, GW, stream())
        dg = new_act(N, C, GH, GW, x)
        call('dmy_resize_bwd', dcode(x), ptr(dpre), C, ptr(dg), C, N, GH, GW, H, W, C, stream())
        dx = dpre if ctx.sink is None else ctx.sink.passthrough(dpre)
        return dx, du3, dg, None


class CAPoolFn(torch.autograd.Function):
    """[N,C,H,W] -> [N,C,H+W,1]: row means then column means (CoorAttention pool_h / pool_w + cat)."""

    @staticmethod
    def forward(ctx, x):
        x, xps = pixel_stride(x)
        N, C, H, W = x.shape
        y = new_act(N, C, H + W, 1, x)
        call('dmy_ca_pool_fwd', dcode(x), ptr(x), xps, ptr(y), N, H, W, C, stream())
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.shape
        dy = dy.contiguous(memory_format=CL)
        dx = new_act(N, C, H, W, dy)
        call('dmy_ca_pool_bwd', dcode(dy), ptr(dy), ptr(dx), C, 0, N, H, W, C, stream())
        return dx


class CAApplyFn(torch.autograd.Function):
    """out = x * sigmoid(lw)[w] * sigmoid(lh)[h]; lh/lw are conv_h/conv_w logits over all H+W rows."""

    @staticmethod
    def forward(ctx, x, lh, lw):
        x, xps = pixel_stride(x)
        lh = lh.contiguous(memory_format=CL)
        lw = lw.contiguous(memory_format=CL)
        N, C, H, W = x.shape
        out = new_act(N, C, H, W, x)
        call('dmy_ca_apply_fwd', dcode(x), ptr(x), xps, ptr(lh), ptr(lw), ptr(out), C, N, H, W, C, stream())
        ctx.save_for_backward(x, lh, lw)
        ctx.xps = xps
        return out

    @staticmethod
    def backward(ctx, dout):
        x, lh, lw = ctx.saved_tensors
        N, C, H, W = x.shape
        dout, dps = pixel_stride(dout)
        dx = new_act(N, C, H, W, x)
        dlh = torch.empty_like(lh)
        dlw = torch.empty_like(lw)
        call('dmy_ca_apply_bwd', dcode(x), ptr(x), ctx.xps, ptr(lh), ptr(lw), ptr(dout), dps, ptr(dx), C, ptr(dlh),
             ptr(dlw), N, H, W, C, stream())
        return dx, dlh, dlw


# ------------------------------------------------------------------ misc pointwise

class AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, asink=None):
        ctx.asink = asink
        a = a.contiguous(memory_format=CL) if a.dim() == 4 else a.contiguous()
        b = b.contiguous(memory_format=CL) if b.dim() == 4 else b.contiguous()
        y = torch.empty_like(a)
        call('dmy_pointwise', dcode(a), 0, 0, ptr(a), ptr(b), ptr(y), a.numel(), 1.0, stream())
        return y

    @staticmethod
    def backward(ctx, dy):
        da = dy if ctx.asink is None else ctx.asink.passthrough(dy)
        return da, dy, None


def image_s2d(x, dtype):
    """NCHW image (uint8 -> /255, or float) -> space-to-depth NHWC storage [N, Cs, H/2, W/2] for the k6 s2 p2
    stem (csrc dmy_image_s2d); the result carries `_dmy_s2d` = C, read by ConvBNActFn.  No gradient."""
    N, C, H, W = x.shape
    Cs = -(-4 * C // VW[dtype]) * VW[dtype]
    buf = torch.empty((N, Cs, H // 2, W // 2), dtype=dtype, device=x.device, memory_format=CL)
    xc = x.detach().contiguous()
    if x.dtype == torch.uint8:
        call('dmy_image_s2d', DT[dtype], 0, ptr(xc), ptr(buf), N, C, H, W, Cs, 1.0 / 255.0, stream())
    else:
        xf = xc if xc.dtype == torch.float32 else xc.float()
        call('dmy_image_s2d', DT[dtype], 1, ptr(xf), ptr(buf), N, C, H, W, Cs, 1.0, stream())
    buf._dmy_s2d = C
    return buf


class ToNHWC(torch.autograd.Function):
    """NCHW float/uint8 image -> NHWC storage dtype (train.py:402 `/255` when uint8).  The pixel
    stride is rounded up to a 16-byte vector with zero channels so the stem conv stays vectorised."""

    @staticmethod
    def forward(ctx, x, dtype):
        N, C, H, W = x.shape
        Cp = -(-C // VW[dtype]) * VW[dtype]
        buf = torch.empty((N, Cp, H, W), dtype=dtype, device=x.device, memory_format=CL)
        xc = x.contiguous()
        if x.dtype == torch.uint8:
            call('dmy_nchw_to_nhwc', DT[dtype], 0, ptr(xc), ptr(buf), N, C, H, W, Cp, 1.0 / 255.0, stream())
        else:
            xf = xc if x.dtype == torch.float32 else xc.float()
            call('dmy_nchw_to_nhwc', DT[dtype], 1, ptr(xf), ptr(buf), N, C, H, W, Cp, 1.0, stream())
        ctx.src_dtype = x.dtype
        ctx.mark_non_differentiable(buf) if x.dtype == torch.uint8 else None
        return buf[:, :C] if Cp != C else buf

    @staticmethod
    def backward(ctx, dy):
        if ctx.src_dtype == torch.uint8:
            return None, None
        dy, dps = pixel_stride(dy)
        N, C, H, W = dy.shape
        dx = torch.empty((N, C, H, W), dtype=torch.float32, device=dy.device)
        call('dmy_nhwc_to_nchw_f32', dcode(dy), ptr(dy), dps, ptr(dx), N, C, H, W, stream())
        return dx.to(ctx.src_dtype), None


# ------------------------------------------------------------------ Swin pieces (csrc/swin.hip)

class LayerNormFn(torch.autograd.Function):
    """nn.LayerNorm over channels of an NHWC activation (common.py:560, 565)."""

    @staticmethod
    def forward(ctx, x, w, b, eps, sink=None):
        ctx.sink = sink
        x, xps = pixel_stride(x)
        N, C, H, W = x.shape
        M = N * H * W
        y = new_act(N, C, H, W, x)
        mean, rstd = f32(M, x.device), f32(M, x.device)
        call('dmy_layernorm_fwd', dcode(x), ptr(x), xps, ptr(w), ptr(b), ptr(y), ptr(mean), ptr(rstd), M, C,
             float(eps), stream())
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.xps = xps
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        N, C, H, W = x.shape
        M = N * H * W
        dy, dps = pixel_stride(dy)
        buf, bps, acc = sink_target(ctx.sink, N, C, H, W, x)
        P = call('dmy_layernorm_bwd_blocks', M)
        pdw, pdb = f32(P * C, x.device), f32(P * C, x.device)
        call('dmy_layernorm_bwd', dcode(x), ptr(x), ctx.xps, ptr(dy), dps, ptr(w), ptr(mean), ptr(rstd), ptr(buf), bps,
             acc, M, C, ptr(pdw), ptr(pdb), stream())
        dx = sink_result(ctx.sink, buf)
        dw, db = f32(C, x.device), f32(C, x.device)
        call('dmy_reduce_rows', ptr(pdw), P, C, ptr(dw), 0, stream())
        call('dmy_reduce_rows', ptr(pdb), P, C, ptr(db), 0, stream())
        return dx, dw, db, None, None


class WinAttnFn(torch.autograd.Function):
    """Shifted-window MHSA core (common.py:500-545 + 595-631): qkv [N,3C,H,W] NHWC -> [N,C,H,W]."""

    @staticmethod
    def forward(ctx, qkv, table, nh, shift, scale):
        qkv = qkv.contiguous(memory_format=CL)
        N, C3, H, W = qkv.shape
        C = C3 // 3
        out = torch.empty((N, C, H, W), dtype=qkv.dtype, device=qkv.device, memory_format=CL)  # every pixel is written
        tab = table.detach().float().contiguous()
        call('dmy_winattn_fwd', dcode(qkv), ptr(qkv), ptr(tab), ptr(out), N, H, W, C, nh, shift, float(scale),
             stream())
        ctx.save_for_backward(qkv, tab)
        ctx.cfg = (nh, shift, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, tab = ctx.saved_tensors
        nh, shift, scale = ctx.cfg
        N, C3, H, W = qkv.shape
        dout = dout.contiguous(memory_format=CL)
        dqkv = torch.empty_like(qkv, memory_format=CL)  # every pixel belongs to exactly one window
        groups = call('dmy_winattn_bwd_groups', N, H, W, nh)
        part = f32(groups * nh * 225, qkv.device)
        dtab = torch.empty_like(tab)
        call('dmy_winattn_bwd', dcode(qkv), ptr(qkv), ptr(dout), ptr(tab), ptr(dqkv), ptr(part), ptr(dtab), N, H, W,
             C3 // 3, nh, shift, float(scale), stream())
        return dqkv, dtab, None, None, None


class MHAFn(torch.autograd.Function):
    """Global multi-head attention core of nn.MultiheadAttention (common.py:323, C3TR): q, k, v are the
    in-projected NHWC token tensors [N, c, H, W] (tokens = the H*W pixels of one image); returns
    softmax(q k^T / sqrt(d)) v per head, [N, c, H, W].  Kernels: csrc/mha.hip (flash-style, nothing
    L x L is stored; the backward recomputes P from the saved log-sum-exp)."""

    @staticmethod
    def forward(ctx, q, k, v, nh):
        q, qps = pixel_stride(q)
        k, kps = pixel_stride(k)
        v, vps = pixel_stride(v)
        N, C, H, W = q.shape
        assert C % nh == 0 and k.shape == q.shape and v.shape == q.shape
        d, L = C // nh, H * W
        o = new_act(N, C, H, W, q)
        lse = f32(N * nh * L, q.device)
        call('dmy_mha_fwd', dcode(q), ptr(q), qps, ptr(k), kps, ptr(v), vps, ptr(o), C, ptr(lse), N, L, nh, d,
             float(d) ** -0.5, stream())
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.ps, ctx.nh = (qps, kps, vps), nh
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        qps, kps, vps = ctx.ps
        N, C, H, W = q.shape
        nh = ctx.nh
        d, L = C // nh, H * W
        do = do.to(q.dtype).contiguous(memory_format=CL)
        dq, dk, dv = new_act(N, C, H, W, q), new_act(N, C, H, W, q), new_act(N, C, H, W, q)
        Dq = f32(N * nh * L, q.device)
        call('dmy_mha_bwd', dcode(q), ptr(q), qps, ptr(k), kps, ptr(v), vps, ptr(o), ptr(do), C, ptr(lse), ptr(Dq),
             ptr(dq), ptr(dk), ptr(dv), N, L, nh, d, float(d) ** -0.5, stream())
        return dq, dk, dv, None


_DROP_STATE = {}


def _seed(dev):
    """A fresh dropout seed in device memory: dmy_dropout_seed advances a per-device generator state (seeded
    once from torch's CPU generator) on the stream, so a HIP-graph replay of the step draws a new mask each
    time instead of replaying the captured one.  Returns the [1] int64 seed tensor the kernels read."""
    st = _DROP_STATE.get(dev)
    if st is None:
        st = _DROP_STATE[dev] = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).to(dev)
    seed = torch.empty(1, dtype=torch.int64, device=dev)
    call('dmy_dropout_seed', ptr(st), ptr(seed), stream())
    return seed


class DropoutFn(torch.autograd.Function):
    """nn.Dropout(p) in train mode (common.py:328): y = x * keep / (1 - p); the keep mask is a counter
    hash of (seed, element index), regenerated in the backward from the same device-resident seed."""

    @staticmethod
    def forward(ctx, x, p):
        x, xps = pixel_stride(x)
        N, C, H, W = x.shape
        y = new_act(N, C, H, W, x)
        seed = _seed(x.device)
        call('dmy_dropout', dcode(x), ptr(x), xps, ptr(y), C, N * H * W, C, float(p), ptr(seed), stream())
        ctx.p, ctx.seed = p, seed
        return y

    @staticmethod
    def backward(ctx, dy):
        dy, dps = pixel_stride(dy)
        N, C, H, W = dy.shape
        dx = new_act(N, C, H, W, dy)
        call('dmy_dropout', dcode(dy), ptr(dy), dps, ptr(dx), C, N * H * W, C, float(ctx.p), ptr(ctx.seed), stream())
        return dx, None


def _sample_major(t):
    """a layout in which each sample (dim 0) is one contiguous block: NHWC for 4-D activations, else row-major"""
    return t.contiguous(memory_format=CL) if t.dim() == 4 else t.contiguous()


class SampleScaleFn(torch.autograd.Function):
    """y = x * s[b] (DropPath with a pre-drawn per-sample keep mask, common.py:386-403), any rank."""

    @staticmethod
    def forward(ctx, x, s):
        x = _sample_major(x)
        y = torch.empty_like(x)  # preserve_format: same strides as x
        call('dmy_sample_scale', dcode(x), ptr(x), ptr(s), ptr(y), x.numel() // x.shape[0], x.numel(), stream())
        ctx.save_for_backward(s)
        return y

    @staticmethod
    def backward(ctx, dy):
        (s,) = ctx.saved_tensors
        dy = _sample_major(dy)
        dx = torch.empty_like(dy)
        call('dmy_sample_scale', dcode(dy), ptr(dy), ptr(s), ptr(dx), dy.numel() // dy.shape[0], dy.numel(), stream())
        return dx, None


class DropPathAddFn(torch.autograd.Function):
    """x + DropPath(f) (common.py:386-403 with the residual of common.py:621-627): y = x + f * s[b], s[b] = floor(keep +
    u[b]) / keep on torch's drawn uniforms u [N] (csrc/swin.hip droppath_add_kernel: one pass, one rounding of the sum;
    was dmy_sample_scale + AddFn + torch's floor / div).  Backward: dx = dy (through the residual's GradSink when it
    has one), df = dy * s[b]."""

    @staticmethod
    def forward(ctx, x, f, u, keep, xsink=None):
        x, f = _sample_major(x), _sample_major(f)
        assert x.shape == f.shape and u.numel() == x.shape[0] and u.dtype == torch.float32
        y = torch.empty_like(x)
        call('dmy_droppath_add', dcode(x), ptr(x), ptr(f), ptr(u), float(keep), ptr(y), x.numel() // x.shape[0],
             x.numel(), stream())
        ctx.save_for_backward(u)
        ctx.keep, ctx.xsink = float(keep), xsink
        return y

    @staticmethod
    def backward(ctx, dy):
        (u,) = ctx.saved_tensors
        dy = _sample_major(dy)
        df = torch.empty_like(dy)
        call('dmy_droppath_grad', dcode(dy), ptr(dy), ptr(u), ctx.keep, ptr(df), dy.numel() // dy.shape[0], dy.numel(),
             stream())
        dx = dy if ctx.xsink is None else ctx.xsink.passthrough(dy)
        return dx, df, None, None, None


# ------------------------------------------------------------------ space_to_depth / TDetect flatten

class SpaceToDepthFn(torch.autograd.Function):
    """models/common.py:1451-1458: cat(x[::2, ::2], x[1::2, ::2], x[::2, 1::2], x[1::2, 1::2]) on channels."""

    @staticmethod
    def forward(ctx, x):
        x, xps = pixel_stride(x)
        N, C, H, W = x.shape
        y = new_act(N, 4 * C, H // 2, W // 2, x)
        call('dmy_space_to_depth', dcode(x), ptr(x), xps, ptr(y), 4 * C, N, H, W, C, 0, stream())
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.shape
        dy, dps = pixel_stride(dy)
        dx = new_act(N, C, H, W, dy)
        call('dmy_space_to_depth', dcode(dy), ptr(dx), C, ptr(dy), dps, N, H, W, C, 1, stream())
        return dx


class FlattenLevelsFn(torch.autograd.Function):
    """TDetect (models/detect_t.py:45-47): per-level NHWC head outputs [B, no, H, W] -> one
    anchor-major [B, A, no] tensor (levels in order, anchors row-major within a level)."""

    @staticmethod
    def forward(ctx, *xs):
        B, no = xs[0].shape[:2]
        A = sum(x.shape[2] * x.shape[3] for x in xs)
        F = torch.empty((B, A, no), dtype=xs[0].dtype, device=xs[0].device)
        a0 = 0
        geo = []
        for x in xs:
            x, xps = pixel_stride(x)
            H, W = x.shape[2:]
            call('dmy_tal_flatten', dcode(x), ptr(x), xps, B, H, W, A, a0, no, ptr(F), 0, stream())
            geo.append((H, W, a0))
            a0 += H * W
        ctx.geo, ctx.B, ctx.no, ctx.A = geo, B, no, A
        return F

    @staticmethod
    def backward(ctx, dF):
        dF = dF.contiguous()
        out = []
        for H, W, a0 in ctx.geo:
            dx = new_act(ctx.B, ctx.no, H, W, dF)
            call('dmy_tal_flatten', dcode(dF), ptr(dx), ctx.no, ctx.B, H, W, ctx.A, a0, ctx.no, ptr(dF), 1, stream())
            out.append(dx)
        return tuple(out)


# ------------------------------------------------------------------ CBAM pieces (models/common.py:260-310)

class GPoolFn(torch.autograd.Function):
    """[N,C,H,W] -> [2N,C,1,1]: global average pool rows, then global max pool rows (first max)."""

    @staticmethod
    def forward(ctx, x, sink=None):
        x, xps = pixel_stride(x)
        N, C, H, W = x.shape
        z = new_act(2 * N, C, 1, 1, x)
        arg = torch.empty((N, C), dtype=torch.int32, device=x.device)
        ws = torch.empty(call('dmy_gpool_ws_bytes', dcode(x), N, H * W, C) // 4, dtype=torch.float32, device=x.device)
        call('dmy_gpool_fwd', dcode(x), ptr(x), xps, N, H * W, C, ptr(z), ptr(arg), ptr(ws), stream())
        ctx.save_for_backward(arg)
        ctx.shape, ctx.sink = (N, C, H, W), sink
        return z

    @staticmethod
    def backward(ctx, dz):
        (arg,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        dz = dz.contiguous()
        buf, bps, acc = sink_target(ctx.sink, N, C, H, W, dz)
        call('dmy_gpool_bwd', dcode(dz), ptr(dz), ptr(arg), ptr(buf), bps, acc, N, H * W, C, stream())
        return sink_result(ctx.sink, buf), None


class HalvesSigmoidFn(torch.autograd.Function):
    """[2N,C,1,1] -> [N,C,1,1]: sigmoid(z[:N] + z[N:]) (CBAM channel attention: sigmoid(avgout + maxout))."""

    @staticmethod
    def forward(ctx, z):
        z = z.contiguous()
        N2, C = z.shape[:2]
        ca = torch.empty((N2 // 2, C, 1, 1), dtype=z.dtype, device=z.device)
        call('dmy_halves_sigmoid', dcode(z), ptr(z), N2 // 2, C, ptr(ca), None, None, stream())
        ctx.save_for_backward(z)
        return ca

    @staticmethod
    def backward(ctx, dca):
        (z,) = ctx.saved_tensors
        N2, C = z.shape[:2]
        dca = dca.contiguous()
        dz = torch.empty_like(z)
        call('dmy_halves_sigmoid', dcode(z), ptr(z), N2 // 2, C, None, ptr(dca), ptr(dz), stream())
        return dz


class CBAMInFn(torch.autograd.Function):
    """(x, ca) -> out1 = ca * x and s2 = cat(mean_c out1, max_c out1) (CBAM spatial-attention input)."""

    @staticmethod
    def forward(ctx, x, ca, sink=None):
        x, xps = pixel_stride(x)
        N, C, H, W = x.shape
        ca = ca.contiguous()
        out1 = new_act(N, C, H, W, x)
        s2 = new_act(N, 2, H, W, x)
        am = torch.empty((N, H, W), dtype=torch.int32, device=x.device)
        call('dmy_cbam_in_fwd', dcode(x), ptr(x), xps, ptr(ca), N, H * W, C, ptr(out1), ptr(s2), ptr(am), stream())
        ctx.save_for_backward(x, ca, am)
        ctx.xps, ctx.sink = xps, sink
        return out1, s2

    @staticmethod
    def backward(ctx, dout1, ds2):
        x, ca, am = ctx.saved_tensors
        N, C, H, W = x.shape
        if dout1 is None:
            dout1 = torch.zeros_like(x)
        dout1, dps = pixel_stride(dout1)
        ds2 = torch.zeros((N, 2, H, W), dtype=x.dtype, device=x.device, memory_format=CL) if ds2 is None else \
            ds2.contiguous(memory_format=CL)
        buf, bps, acc = sink_target(ctx.sink, N, C, H, W, x)
        dca = f32(N * C, x.device)
        ws = f32(call('dmy_cbam_in_bwd_ws_elems', N, H * W, C), x.device)  # per-wave partials, folded in order
        call('dmy_cbam_in_bwd', dcode(x), ptr(x), ctx.xps, ptr(ca), ptr(dout1), dps, ptr(ds2), ptr(am), N, H * W, C,
             ptr(buf), bps, acc, ptr(dca), ptr(ws), stream())
        return sink_result(ctx.sink, buf), dca.view(N, C, 1, 1).to(ca.dtype), None


class PixScaleFn(torch.autograd.Function):
    """out = out1 * sa, sa one value per pixel [N,1,H,W] (CBAM: spatial_attention(out) * out)."""

    @staticmethod
    def forward(ctx, out1, sa):
        out1 = out1.contiguous(memory_format=CL)
        sa, sps = pixel_stride(sa)
        N, C, H, W = out1.shape
        out = new_act(N, C, H, W, out1)
        call('dmy_pixscale', dcode(out1), ptr(out1), ptr(sa), sps, N, H * W, C, ptr(out), C, None, 0, None, None,
             stream())
        ctx.save_for_backward(out1, sa)
        ctx.sps = sps
        return out

    @staticmethod
    def backward(ctx, dout):
        out1, sa = ctx.saved_tensors
        N, C, H, W = out1.shape
        dout, dps = pixel_stride(dout)
        dout1 = new_act(N, C, H, W, out1)
        dsa = new_act(N, 1, H, W, out1)
        call('dmy_pixscale', dcode(out1), ptr(out1), ptr(sa), ctx.sps, N, H * W, C, None, 0, ptr(dout), dps,
             ptr(dout1), ptr(dsa), stream())
        return dout1, dsa
