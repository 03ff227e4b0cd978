"""Fused multi-tensor optimizers and EMA on gfx950 (csrc/optim.hip).

FusedSGD / FusedAdam are torch.optim.Optimizer subclasses (so LambdaLR, param_groups, warmup
writes to group['lr'] / group['momentum'] work exactly as in train.py:216-235, 408-422); each
step() is one kernel launch per parameter group.  Semantics follow torch.optim.SGD(nesterov=True)
and torch.optim.Adam (L2 weight decay, bias correction) as used by the reference.
"""
import ctypes

import torch

from ._lib import lib, stream, call
from .functional import PARAM_GEN

lib.dmy_chunk_size.restype = ctypes.c_int
lib.dmy_chunk_size.argtypes = []
CHUNK = lib.dmy_chunk_size()
_P, _I, _F, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_long
lib.dmy_sgd.argtypes = [_P, _P, _P, _P, _P, _P, _I, _F, _F, _F, _I, _P, _P, _P]
lib.dmy_adam.argtypes = [_P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _F, _F, _F, _F, _F, _P, _P, _P, _P]
lib.dmy_ema.argtypes = [_P, _P, _P, _P, _P, _I, _F, _P]
lib.dmy_amp_check.argtypes = [_P, _P, _P, _P, _I, _P, _P, _P]
lib.dmy_amp_update.argtypes = [_P, _P, _P, _P, _F, _F, _F, _I, _P]
for _f in (lib.dmy_sgd, lib.dmy_adam, lib.dmy_ema, lib.dmy_amp_check, lib.dmy_amp_update):
    _f.restype = ctypes.c_int


class _Table:
    """Device-side pointer table + (tensor, chunk) map for a list of tensors.

    One table per tensor LIST (keyed by the identity of its first list -- the parameters -- and the sizes), kept for
    the run.  With the caching allocator the gradients of a parameter list usually land at the same addresses every
    step; when they do not (gradients autograd assembles from slices, e.g. nn.MultiheadAttention's in_proj_weight in
    config 5's C3TR) only the changed pointer arrays are rewritten in place -- round 4 cached a NEW table per pointer
    set, so those models built and kept (up to 64) tables, ~190 KB of device memory a step.  A table is staged in
    pinned host memory and copied asynchronously, stream-ordered behind the kernels that read the old pointers (a
    pageable H2D copy would block the host until the GPU drained its queue); before its pinned buffer is rewritten
    the previous copy's event is waited on (long complete by then)."""
    _cache = {}

    def __init__(self, lists, dev):
        n = [t.numel() for t in lists[0]]
        tid, off = [], []
        for i, k in enumerate(n):
            for o in range(0, k, CHUNK):
                tid.append(i)
                off.append(o)
        self.nchunks = len(tid)
        self.ptrs = [tuple(t.data_ptr() for t in L) for L in lists]
        host = [torch.tensor(list(pl), dtype=torch.int64) for pl in self.ptrs]
        host += [torch.tensor(n, dtype=torch.int64), torch.tensor(tid, dtype=torch.int32),
                 torch.tensor(off, dtype=torch.int64)]
        self.pinned = [h.pin_memory() for h in host]  # kept alive with the cached table
        self.dev = [h.to(dev, non_blocking=True) for h in self.pinned]
        self.ev = torch.cuda.Event() if torch.device(dev).type == 'cuda' else None
        if self.ev is not None:
            self.ev.record()

    def refresh(self, lists):
        for i, L in enumerate(lists):
            pl = tuple(t.data_ptr() for t in L)
            if pl == self.ptrs[i]:
                continue
            if self.ev is not None:
                self.ev.synchronize()  # the previous async copy out of this pinned buffer has finished
            self.pinned[i].copy_(torch.tensor(list(pl), dtype=torch.int64))
            self.dev[i].copy_(self.pinned[i], non_blocking=True)
            self.ptrs[i] = pl
            if self.ev is not None:
                self.ev.record()

    @classmethod
    def get(cls, lists, dev, ident=None):
        """ident: the tensors whose identity names the table (default lists[0])"""
        ident = lists[0] if ident is None else ident
        key = (str(dev), len(lists), tuple(id(t) for t in ident), tuple(t.numel() for t in lists[0]))
        tb = cls._cache.get(key)
        if tb is None:
            if len(cls._cache) > 256:
                cls._cache.clear()
            tb = cls._cache[key] = cls(lists, dev)
        else:
            tb.refresh(lists)
        return tb

    def p(self, i):
        return ctypes.c_void_p(self.dev[i].data_ptr())


def _check(rc, name):
    if rc != 0:
        raise RuntimeError(f'{name} failed with hipError {rc}')


def _amp_ptrs(opt):
    """(scale, found) device pointers while a GradScaler.step() runs this optimizer, else (None, None)"""
    amp = getattr(opt, '_amp', None)
    return (None, None) if amp is None else (ctypes.c_void_p(amp[0].data_ptr()), ctypes.c_void_p(amp[1].data_ptr()))


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params, lr=0.01, momentum=0.0, weight_decay=0.0, nesterov=False):
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, nesterov=nesterov))

    @torch.no_grad()
    def step(self, closure=None):
        for g in self.param_groups:
            ps = [p for p in g['params'] if p.grad is not None]
            if not ps:
                continue
            for p in ps:
                assert p.dtype == torch.float32 and p.is_contiguous() and p.grad.is_contiguous()
            bufs = []
            for p in ps:
                st = self.state[p]
                if 'momentum_buffer' not in st:  # per parameter: a grad that first appears later starts at zero
                    st['momentum_buffer'] = torch.zeros_like(p)
                bufs.append(st['momentum_buffer'])
            tb = _Table.get([ps, [p.grad for p in ps], bufs], ps[0].device)
            PARAM_GEN[0] += 1
            _check(lib.dmy_sgd(tb.p(0), tb.p(1), tb.p(2), tb.p(3), tb.p(4), tb.p(5), tb.nchunks, float(g['lr']),
                               float(g['momentum']), float(g['weight_decay']), int(g['nesterov']), *_amp_ptrs(self),
                               stream()), 'dmy_sgd')
        return None


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam semantics with the step count on the device.  The count is a per-parameter quantity in torch
    (a parameter whose gradient first appears later starts at t = 0); here parameters that started together share one
    device int32 counter (a cohort), and each cohort of a group is one kernel launch -- normally one per group.  The
    counters live in the optimizer (not in param_groups / state), and state_dict() stores torch's format: a float32
    CPU 'step' per parameter, from which load_state_dict + the next step() rebuild the counters on the parameters'
    device (a checkpoint loaded with map_location='cpu' works).  A member that has no gradient in some step leaves
    its cohort on a copy of the counter, so its count stops as torch's would."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._ctr = {}  # id(param) -> its cohort's device int32 counter

    def _counter(self, p, fresh):
        """the device counter of parameter p; `fresh` (t0, device) -> counter shares new counters per start count"""
        c = self._ctr.get(id(p))
        if c is not None and c.device == p.device:
            return c
        st = self.state[p]
        s = st.get('step')
        t0 = int(float(c.item() if c is not None else s.item() if torch.is_tensor(s) else s)) \
            if (c is not None or s is not None) else 0
        key = (t0, p.device)
        if key not in fresh:
            fresh[key] = torch.full((1,), t0, dtype=torch.int32, device=p.device)
        c = self._ctr[id(p)] = fresh[key]
        return c

    @torch.no_grad()
    def step(self, closure=None):
        for g in self.param_groups:
            ps = [p for p in g['params'] if p.grad is not None]
            if not ps:
                continue
            fresh, cohorts = {}, {}
            for p in ps:
                st = self.state[p]
                if 'exp_avg' not in st:
                    st['exp_avg'] = torch.zeros_like(p)
                    st['exp_avg_sq'] = torch.zeros_like(p)
                c = self._counter(p, fresh)
                st['step'] = c  # torch keeps Adam's step as a tensor too; read it (host sync) only to log / save
                cohorts.setdefault(id(c), (c, []))[1].append(p)
            # a cohort member without a gradient this step must keep its count (torch leaves its 'step' alone): it
            # leaves the cohort on a copy of the counter taken before the launch advances it
            for q in g['params']:
                cq = self._ctr.get(id(q)) if q.grad is None else None
                if cq is not None and id(cq) in cohorts:
                    self._ctr[id(q)] = self.state[q]['step'] = cq.clone()
            b1, b2 = g['betas']
            PARAM_GEN[0] += 1
            for c, cp in cohorts.values():
                st = [self.state[p] for p in cp]
                tb = _Table.get([cp, [p.grad for p in cp], [s['exp_avg'] for s in st], [s['exp_avg_sq'] for s in st]],
                                cp[0].device)
                # bias corrections from the device count (t = count + 1), which the kernel advances unless the
                # GradScaler found a non-finite gradient: a skipped step leaves t alone, as torch (scaler.step skips
                # optimizer.step)
                _check(lib.dmy_adam(tb.p(0), tb.p(1), tb.p(2), tb.p(3), tb.p(4), tb.p(5), tb.p(6), tb.nchunks,
                                    float(g['lr']), float(b1), float(b2), float(g['eps']), float(g['weight_decay']),
                                    0.0, 0.0, *_amp_ptrs(self), ctypes.c_void_p(c.data_ptr()), stream()), 'dmy_adam')
        return None

    def state_dict(self):
        sd = super().state_dict()
        order = [p for g in self.param_groups for p in g['params']]
        for i, p in enumerate(order):
            ent = sd['state'].get(i)
            if ent is not None and torch.is_tensor(ent.get('step')):
                ent = sd['state'][i] = dict(ent)
                ent['step'] = torch.tensor(float(ent['step'].item()), dtype=torch.float32)  # torch Adam's format
        for g in sd['param_groups']:
            g.pop('_dstep', None)
        return sd

    def load_state_dict(self, state_dict):
        for g in state_dict.get('param_groups', []):
            g.pop('_dstep', None)  # checkpoints of the earlier format kept the counter in the group
        super().load_state_dict(state_dict)
        self._ctr = {}  # rebuilt from state['step'] on the parameters' device at the next step()


class GradScaler:
    """torch.amp.GradScaler as train.py uses it (train.py:354 GradScaler(enabled=cuda); 445 scale(loss).backward();
    449-450 step / update) with its state on the device: loss scale (init 2**16, growth 2 every 2000 clean steps,
    backoff 0.5), growth tracker and the non-finite flag.  step() runs one check kernel over every gradient, then
    the optimizer kernels unscale on the fly and skip themselves when a gradient was non-finite -- no host sync.
    `upstream` is the loss's backward seed: scale * world (loss *= WORLD_SIZE, train.py:438-440, folded in).
    Disabled: upstream = world, step() = optimizer.step().  Unlike torch, the .grad tensors keep the scaled
    values after step() (unscaling is fused into the update)."""

    def __init__(self, device, enabled=True, world=1, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5,
                 growth_interval=2000):
        self.enabled, self.world = enabled, float(world)
        self.growth, self.backoff, self.interval = growth_factor, backoff_factor, growth_interval
        s = init_scale if enabled else 1.0
        self.scale = torch.full((1,), s, dtype=torch.float32, device=device)
        self.upstream = torch.full((1,), s * world, dtype=torch.float32, device=device)
        self.tracker = torch.zeros(1, dtype=torch.int32, device=device)
        self.found = torch.zeros(1, dtype=torch.float32, device=device)

    def step(self, optimizer):
        if not self.enabled:
            return optimizer.step()
        ps = [p for g in optimizer.param_groups for p in g['params'] if p.grad is not None]
        gs = [p.grad for p in ps]
        if gs:
            tb = _Table.get([gs], gs[0].device, ident=ps)
            _check(lib.dmy_amp_check(tb.p(0), tb.p(1), tb.p(2), tb.p(3), tb.nchunks, ctypes.c_void_p(self.scale.data_ptr()),
                                     ctypes.c_void_p(self.found.data_ptr()), stream()), 'dmy_amp_check')
        optimizer._amp = (self.scale, self.found)
        try:
            return optimizer.step()
        finally:
            optimizer._amp = None

    def update(self):
        if self.enabled:
            P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
            _check(lib.dmy_amp_update(P(self.scale), P(self.upstream), P(self.tracker), P(self.found), self.world,
                                      self.growth, self.backoff, self.interval, stream()), 'dmy_amp_update')

    def get_scale(self):
        return float(self.scale)  # host sync: logging only


def ema_update(ema_tensors, model_tensors, d):
    """e = d*e + (1-d)*m for every float tensor pair (utils/torch_utils.py:335-339)."""
    es = [e for e in ema_tensors]
    ms = [m.float() if m.dtype != torch.float32 else m for m in model_tensors]
    for e in es:
        assert e.dtype == torch.float32 and e.is_contiguous()
    tb = _Table.get([es, [m.contiguous() for m in ms]], es[0].device)
    _check(lib.dmy_ema(tb.p(0), tb.p(1), tb.p(2), tb.p(3), tb.p(4), tb.nchunks, float(d), stream()), 'dmy_ema')


def param_groups(model):
    """train.py:197-214 grouping: g0 BN weights (no decay), g1 weights + AdConcat.w (decay), g2 biases.
    (relative_position_bias_table and other non-weight/bias params are NOT collected, as in the reference.)"""
    import torch.nn as nn
    from .models.common import AdConcat2, AdConcat3
    g0, g1, g2 = [], [], []
    for v in model.modules():
        if hasattr(v, 'bias') and isinstance(v.bias, nn.Parameter):
            g2.append(v.bias)
        if isinstance(v, nn.BatchNorm2d):
            g0.append(v.weight)
        elif hasattr(v, 'weight') and isinstance(v.weight, nn.Parameter):
            g1.append(v.weight)
        elif isinstance(v, (AdConcat2, AdConcat3)) and isinstance(v.w, nn.Parameter):
            g1.append(v.w)
    return g0, g1, g2


def build_optimizer(model, kind='sgd', lr0=0.01, momentum=0.937, weight_decay=5e-4):
    """train.py:216-222 (Adam hard-codes lr=3e-4 for g0)."""
    g0, g1, g2 = param_groups(model)
    if kind == 'adam':
        opt = FusedAdam(g0, lr=3e-4, betas=(momentum, 0.999))
    else:
        opt = FusedSGD(g0, lr=lr0, momentum=momentum, nesterov=True)
    opt.add_param_group({'params': g1, 'weight_decay': weight_decay})
    opt.add_param_group({'params': g2})
    return opt
