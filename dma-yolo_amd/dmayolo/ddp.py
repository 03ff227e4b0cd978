"""Data-parallel gradient exchange over the weight-gradient arena (reference train.py:322-326, 438-440).

The reference wraps the model in torch DistributedDataParallel: its reducer copies every parameter gradient into
25 MB buckets, all-reduces (averages) the buckets while backward still runs, and copies the result back.  The product
already writes every conv / BN gradient straight into ONE fp32 buffer per training forward (functional.WgradArena,
parameter order), so here the buckets ARE contiguous slices of that buffer and nothing is copied:

  * buckets: contiguous arena ranges taken from the END of the arena (backward produces the last layers' gradients
    first), a small first bucket (`first_bucket_mb`) so the first collective starts early, then `bucket_cap_mb` each;
  * a post-accumulate-grad hook per parameter marks it ready; when every parameter of a bucket is ready -- and every
    earlier bucket has been launched (collectives must be issued in the same order on every rank) -- the bucket's
    slice is all-reduced with ReduceOp.AVG, asynchronously: RCCL runs on its own stream, overlapped with the rest of
    the backward;
  * a callback queued on the autograd engine runs at the end of backward: it launches what is left (in order) and
    makes the current stream wait for the collectives (no host synchronisation with RCCL);
  * a gradient that did not land in the arena (kernels that allocate their own, or the accumulated gradient of an
    earlier step, train.py's `accumulate`) is copied into its slice first, and the parameter's .grad becomes the
    slice, so after backward every .grad is a view of the arena holding the rank average, as DDP leaves it;
  * `compress='bf16'` (optional, off by default): a bucket is divided by the world size in fp32, sent as bf16 and
    copied back -- DDP's bf16_compress_hook; halves the bytes on the xGMI links, at bf16 precision of the gradient;
  * buffers (BN running statistics) are broadcast from rank 0 before each forward and the initial state once at
    construction, as DDP's defaults (broadcast_buffers=True).

A parameter that gets no gradient on this rank still has its (zeroed) slice reduced with the rest, and after backward
its .grad is that slice -- the rank average -- as torch DDP writes the reduced gradient into locally unused
parameters, so replicas cannot diverge.  A parameter that NO rank used is told apart only with
`find_unused_parameters=True` (train.py:326 sets it when the model holds nn.MultiheadAttention): every rank then
all-reduces a used-flag vector after the buckets and reads it back (one host synchronisation per backward, as DDP's own
find-unused mode), and a globally unused parameter keeps the .grad it had (None after zero_grad), so SGD's weight decay
and momentum, and Adam's step count, do not advance for it.  Without the flag the graph is assumed static, as DDP does
without it, and such a parameter gets a zero gradient.  The hooks act only for a backward this wrapper armed (a
training forward through it); `close()` removes them, and a model may be wrapped again after that.  The loss *
WORLD_SIZE of train.py:440 stays in the backward seed (GradScaler.upstream), so the averaged gradient is the sum over
ranks, exactly as with DDP.
"""
import torch
import torch.distributed as dist

ALIGN = 64  # elements; the same layout rule as functional.WgradArena.layout


def arena_layout(params):
    """id(param) -> (offset, numel) over the fp32 parameters that require a gradient, in order; total size"""
    offs, n = {}, 0
    for q in params:
        if q.dim() >= 1 and q.dtype == torch.float32 and q.requires_grad:
            offs[id(q)] = (n, q.numel())
            n += -(-q.numel() // ALIGN) * ALIGN
    return offs, n


class _Backward:
    __slots__ = ('buf', 'pending', 'ready', 'next', 'works', 'seen')

    def __init__(self, buf, counts):
        self.buf, self.pending = buf, list(counts)
        self.ready, self.next, self.works, self.seen = [False] * len(counts), 0, [], set()


class ArenaDDP(torch.nn.Module):
    def __init__(self, module, process_group=None, bucket_cap_mb=32.0, first_bucket_mb=4.0, compress=None,
                 broadcast_buffers=True, find_unused_parameters=False):
        super().__init__()
        assert compress in (None, 'bf16'), compress
        self.module, self.pg, self.compress, self.broadcast_buffers = module, process_group, compress, broadcast_buffers
        self.find_unused = bool(find_unused_parameters)
        self.world = dist.get_world_size(process_group)
        self.params = [p for p in module.parameters() if p.requires_grad]
        all_params = list(module.parameters())
        self.offs, self.n = arena_layout(all_params)
        self.reduced = [p for p in all_params if id(p) in self.offs]
        # buckets from the end of the arena (reverse parameter order ~ backward order)
        order = sorted(self.reduced, key=lambda p: -self.offs[id(p)][0])
        self.buckets, self.bucket_of, cur, hi, cap = [], {}, [], None, first_bucket_mb
        for p in order:
            o, k = self.offs[id(p)]
            if hi is None:
                hi = o + -(-k // ALIGN) * ALIGN
            cur.append(p)
            if (hi - o) * 4 >= cap * 2 ** 20:
                self.buckets.append((o, hi, cur))
                cur, hi, cap = [], None, bucket_cap_mb
        if cur:
            self.buckets.append((self.offs[id(cur[-1])][0], hi, cur))
        for b, (_, _, ps) in enumerate(self.buckets):
            for p in ps:
                self.bucket_of[id(p)] = b
        self._bw = None
        self._buf = None
        self._handles = []
        self.trace = None  # a list to record ('hook', name) / ('launch', bucket) events in order (tests: overlap)
        with torch.no_grad():
            state = [t for t in module.state_dict().values() if torch.is_tensor(t)]
            if state:
                dist._broadcast_coalesced(self._group(), state, 250 * 2 ** 20, 0)
        self._owner = object()  # identity token: a flag on a parameter names the wrapper that set it
        for p in self.reduced:
            if getattr(p, '_dmy_arena_ddp', None) is not None:
                self.close()  # release only the flags this wrapper set so far
                raise RuntimeError('ArenaDDP: a parameter is already hooked by another live wrapper; close() it first')
            p._dmy_arena_ddp = self._owner
            self._handles.append(p.register_post_accumulate_grad_hook(self._hook))

    def close(self):
        """remove the gradient hooks (the model can then be used unwrapped, or wrapped again); a flag another live
        wrapper set on a parameter is left alone, e.g. when an old wrapper is garbage-collected after a new one"""
        for h in self._handles:
            h.remove()
        self._handles = []
        owner = getattr(self, '_owner', None)
        for p in getattr(self, 'reduced', ()):
            if owner is not None and getattr(p, '_dmy_arena_ddp', None) is owner:
                p._dmy_arena_ddp = None
        self._bw = self._buf = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _group(self):
        return self.pg if self.pg is not None else dist.group.WORLD

    def bucket_sizes_mb(self):
        return [round((hi - lo) * 4 / 2 ** 20, 2) for lo, hi, _ in self.buckets]

    # ------------------------------------------------------------------ forward
    def forward(self, *args, **kw):
        if self.broadcast_buffers and self.world > 1:
            bufs = [b for b in self.module.buffers()]
            if bufs:
                with torch.no_grad():
                    dist._broadcast_coalesced(self._group(), bufs, 250 * 2 ** 20, 0)
        out = self.module(*args, **kw)
        ref = getattr(self.module, '_last_arena', None)
        arena = ref() if ref is not None else None
        if arena is not None and arena.buf.numel() == self.n and torch.is_grad_enabled() and self.module.training:
            self._buf = arena.buf  # the conv kernels' gradient arena of THIS forward: buckets are its slices
        elif torch.is_grad_enabled():
            dev = self.reduced[0].device if self.reduced else 'cpu'
            self._buf = torch.zeros(self.n, dtype=torch.float32, device=dev)
        return out

    # ------------------------------------------------------------------ backward
    def _slice(self, buf, p):
        o, k = self.offs[id(p)]
        return buf[o:o + k].view_as(p)

    def _begin(self):
        self._bw = _Backward(self._buf, [len(ps) for _, _, ps in self.buckets])
        self._buf = None
        torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        return self._bw

    def _hook(self, p):
        if self._bw is None and self._buf is None:
            return  # a backward this wrapper did not arm (e.g. through de_parallel(model) under no wrapper forward)
        bw = self._bw if self._bw is not None else self._begin()
        sl = self._slice(bw.buf, p)
        if p.grad is not None and p.grad.data_ptr() != sl.data_ptr():
            sl.copy_(p.grad)  # a gradient allocated outside the arena, or accumulated into an earlier step's arena
            p.grad = sl
        if id(p) in bw.seen:  # a parameter used twice accumulates once more: its slice already holds the total
            return
        bw.seen.add(id(p))
        if self.trace is not None:
            self.trace.append(('hook', id(p)))
        b = self.bucket_of[id(p)]
        bw.pending[b] -= 1
        if bw.pending[b] == 0:
            bw.ready[b] = True
            self._launch(bw, upto=None)

    def _launch(self, bw, upto):
        """issue the collectives of every bucket that is ready (all, when upto == 'all') in bucket order"""
        while bw.next < len(self.buckets) and (upto == 'all' or bw.ready[bw.next]):
            lo, hi, _ = self.buckets[bw.next]
            view = bw.buf[lo:hi]
            if self.trace is not None:
                self.trace.append(('launch' if upto is None else 'launch_final', bw.next))
            # no world-size-1 shortcut: a one-rank group issues its collectives as well, so the RCCL stream
            # semantics (async all_reduce, work.wait() making the current stream wait) run on one GPU too
            if self.compress == 'bf16':
                c = (view / self.world).to(torch.bfloat16)
                bw.works.append((dist.all_reduce(c, op=dist.ReduceOp.SUM, group=self.pg, async_op=True), c, view))
            else:
                bw.works.append((dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.pg, async_op=True), None, view))
            bw.next += 1

    def _finalize(self):
        bw, self._bw = self._bw, None
        if bw is None:
            return
        self._launch(bw, upto='all')
        for work, c, view in bw.works:
            if work is not None:
                work.wait()  # RCCL: the current stream waits on the collective's stream (no host sync)
            if c is not None:
                view.copy_(c)
        unused = [i for i, p in enumerate(self.reduced) if id(p) not in bw.seen]
        if self.find_unused:
            # which parameters some rank used: a MAX over the ranks' used flags, read on the host (DDP's find-unused
            # mode synchronises the same way); every rank issues it, whether or not it has locally unused parameters
            flags = torch.ones(len(self.reduced), dtype=torch.int32)
            flags[unused] = 0
            flags = flags.to(bw.buf.device)
            dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=self.pg)
            used = flags.cpu()
            unused = [i for i in unused if used[i] != 0]
        for i in unused:  # no gradient on this rank but on some other: it gets the rank average (DDP semantics)
            p = self.reduced[i]
            p.grad = self._slice(bw.buf, p)
