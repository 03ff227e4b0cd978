"""CPU, world_size 2 over gloo: the data-parallel step of dmayolo.trainer.Trainer (train.py:400-454 + DDP at
train.py:326) shards images by rank and applies the SUM of the per-rank gradients (the backward is seeded with
WORLD_SIZE, train.py:440, and DDP averages).  The model here is the CPU oracle, stepped the way Trainer.step does
(loss.backward(upstream = scale * WORLD_SIZE), scale 1 without a GPU); the product Model / ComputeLoss / FusedSGD
under DDP is the GPU test tests/test_gpu_ddp.py (two gloo ranks on cuda:0)."""
import os
import socket
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs', 'yolov5n.yaml')
IMG, BS, NC = 64, 2, 10


def _setup():
    for p in (ROOT, os.path.join(ROOT, 'dma-yolo_amd')):
        if p not in sys.path:
            sys.path.insert(0, p)


def _model():
    from oracle import nn as onn
    torch.manual_seed(0)
    with open(CFG) as f:
        d = yaml.safe_load(f)
    return onn.bn_defaults(onn.Model(d, nc=NC)).train()


def _loss_fn(model):
    from oracle.loss import compute_loss
    from dmayolo.synthetic import HYP_SCRATCH, scaled_hyp
    det = model.model[-1]
    anchors = det.anchors / det.stride.view(-1, 1, 1)
    hyp = scaled_hyp(HYP_SCRATCH, NC, IMG)
    return lambda p, t: compute_loss(p, t, anchors, hyp, NC)


def _batch(rank):
    from dmayolo.synthetic import images, targets
    return images(BS, IMG, seed=1 + rank).float() / 255, targets(BS, NC, per_image=6, seed=1 + rank)


def _worker(rank, world, port, out):
    _setup()
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    model = _model()
    net = torch.nn.parallel.DistributedDataParallel(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, nesterov=True)
    x, t = _batch(rank)
    loss, _ = _loss_fn(model)(net(x), t)
    loss.backward(torch.full((1,), float(world)))  # Trainer.step: GradScaler.upstream = scale * WORLD_SIZE
    opt.step()
    assert torch.isfinite(loss).all()
    if rank == 0:
        torch.save({k: v.detach().clone() for k, v in model.state_dict().items()}, out)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_ddp_world2_applies_sum_of_rank_gradients():
    _setup()
    world = 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, 'rank0.pt')
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        got = torch.load(out, weights_only=True)
    # expected: one process, per-shard forward (BN batch stats per rank, no SyncBN), grads summed
    model = _model()
    lf = _loss_fn(model)
    grads = None
    for r in range(world):
        x, t = _batch(r)
        model.zero_grad(set_to_none=True)
        loss, _ = lf(model(x), t)
        loss.backward()
        g = [p.grad.clone() for p in model.parameters()]
        grads = g if grads is None else [a + b for a, b in zip(grads, g)]
    ref = _model()
    opt = torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9, nesterov=True)
    for p, g in zip(ref.parameters(), grads):
        p.grad = g
    opt.step()
    exp = dict(ref.named_parameters())
    n = 0
    for k, v in got.items():
        if k in exp:
            torch.testing.assert_close(v, exp[k].detach(), rtol=1e-4, atol=1e-6)
            n += 1
    assert n == len(exp)


def _arena_worker(rank, world, port, out, compress):
    _setup()
    from dmayolo.ddp import ArenaDDP
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    model = _model()
    if rank == 1:  # the wrapper broadcasts rank 0's initial state, as DDP does
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    net = ArenaDDP(model, bucket_cap_mb=0.25, first_bucket_mb=0.05, compress=compress)
    assert len(net.buckets) > 3, net.bucket_sizes_mb()  # several buckets, so the in-order launch logic is exercised
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, nesterov=True)
    x, t = _batch(rank)
    loss, _ = _loss_fn(model)(net(x), t)
    loss.backward(torch.full((1,), float(world)))
    # every gradient is a view of the wrapper's flat buffer afterwards, identical on both ranks
    assert all(p.grad is not None for p in model.parameters())
    flat = torch.cat([p.grad.flatten() for p in model.parameters()])
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.equal(flat, other)
    opt.step()
    if rank == 0:
        torch.save({k: v.detach().clone() for k, v in model.state_dict().items()}, out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('compress', [None, 'bf16'])
def test_arena_reducer_world2_matches_ddp_sum(compress):
    """dmayolo.ddp.ArenaDDP (bucketed AVG all-reduce of arena slices from post-accumulate hooks, in bucket order,
    optional bf16 compression) on the CPU oracle model over gloo: the step equals the one that applies the sum of the
    two ranks' gradients (rtol 1e-4; bf16 compression: the step delta within bf16 precision)"""
    _setup()
    world = 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, 'rank0.pt')
        mp.spawn(_arena_worker, args=(world, _free_port(), out, compress), nprocs=world, join=True)
        got = torch.load(out, weights_only=True)
    model = _model()
    init = {k: v.detach().clone() for k, v in model.named_parameters()}
    lf = _loss_fn(model)
    for r in range(world):
        x, t = _batch(r)
        loss, _ = lf(model(x), t)
        loss.backward()
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, nesterov=True)
    opt.step()
    dmax = max(float((v.detach() - init[k]).norm()) for k, v in model.named_parameters())
    for k, v in model.named_parameters():
        if compress is None:
            torch.testing.assert_close(got[k], v.detach(), rtol=1e-4, atol=1e-6)
        else:
            de, dg = v.detach() - init[k], got[k] - init[k]
            # bf16 carries ~3 significant digits of each rank's half; floor for the near-cancelling BN sums
            assert float((dg - de).norm()) <= 1e-2 * max(float(de.norm()), 1e-2 * dmax), k


def _overlap_worker(rank, world, port, out):
    """the first bucket's collective is issued from a gradient hook while backward still runs (before the last
    parameter's hook), i.e. communication overlaps the rest of backward (train.py:322-326 DDP behaviour)"""
    _setup()
    from dmayolo.ddp import ArenaDDP
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    model = _model()
    net = ArenaDDP(model, bucket_cap_mb=0.25, first_bucket_mb=0.05)
    net.trace = []
    x, t = _batch(rank)
    loss, _ = _loss_fn(model)(net(x), t)
    loss.backward()
    kinds = [k for k, _ in net.trace]
    last_hook = max(i for i, k in enumerate(kinds) if k == 'hook')
    first_launch = kinds.index('launch')
    early = sum(1 for i, k in enumerate(kinds) if k == 'launch' and i < last_hook)
    buckets = [b for k, b in net.trace if k.startswith('launch')]
    if rank == 0:
        torch.save(dict(first_launch=first_launch, last_hook=last_hook, early=early, n=len(net.buckets),
                        order=buckets), out)
    dist.barrier()
    dist.destroy_process_group()


def test_arena_reducer_overlaps_backward():
    _setup()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, 'r.pt')
        mp.spawn(_overlap_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        r = torch.load(out, weights_only=True)
    assert r['first_launch'] < r['last_hook'], r
    assert r['early'] >= r['n'] // 2, r  # most buckets go out before backward ends
    assert r['order'] == list(range(r['n'])), r  # every bucket once, in bucket order


class _Branchy(torch.nn.Module):
    """a parameter (`b`) that only rank 0 uses, and one (`c`) that no rank uses"""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = torch.nn.Linear(8, 8)
        self.b = torch.nn.Linear(8, 8)
        self.c = torch.nn.Linear(8, 8)

    def forward(self, x, use_b):
        y = self.a(x)
        return self.b(y) if use_b else y


def _unused_worker(rank, world, port, out):
    _setup()
    from dmayolo.ddp import ArenaDDP
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    m = _Branchy()
    net = ArenaDDP(m, first_bucket_mb=1e-4, bucket_cap_mb=1e-4, find_unused_parameters=True)
    x = torch.randn(4, 8, generator=torch.Generator().manual_seed(rank))
    net(x, use_b=rank == 0).square().sum().backward()
    g = {k: (None if p.grad is None else p.grad.clone()) for k, p in m.named_parameters()}
    # the wrapper's hooks act only for backward passes it armed; close() removes them and the model can be wrapped
    # again: a backward through the bare model, then a second wrapper
    m.zero_grad(set_to_none=True)
    m(x, True).sum().backward()
    net.close()
    m.zero_grad(set_to_none=True)
    net2 = ArenaDDP(m, first_bucket_mb=1e-4, bucket_cap_mb=1e-4)
    net2(x, use_b=rank == 0).square().sum().backward()
    g2 = {k: p.grad.clone() for k, p in m.named_parameters()}
    # a wrapper garbage-collected after a new one wraps the model must not clear the live wrapper's flags
    net2.close()
    net3 = ArenaDDP(m, first_bucket_mb=1e-4, bucket_cap_mb=1e-4)
    del net2
    import gc
    gc.collect()
    try:
        ArenaDDP(m)
        double = True
    except RuntimeError:
        double = False
    net3.close()
    torch.save(dict(g=g, g2=g2, double=double), out + f'.{rank}')
    dist.barrier()
    dist.destroy_process_group()


def test_arena_reducer_unused_parameter_and_rewrap():
    """a parameter with a gradient on rank 0 only gets the rank average on BOTH ranks (torch DDP writes the reduced
    gradient into locally unused parameters); with find_unused_parameters=True a parameter NO rank used keeps
    .grad None (so the optimizer leaves it alone), without it (static graph) it gets zeros; wrapping a model twice
    works after close(), and an old wrapper's garbage collection leaves a live wrapper's guard in place"""
    _setup()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, 'r.pt')
        mp.spawn(_unused_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        r = [torch.load(out + f'.{k}', weights_only=True) for k in range(2)]
    exp = {}
    for rank in range(2):
        m = _Branchy()
        x = torch.randn(4, 8, generator=torch.Generator().manual_seed(rank))
        m(x, rank == 0).square().sum().backward()
        for k, p in m.named_parameters():
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            exp[k] = exp.get(k, 0) + g / 2
    for key in ('g', 'g2'):
        for k in exp:
            if key == 'g' and k.startswith('c.'):  # globally unused, find_unused_parameters=True: untouched
                assert r[0][key][k] is None and r[1][key][k] is None, k
                continue
            torch.testing.assert_close(r[0][key][k], exp[k], rtol=1e-5, atol=1e-7)
            assert torch.equal(r[0][key][k], r[1][key][k]), (key, k)
    assert not r[0]['double'] and not r[1]['double']
