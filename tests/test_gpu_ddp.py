"""GPU, world_size 2: the PRODUCT training step (Model / ComputeLoss / FusedSGD / GradScaler through
dmayolo.trainer.Trainer) under torch DistributedDataParallel (train.py:322-326; loss * WORLD_SIZE, train.py:438-440) with
two gloo ranks sharing cuda:0, against one process that accumulates the two ranks' batches' gradients and takes the
same optimizer step.  This is the path bench.py runs over RCCL at N > 1 (the collective here is gloo because both
ranks sit on one GPU).

Topologies (BASELINE.json configs 4 and 5 at test size, fp32 storage, deterministic mode so the only difference
between the two runs is the gradient all-reduce's summation):
  * yolov5n @128 (Conv / C3 / SPPF / Detect);
  * the DMA-YOLO-l topology (the width-0.125 derivation of yolov5l-ca-sppfcspc-bifpn-scconv.yaml that
    tests/golden/model_dma.npz pins): SCConv, C3STR / Swin (relative-position table, shift mask), CA, SPPFCSPC, the
    trainable AdConcat2/3 weights, the BiFPN skips;
  * the config-5 topology (yolov5l-xs-tr-cbam-spp-bifpn.yaml derivation of model_c5.npz): C3TR's
    nn.MultiheadAttention, so DDP runs with find_unused_parameters=True exactly as train.py:326 decides, CBAM, SPP,
    4 Detect levels.
Checked: every parameter after the step (rtol 1e-4) and, more sharply, every parameter's step delta
(p_after - p_before) against the single-process delta: relative L2 per tensor <= 2e-3 (floor: 1e-3 of the largest
delta norm, for the exactly-zero gradients of biases feeding a train-mode BN, which are pure rounding noise)."""
import os
import socket
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFGDIR = os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs')
BS, NI = 2, 500  # NI: integrated batch index (mid-warmup: every group has a non-zero lr)


def _setup():
    for p in (ROOT, os.path.join(ROOT, 'dma-yolo_amd'), os.path.join(ROOT, 'tests')):
        if p not in sys.path:
            sys.path.insert(0, p)


def _cfg(topology):
    _setup()
    if topology == 'yolov5n':
        return os.path.join(CFGDIR, 'yolov5n.yaml'), 10, 128
    from golden_util import Fixture
    fx = Fixture({'dma': 'model_dma', 'c5': 'model_c5'}[topology])
    return fx.meta['yaml'], 10, 128


def _model(topology):
    from dmayolo.models.yolo import Model
    from dmayolo.synthetic import HYP_SCRATCH, scaled_hyp
    cfg, nc, img = _cfg(topology)
    torch.manual_seed(0)
    m = Model(cfg, nc=nc, act_dtype=torch.float32)
    for mod in m.modules():
        if type(mod).__name__ == 'SwinTransformerLayer':
            mod.drop_path = torch.nn.Identity()  # DropPath / dropout draws differ between processes
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    m = m.cuda().train()
    m.hyp = scaled_hyp(HYP_SCRATCH, nc, img, m.model[-1].nl)
    return m, nc, img


def _batch(rank, nc, img):
    from dmayolo.synthetic import images, targets
    return images(BS, img, seed=1 + rank, device='cuda'), targets(BS, nc, per_image=6, seed=1 + rank, device='cuda')


def _worker(rank, world, port, out, topology, reducer='torch'):
    _setup()
    import torch.distributed as dist
    import dmayolo.functional as Fn
    from dmayolo.trainer import Trainer
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    Fn.set_deterministic(True)
    model, nc, img = _model(topology)
    # train.py:326: find_unused_parameters iff the model holds nn.MultiheadAttention
    fup = any(isinstance(mm, torch.nn.MultiheadAttention) for mm in model.modules())
    assert fup == (topology == 'c5')
    if reducer == 'torch':
        net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], output_device=0,
                                                        find_unused_parameters=fup)
    else:  # the arena reducer (dmayolo.ddp), small buckets so several collectives overlap the backward
        from dmayolo.ddp import ArenaDDP
        net = ArenaDDP(model, bucket_cap_mb=1.0, first_bucket_mb=0.25, compress='bf16' if reducer == 'arena-bf16' else None,
                       find_unused_parameters=fup)
    tr = Trainer(model, model.hyp, BS * world, nb=100, world_size=world, rank=rank, net=net, ema=False)
    tr.i = NI
    x, t = _batch(rank, nc, img)
    loss, items = tr.step(x, t)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all()
    if rank == 0:
        torch.save({k: v.detach().cpu().clone() for k, v in model.named_parameters()}, out)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('topology,reducer', [('yolov5n', 'torch'), ('dma', 'torch'), ('c5', 'torch'),
                                              ('yolov5n', 'arena'), ('dma', 'arena'), ('c5', 'arena'),
                                              ('dma', 'arena-bf16')])
def test_product_ddp_world2_matches_accumulated_single_process(topology, reducer):
    """reducer: torch DDP (train.py:326), or dmayolo.ddp.ArenaDDP (bucketed AVG all-reduce of gradient-arena slices;
    'arena-bf16' with its bf16 compression, held to bf16 precision of the step delta instead)"""
    import torch.multiprocessing as mp
    import dmayolo.functional as Fn
    from dmayolo.trainer import Trainer
    _setup()
    world = 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, 'rank0.pt')
        mp.spawn(_worker, args=(world, _free_port(), out, topology, reducer), nprocs=world, join=True)
        got = torch.load(out, weights_only=True)
    # one process: per-rank forward / backward (BN batch statistics per shard, no SyncBN) accumulated, one step
    Fn.set_deterministic(True)
    try:
        model, nc, img = _model(topology)
        init = {k: v.detach().cpu().clone() for k, v in model.named_parameters()}
        tr = Trainer(model, model.hyp, BS * world, nb=100, world_size=1, rank=-1, ema=False)
        tr.warmup(NI)
        for r in range(world):
            x, t = _batch(r, nc, img)
            loss, _ = tr.compute_loss(model(x), t)
            loss.backward(tr.scaler.upstream)
        tr.scaler.step(tr.optimizer)
        tr.scaler.update()
    finally:
        Fn.set_deterministic(False)
    exp = {k: v.detach().cpu() for k, v in model.named_parameters()}
    assert set(got) == set(exp)
    moved = 0
    dmax = max(float((exp[k] - init[k]).norm()) for k in exp)
    worst = (-1.0, '')
    bf16 = reducer == 'arena-bf16'
    for k, v in got.items():
        if not bf16:
            torch.testing.assert_close(v, exp[k], rtol=1e-4, atol=1e-6, msg=lambda s: f'{k}: {s}')
        de, dg = exp[k] - init[k], v - init[k]
        err = float((dg - de).norm()) / max(float(de.norm()), (1e-2 if bf16 else 1e-3) * dmax)
        worst = max(worst, (err, k))
        moved += int(not torch.equal(v, init[k]))
    print(f'{topology} {reducer}: {len(got)} tensors, worst step-delta relative error {worst[0]:.2e} ({worst[1]})')
    assert worst[0] <= (2e-2 if bf16 else 2e-3), worst
    assert moved > 0.9 * len(got), (moved, len(got))  # the step really updated (nearly) every parameter


def _rccl1_worker(rank, world, port, out, topology):
    """one rank over RCCL: the arena reducer's collectives on a real nccl process group (no world-size-1 shortcut in
    ddp.py), against the unwrapped step of an identical model copy; then both step rates at a larger batch"""
    import copy
    import time
    _setup()
    import torch.distributed as dist
    import dmayolo.functional as Fn
    from dmayolo.ddp import ArenaDDP
    from dmayolo.trainer import Trainer
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', 0))
    assert dist.get_backend() == 'nccl'
    res = {}
    Fn.set_deterministic(True)
    try:
        m1, nc, img = _model(topology)
        m2 = copy.deepcopy(m1)
        fup = any(isinstance(mm, torch.nn.MultiheadAttention) for mm in m1.modules())
        net = ArenaDDP(m1, bucket_cap_mb=0.25, first_bucket_mb=0.05, find_unused_parameters=fup)
        net.trace = []
        t1 = Trainer(m1, m1.hyp, BS, nb=100, world_size=1, rank=0, net=net, ema=False)
        t2 = Trainer(m2, copy.deepcopy(m2.hyp), BS, nb=100, world_size=1, rank=-1, ema=False)
        t1.i = t2.i = NI
        for s in range(3):
            x, t = _batch(s, nc, img)
            l1, _ = t1.step(x, t)
            l2, _ = t2.step(x, t)
            res[f'loss{s}'] = (float(l1), float(l2))
        torch.cuda.synchronize()
        res['launches'] = sum(1 for e in net.trace if e[0].startswith('launch'))
        res['buckets'] = len(net.buckets)
        res['params'] = {k: (v.detach().cpu().clone(), dict(m2.named_parameters())[k].detach().cpu().clone())
                         for k, v in m1.named_parameters()}
        net.close()
    finally:
        Fn.set_deterministic(False)
    if topology != 'dma':
        torch.save(res, out)
        dist.destroy_process_group()
        return
    # the step's extra time with the reducer: DMA-YOLO-l (81 M parameters, 11 buckets of 32 MB), bf16, bs16 @512,
    # wrapped vs unwrapped, alternating
    from dmayolo.models.yolo import Model
    from dmayolo.synthetic import HYP_VISDRONE, scaled_hyp, images, targets
    cfg, nc = os.path.join(CFGDIR, 'yolov5l-ca-sppfcspc-bifpn-scconv.yaml'), 10
    torch.manual_seed(0)
    m = Model(cfg, nc=nc, act_dtype=torch.bfloat16).cuda().train()
    m.hyp = scaled_hyp(HYP_VISDRONE, nc, 512, m.model[-1].nl)
    x, t = images(16, 512, seed=1, device='cuda'), targets(16, nc, seed=1, device='cuda')
    net = ArenaDDP(m, find_unused_parameters=False)
    tw = Trainer(m, m.hyp, 16, nb=100, world_size=1, rank=0, net=net, ema=False)
    tp = Trainer(m, copy.deepcopy(m.hyp), 16, nb=100, world_size=1, rank=-1, ema=False)
    times = {'wrapped': [], 'plain': []}
    for rep in range(3):
        for name, tr in (('wrapped', tw), ('plain', tp)):
            for _ in range(2):
                tr.step(x, t)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                tr.step(x, t)
            torch.cuda.synchronize()
            times[name].append((time.perf_counter() - t0) / 5)
    res['ms'] = {k: sorted(v)[1] * 1e3 for k, v in times.items()}
    res['bucket_mb'] = net.bucket_sizes_mb()
    net.close()
    torch.save(res, out)
    dist.destroy_process_group()


@pytest.mark.parametrize('topology', ['dma', 'c5'])
def test_arena_ddp_on_rccl_world1_matches_unwrapped(topology):
    """ArenaDDP on a world-size-1 `nccl` (RCCL) process group: every bucket goes through an async RCCL all_reduce
    (AVG over one rank = the identity) and the end-of-backward work.wait(), so the parameters after 3 deterministic
    Trainer steps must equal the unwrapped model's bit for bit; c5 also runs the find-unused flag all-reduce
    (train.py:326).  Prints the reducer's extra step time at bs16 @512 bf16."""
    import torch.multiprocessing as mp
    _setup()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, 'r.pt')
        mp.spawn(_rccl1_worker, args=(1, _free_port(), out, topology), nprocs=1, join=True)
        r = torch.load(out, weights_only=True)
    assert r['launches'] == 3 * r['buckets'] and r['buckets'] > 3, (r['launches'], r['buckets'])
    # deterministic mode leaves the Swin LayerNorm / bias-table and CA pooled-gradient atomics, so the
    # two copies agree to the DDP test's tolerance rather than bit for bit after the first step
    assert r['loss0'][0] == r['loss0'][1], r['loss0']
    for s in (1, 2):
        assert abs(r[f'loss{s}'][0] - r[f'loss{s}'][1]) <= 1e-4 * abs(r[f'loss{s}'][1]), r[f'loss{s}']
    for k, (a, b) in r['params'].items():
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=lambda s: f'{k}: {s}')
    if 'ms' not in r:
        return
    ms = r['ms']
    print(f'{topology} RCCL world-1 arena reducer: step {ms["wrapped"]:.2f} ms wrapped vs {ms["plain"]:.2f} ms plain '
          f'(+{ms["wrapped"] - ms["plain"]:.2f} ms, {len(r["bucket_mb"])} buckets)')
