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
        net = ArenaDDP(model, bucket_cap_mb=1.0, first_bucket_mb=0.25, compress='bf16' if reducer == 'arena-bf16' else None)
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
