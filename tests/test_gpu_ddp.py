"""GPU, world_size 2: the PRODUCT training step (Model / ComputeLoss / FusedSGD / GradScaler through
dmayolo.trainer.Trainer) under torch DistributedDataParallel (train.py:326; loss * WORLD_SIZE, train.py:438-440) with
two gloo ranks sharing cuda:0, against one process that accumulates the two ranks' batches' gradients and takes the
same optimizer step.  This is the path bench.py runs over RCCL at N > 1 (the collective here is gloo because both
ranks sit on one GPU).  fp32 storage; tolerance covers the split-K weight-gradient atomics' summation order."""
import os
import socket
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs', 'yolov5n.yaml')
IMG, BS, NC, NI = 128, 2, 10, 500  # NI: integrated batch index (mid-warmup: every group has a non-zero lr)


def _setup():
    for p in (ROOT, os.path.join(ROOT, 'dma-yolo_amd')):
        if p not in sys.path:
            sys.path.insert(0, p)


def _model():
    from dmayolo.models.yolo import Model
    from dmayolo.synthetic import HYP_SCRATCH, scaled_hyp
    torch.manual_seed(0)
    m = Model(CFG, nc=NC, act_dtype=torch.float32).cuda().train()
    m.hyp = scaled_hyp(HYP_SCRATCH, NC, IMG)
    return m


def _batch(rank):
    from dmayolo.synthetic import images, targets
    return images(BS, IMG, seed=1 + rank, device='cuda'), targets(BS, NC, per_image=6, seed=1 + rank, device='cuda')


def _worker(rank, world, port, out):
    _setup()
    import torch.distributed as dist
    from dmayolo.trainer import Trainer
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    model = _model()
    net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], output_device=0)
    tr = Trainer(model, model.hyp, BS * world, nb=100, world_size=world, rank=rank, net=net, ema=False)
    tr.i = NI
    x, t = _batch(rank)
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


def test_product_ddp_world2_matches_accumulated_single_process():
    import torch.multiprocessing as mp
    from dmayolo.trainer import Trainer
    _setup()
    world = 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, 'rank0.pt')
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        got = torch.load(out, weights_only=True)
    # one process: per-rank forward / backward (BN batch statistics per shard, no SyncBN) accumulated, one step
    model = _model()
    init = {k: v.detach().cpu().clone() for k, v in model.named_parameters()}
    tr = Trainer(model, model.hyp, BS * world, nb=100, world_size=1, rank=-1, ema=False)
    tr.warmup(NI)
    for r in range(world):
        x, t = _batch(r)
        loss, _ = tr.compute_loss(model(x), t)
        loss.backward(tr.scaler.upstream)
    tr.scaler.step(tr.optimizer)
    tr.scaler.update()
    exp = dict(model.named_parameters())
    assert set(got) == set(exp)
    moved = 0
    for k, v in got.items():
        e = exp[k].detach().cpu()
        torch.testing.assert_close(v, e, rtol=1e-4, atol=1e-6, msg=lambda s: f'{k}: {s}')
        moved += int(not torch.equal(v, init[k]))
    assert moved > 0.9 * len(got), (moved, len(got))  # the step really updated (nearly) every parameter
