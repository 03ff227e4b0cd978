"""DMA-YOLO hot-path benchmark (BASELINE.json metric: training images/s fwd+bwd, detect p50 ms incl. NMS).

python bench.py --gpus N --steps K --warmup W [--config v5s-640|dma-1536|dma-640] [--batch B]

One timed step = one full training iteration of the reference loop (train.py:400-454) on a
pre-staged synthetic VisDrone-shaped batch: uint8 -> /255 -> forward -> ComputeLoss (SIoU) ->
loss*WORLD_SIZE -> backward (DDP all-reduce over RCCL when N > 1) -> SGD-nesterov step -> EMA
(rank 0).  value = images/s over all ranks (max-over-ranks time), scaling weak (per-GPU batch fixed).
Also reported: live HIP-event roofline of the dominant implicit-GEMM conv kernel, detect p50
(bs1, uint8 -> forward -> NMS), and the CPU oracle (`cpu_baseline`, kind "port") on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'dma-yolo_amd'))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # name: (yaml, nc, img, per-GPU batch, hyp)
    'v5s-640': ('yolov5s.yaml', 10, 640, 64, 'visdrone'),
    'dma-640': ('yolov5l-ca-sppfcspc-bifpn-scconv.yaml', 10, 640, 32, 'visdrone'),
    'dma-1536': ('yolov5l-ca-sppfcspc-bifpn-scconv.yaml', 10, 1536, 32, 'visdrone'),
    'dmaca-1536': ('yolov5l-ca-sppfcspc-bifpn.yaml', 10, 1536, 32, 'visdrone'),  # C3CA sibling
    'c5-1920': ('yolov5l-xs-tr-cbam-spp-bifpn.yaml', 3, 1920, 8, 'visdrone'),  # config 5 (UAVDT nc=3)
}
PEAK = {torch.bfloat16: 2500.0, torch.float32: 157.3}  # dense TFLOP/s (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', default='v5s-640', choices=list(CONFIGS))
    ap.add_argument('--batch', type=int, default=0, help='per-GPU batch (default: the config)')
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-detect', action='store_true')
    ap.add_argument('--graph', action='store_true',
                    help='replay fwd+loss+bwd as one HIP graph (train_graph.py; measured 3405 vs 3398 img/s eager '
                         'on yolov5s: the gaps between dependent kernels are not launch overhead)')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--layer-report', action='store_true', help='per-conv-shape timing table on stderr')
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'],
                    help='process-group backend (nccl = RCCL; gloo only to rehearse several ranks on one GPU)')
    return ap.parse_args()


def build(cfg, dtype, device):
    from dmayolo.models.yolo import Model
    from dmayolo.synthetic import CONFIGS as CDIR, HYP_VISDRONE, scaled_hyp
    yml, nc, img, _, _ = cfg
    torch.manual_seed(0)
    m = Model(os.path.join(CDIR, yml), nc=nc, act_dtype=dtype).to(device)
    m.hyp = scaled_hyp(HYP_VISDRONE, nc, img, m.model[-1].nl)
    return m


def train_step(net, model, compute_loss, opt, ema, imgs, tg, world):
    """One iteration of train.py:400-454 on a staged batch: forward (DDP-wrapped `net` when world > 1),
    loss * WORLD_SIZE (train.py:440; DDP averages, so the applied gradient is the sum over ranks),
    backward (RCCL bucketed all-reduce overlapped by DDP), optimizer step, rank-0 EMA."""
    pred = net(imgs)
    loss, _ = compute_loss(pred, tg)
    if world > 1:
        loss = loss * world
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)
    if ema is not None:
        ema.update(model)
    return loss


def cpu_baseline(cfg, seconds):
    """The oracle (CPU fp32 restatement of the reference) timed on this host: bs1 train step at the
    bench resolution (fwd + loss + bwd + SGD), repeated for a bounded ~`seconds` sample."""
    from oracle import nn as onn
    from oracle.loss import compute_loss
    from dmayolo.synthetic import CONFIGS as CDIR, HYP_VISDRONE, scaled_hyp, images, targets
    import yaml
    yml, nc, img, _, _ = cfg
    torch.manual_seed(0)
    d = yaml.safe_load(open(os.path.join(CDIR, yml)))
    m = onn.bn_defaults(onn.Model(d, nc=nc)).train()
    for mod in m.modules():
        if isinstance(mod, onn.SwinTransformerLayer):
            mod.drop_prob = 0.0
    det = m.model[-1]
    hyp = scaled_hyp(HYP_VISDRONE, nc, img, det.nl)
    anchors = det.anchors / det.stride.view(-1, 1, 1)
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.937, nesterov=True)
    x = images(1, img).float() / 255
    t = targets(1, nc)
    for _ in range(2):  # untimed warmup (allocator, oneDNN primitive cache)
        loss, _ = compute_loss(m(x), t, anchors, hyp, nc)
        loss.backward()
        opt.zero_grad(set_to_none=True)
    n, t0 = 0, time.perf_counter()
    while True:
        p = m(x)
        loss, _ = compute_loss(p, t, anchors, hyp, nc)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        n += 1
        el = time.perf_counter() - t0
        if (el > seconds and n >= 2) or n >= 2000:
            break
    return dict(value=n / el, unit='images/s', cores=torch.get_num_threads(), kind='port',
                sample=f'{n} bs1 train steps of {yml} @{img} (fp32 CPU oracle, {el:.1f} s)')


def main():
    a = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    ndev = torch.cuda.device_count()
    dev_idx = local % max(ndev, 1)
    if world > 1:
        torch.cuda.set_device(dev_idx)
        if a.backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev_idx))
        else:
            dist.init_process_group('gloo')
    device = torch.device('cuda', dev_idx)
    cfg = list(CONFIGS[a.config])
    if a.batch:
        cfg[3] = a.batch
    yml, nc, img, bs, _ = cfg
    dtype = torch.bfloat16 if a.dtype == 'bf16' else torch.float32

    from dmayolo.functional import KernelTimer
    from dmayolo.optim import build_optimizer
    from dmayolo.synthetic import images, targets, clustered_predictions
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.infer import GraphedDetector
    from dmayolo.train_graph import GraphedTrainStep
    from dmayolo.utils.general import non_max_suppression
    from dmayolo.utils.torch_utils import ModelEMA

    model = build(cfg, dtype, device)
    hyp = model.hyp
    compute_loss = ComputeLoss(model)
    opt = build_optimizer(model, 'sgd', hyp['lr0'], hyp['momentum'], hyp['weight_decay'] * bs * max(round(64 / bs), 1) / 64)
    ema = ModelEMA(model) if rank == 0 else None
    net = model
    if world > 1:
        net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev_idx], output_device=dev_idx)
    imgs = images(bs, img, seed=1 + rank, device=device)
    tg = targets(bs, nc, seed=1 + rank, device=device)

    graphed = GraphedTrainStep(model, compute_loss, opt, ema) if world == 1 and a.graph else None

    def step():
        if graphed is not None:  # forward + loss + backward replayed as one HIP graph (train_graph.py)
            return graphed(imgs, tg)[0]
        return train_step(net, model, compute_loss, opt, ema, imgs, tg, world)

    def eager_step():
        return train_step(net, model, compute_loss, opt, ema, imgs, tg, world)

    model.train()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # roofline pass: the same K steps again with a HIP event pair around every implicit-GEMM launch on its
    # stream (functional.KernelTimer).  Kept out of the timed region: ~380 event records per yolov5s step
    # cost ~6 % of the step (3400 vs 3184 img/s measured), which would understate `value`.
    KernelTimer.enabled = True
    KernelTimer.records = []
    t1 = time.perf_counter()
    for _ in range(a.steps):
        eager_step()  # events need the eager launches (a graph replays without the Python timer)
    torch.cuda.synchronize()
    el_events = time.perf_counter() - t1
    KernelTimer.enabled = False
    detail = {} if a.layer_report else None
    ks = KernelTimer.summary(detail)
    if detail and rank == 0:
        tot = sum(v[2] for v in detail.values())
        print('kind        N    C    H    W    K  k s  launches  ms/step  TFLOP/s  share', file=sys.stderr)
        for (kind, tag), v in sorted(detail.items(), key=lambda kv: -kv[1][2]):
            print('%-10s %s %6d %8.3f %8.1f %6.3f' % (kind, ' '.join('%4d' % t for t in tag), v[0],
                  v[2] * 1e3 / a.steps, v[1] / v[2] / 1e12, v[2] / tot), file=sys.stderr)
    if world > 1:
        t = torch.tensor([el], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    assert torch.isfinite(loss).all(), 'non-finite loss'
    peak_gb = torch.cuda.max_memory_allocated(device) / 2 ** 30
    ips = world * bs * a.steps / el

    # dominant kernel family by time -> roofline
    dom = max(ks, key=lambda k: ks[k]['seconds'])
    d = ks[dom]
    achieved = d['flops'] / d['launches'] / (d['seconds'] / d['launches']) / 1e12
    # traffic: HBM bytes per launch of the same kernel family from the committed rocprofv3 --pmc passes
    # (FETCH_SIZE / WRITE_SIZE in separate runs of this bench command, tools/gpu/pmc.sh + tools/pmc_traffic.py)
    traffic, tsrc = None, None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'pmc_traffic.json')
    if os.path.exists(tpath):
        tr = json.load(open(tpath)).get(a.config, {}).get(dom)
        if tr:
            traffic, tsrc = round(tr['bytes_per_launch']), 'profiles/pmc_traffic.json: ' + tr['source']
    roof = dict(bound='mfma', kernel=f'dmy_{dom} (implicit-GEMM, all launches of the roofline pass)',
                achieved=round(achieved, 2), peak=PEAK[dtype], unit='TFLOP/s', frac=round(achieved / PEAK[dtype], 4),
                traffic=traffic, traffic_unit='bytes/launch (HBM, PMC)', traffic_source=tsrc,
                algorithmic_bytes_per_launch=round(d['bytes'] / d['launches']),
                launches=d['launches'], avg_launch_us=round(d['seconds'] / d['launches'] * 1e6, 2),
                kernels={k: dict(launches=v['launches'], ms=round(v['seconds'] * 1e3 / a.steps, 3),
                                 tflops=round(v['flops'] / v['seconds'] / 1e12, 2)) for k, v in ks.items()},
                conv_share_of_step=round(sum(v['seconds'] for v in ks.values()) / el_events, 3),
                measured_in='separate pass of the same %d steps with per-launch HIP events (%.1f ms/step there)'
                            % (a.steps, el_events * 1e3 / a.steps))

    extra = {}
    if rank == 0 and not a.no_detect:
        # detect p50 (detect.py:175-243): bs1 uint8 on device -> forward -> NMS(0.25, 0.45, max_det 1000)
        model.eval()
        x1 = images(1, img, seed=3, device=device)
        graphed = GraphedDetector(model)

        def p50(fwd, n=60):
            lat = []
            for i in range(n):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                z, _ = fwd(x1)
                non_max_suppression(z, 0.25, 0.45, max_det=1000)
                torch.cuda.synchronize()
                lat.append(time.perf_counter() - t1)
            lat = sorted(lat[10:])
            return z, round(lat[len(lat) // 2] * 1e3, 3)

        with torch.no_grad():
            z, extra['detect_eager_p50_ms'] = p50(model)
            zg, extra['detect_p50_ms'] = p50(graphed)  # HIP-graph replay of the forward + NMS (infer.py)
            assert torch.equal(z, zg), 'graph replay differs from the eager forward'
            A = z.shape[1]
            sp = clustered_predictions(1, A, nc, device=device)
            nl = []
            for i in range(30):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                non_max_suppression(sp, 0.25, 0.45, max_det=1000)
                torch.cuda.synchronize()
                nl.append(time.perf_counter() - t1)
            nl = sorted(nl[5:])
            extra['nms_2000cand_p50_ms'] = round(nl[len(nl) // 2] * 1e3, 3)
        model.train()

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(cfg, a.cpu_seconds)

    if rank == 0:
        line = {
            'metric': 'train images/sec (fwd+loss+bwd+SGD+EMA) @%d; detect p50 ms incl. NMS' % img,
            'value': round(ips, 2), 'unit': 'images/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': round(el / a.steps * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'bf16' if dtype == torch.bfloat16 else 'fp32',
            'data': 'synthetic (uint8 images seed 1, 50 VisDrone-like targets/img; random-init weights)',
            'config': {'workload': f'{yml} train @{img} nc={nc}', 'model': yml, 'global_batch': bs * world,
                       'img': img, 'parallelism': f'dp{world}'},
            'roofline': roof, 'cpu_baseline': cpu, 'peak_hbm_gib': round(peak_gb, 1), **extra,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
