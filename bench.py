"""DMA-YOLO hot-path benchmark (BASELINE.json metric: training images/s fwd+bwd @640 & @1536, detect p50 ms incl.
NMS, 1/2/4/8 GPUs).

python bench.py --gpus N --steps K --warmup W [--config dma-1536|v5s-640|...] [--also v5s-640|none]

The headline line is DMA-YOLO-l @1536 (BASELINE configs[2]; configs[3] at N = 8), the north-star model; the same
measurement on yolov5s @640 bs64 (configs[1]) rides in the same JSON line under "at_640" so one default run covers
both halves of the metric.  `--gpus N` without a torchrun environment re-launches itself as N ranks
(torch.distributed.run as a child process; this parent never touches the GPU).

One timed step = one iteration of the reference's batch loop (train.py:400-454) through dmayolo.trainer.Trainer on a
pre-staged synthetic VisDrone-shaped batch: uint8 -> /255 -> forward -> ComputeLoss (SIoU) -> backward seeded with
loss-scale * WORLD_SIZE (DDP all-reduce over RCCL when N > 1) -> GradScaler step (SGD-nesterov, warmup lr/momentum,
accumulate) -> EMA (rank 0).  value = images/s over all ranks (max-over-ranks time), scaling weak (per-GPU batch
fixed).  Also reported: the roofline of the dominant conv kernel family from live HIP events, detect p50 (bs1,
uint8 -> forward -> NMS) and NMS under a 2,000-candidate load, and the CPU oracle (`cpu_baseline`, kind "port") on a
bounded sample.
"""
import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'dma-yolo_amd'))
sys.path.insert(0, ROOT)

if os.environ.get('DMY_SEGV_REPORT'):  # diagnostic fault reporter (tools/segv/segv_report.c): PC / address / maps
    import ctypes
    ctypes.CDLL(os.path.join(ROOT, 'tools', 'segv', 'libsegv_report.so')).segv_report_install()

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
PEAK_FLOPS = {torch.bfloat16: 2500.0e12, torch.float32: 157.3e12, 'fp8': 5000.0e12}  # dense MFMA (MI355X_MICROARCH.md)
PEAK_BW = 8.0e12  # HBM3E bytes/s (MI355X_MICROARCH.md)
VISDRONE_TRAIN_IMAGES = 6471  # VisDrone2019-DET-train (data/VisDrone.yaml): batches per epoch for the schedule


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', default='dma-1536', choices=list(CONFIGS))
    ap.add_argument('--also', default='v5s-640,c5-1920',
                    help='comma list of further configurations measured in the same run, each nested in the JSON '
                         'line as at_<img> ("none": only --config).  c5-1920 (BASELINE configs[4]) runs with the fp8 '
                         'forward, plus a bf16 run of the same steps for its step time')
    ap.add_argument('--batch', type=int, default=0, help='per-GPU batch of --config (default: the config)')
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-detect', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--layer-report', action='store_true', help='per-conv-shape timing table on stderr')
    ap.add_argument('--launch-table', default='', help='CSV of every timed conv launch of the roofline pass (kind, '
                    'shape, algorithmic flops / bytes, measured us, roofline us): the table behind roofline.frac')
    ap.add_argument('--fp8', action='store_true',
                    help='config 5 (BASELINE configs[4]): e4m3 MFMA forward for every conv with C %% 128 == 0')
    ap.add_argument('--ddp', default='arena', choices=['arena', 'torch'],
                    help='N > 1 gradient exchange: the arena reducer (dmayolo.ddp.ArenaDDP: bucketed AVG all-reduce of '
                         'slices of the weight-gradient arena, overlapped with backward) or torch DDP')
    ap.add_argument('--bucket-mb', type=float, default=32.0, help='ArenaDDP bucket size (first bucket 4 MB)')
    ap.add_argument('--grad-compress', default='none', choices=['none', 'bf16'],
                    help='ArenaDDP: send the gradient buckets as bf16 (DDP bf16_compress_hook semantics)')
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'],
                    help='process-group backend (nccl = RCCL; gloo only to rehearse several ranks on one GPU)')
    return ap.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """--gpus N outside torchrun: run this script as N ranks under torch.distributed.run (a child process; the
    parent has not initialised the GPU and only waits) and exit with its status."""
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr=127.0.0.1', f'--master-port={_free_port()}', os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    return subprocess.call(cmd, env=env)


def build(cfg, dtype, device, fp8=False):
    from dmayolo.models.yolo import Model
    from dmayolo.functional import set_fp8
    from dmayolo.synthetic import CONFIGS as CDIR, HYP_VISDRONE, scaled_hyp
    yml, nc, img, _, _ = cfg
    torch.manual_seed(0)
    m = Model(os.path.join(CDIR, yml), nc=nc, act_dtype=dtype)
    m.hyp = scaled_hyp(HYP_VISDRONE, nc, img, m.model[-1].nl)
    if isinstance(m.yaml['anchors'], int):
        # `anchors: N` placeholders (config 5): train.py:318 check_anchors recomputes them from the labels at train
        # start -- here from 200 synthetic images of the bench's label distribution, seeds 0 (utils/autoanchor.py)
        import random
        import numpy as np
        from dmayolo.synthetic import targets
        from dmayolo.utils.autoanchor import check_anchors
        t = targets(200, nc, seed=0).numpy()
        labels = [t[t[:, 0] == i][:, 1:] for i in range(200)]
        np.random.seed(0)
        random.seed(0)
        check_anchors(np.full((200, 2), float(img)), labels, m, thr=m.hyp['anchor_t'], imgsz=img)
    if fp8:
        set_fp8(m, True)
    return m.to(device)


def cpu_baseline(cfg, seconds):
    """The oracle (CPU fp32 restatement of the reference) timed on this host: bs1 train step at the bench
    resolution (fwd + loss + bwd + SGD), repeated for a bounded ~`seconds` sample, on every CPU this job is allotted.
    SURVEY §8(d) asks for all host cores; on the GPU box the job's share is OMP_NUM_THREADS (16 of the machine's 256
    logical CPUs; the harness sizes every pool to it), and a round-5 run with one thread per machine CPU (256) did not
    finish the bench within 900 s, so the baseline runs at torch's thread count = that share, and reports both."""
    v, n, el = _cpu_baseline_run(cfg, seconds)
    return dict(value=v, unit='images/s', cores=torch.get_num_threads(), kind='port',
                sample=f'{n} bs1 train steps of {cfg[0]} @{cfg[2]} (fp32 CPU oracle, {el:.1f} s, '
                       f'{torch.get_num_threads()} threads)', **host_cpu())


def _cpu_baseline_run(cfg, seconds):
    from oracle import nn as onn
    from oracle.loss import compute_loss
    from dmayolo.synthetic import CONFIGS as CDIR, HYP_VISDRONE, scaled_hyp, images, targets
    import yaml
    yml, nc, img, _, _ = cfg
    torch.manual_seed(0)
    with open(os.path.join(CDIR, yml)) as f:
        d = yaml.safe_load(f)
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
    loss, _ = compute_loss(m(x), t, anchors, hyp, nc)  # untimed warmup (allocator, oneDNN primitive cache)
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
    return n / el, n, el


def host_cpu():
    """the host CPU the baseline ran on: model name (lscpu's 'Model name' = /proc/cpuinfo 'model name'), the logical
    CPUs this process may run on, and the machine's total"""
    model = None
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.lower().startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    quota = None  # cgroup CPU quota in CPUs (v2 cpu.max, v1 cfs quota / period), if the job has one
    for path, split in (('/sys/fs/cgroup/cpu.max', True), ('/sys/fs/cgroup/cpu/cpu.cfs_quota_us', False)):
        try:
            with open(path) as f:
                t = f.read().split()
            if split and t[0] != 'max':
                quota = round(int(t[0]) / int(t[1]), 2)
            elif not split and int(t[0]) > 0:
                with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
                    quota = round(int(t[0]) / int(f.read()), 2)
            break
        except (OSError, ValueError, IndexError):
            continue
    return dict(cpu_model=model, cpus_available=avail, cpus_machine=os.cpu_count(), cgroup_cpu_quota=quota,
                omp_num_threads=os.environ.get('OMP_NUM_THREADS'))


def write_launch_table(path, table, ks, cfg_name):
    """One row per timed conv launch: T_roof = max(F / P_mfma, B / BW_hbm) (the bench's peaks), and per kind the
    check line sum T_roof / sum t, which is roofline.frac for the dominant kind."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, 'w') as f:
        f.write(f'# {cfg_name}: conv launches of the roofline pass; peaks {PEAK_FLOPS[torch.bfloat16] / 1e12:.0f} '
                f'TFLOP/s bf16, {PEAK_FLOPS["fp8"] / 1e12:.0f} fp8, {PEAK_BW / 1e9:.0f} GB/s\n')
        f.write('kind,N,C,H,W,K,k,s,flops,bytes,us,troof_us,bound\n')
        for kind, tag, fl, nb, t, tr in table:
            pk = PEAK_FLOPS['fp8'] if kind.endswith('_f8') else PEAK_FLOPS[torch.bfloat16]
            f.write('%s,%s,%.0f,%.0f,%.3f,%.3f,%s\n' % (kind, ','.join(str(v) for v in tag), fl, nb, t * 1e6, tr * 1e6,
                                                        'mfma' if fl / pk >= nb / PEAK_BW else 'hbm'))
        for kind, d in ks.items():
            f.write('# %s: %d launches, sum t %.3f ms, sum T_roof %.3f ms, frac %.4f\n'
                    % (kind, d['launches'], d['seconds'] * 1e3, (d['troof_mfma'] + d['troof_hbm']) * 1e3,
                       (d['troof_mfma'] + d['troof_hbm']) / d['seconds']))


def roofline(ks, steps, el_events, dtype, cfg_name):
    """Dominant conv family by time.  Per launch T_roof = max(F / P_mfma, B / BW_hbm) with F / B its algorithmic
    flops / bytes; frac = sum T_roof / sum measured launch time; `bound` is the resource that
    binds the larger share of sum T_roof, and `achieved` / `peak` are in that resource's unit."""
    dom = max(ks, key=lambda k: ks[k]['seconds'])
    d = ks[dom]
    troof = d['troof_mfma'] + d['troof_hbm']
    hbm = d['troof_hbm'] >= d['troof_mfma']
    if hbm:
        achieved, peak, unit = d['bytes'] / d['seconds'] / 1e9, PEAK_BW / 1e9, 'GB/s'
    else:
        pk = PEAK_FLOPS['fp8'] if dom.endswith('_f8') else PEAK_FLOPS[dtype]
        achieved, peak, unit = d['flops'] / d['seconds'] / 1e12, pk / 1e12, 'TFLOP/s'
    # PMC traffic of the same call population (tools/pmc_traffic.py: every dispatch assigned to the dmy_conv_* call
    # family that launches it, bytes divided by the calls the profiled bench command made); used only when the
    # profiled command made as many calls per step of this family as this run does
    traffic, tsrc, tnote, per_step = None, None, None, None
    tpath = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f).get(cfg_name, {})
        tr = tj.get(dom)
        if tr and 'bytes_per_call' in tr:
            if abs(tr['calls_per_step'] - d['launches'] / steps) < 0.5:
                traffic, tsrc = round(tr['bytes_per_call']), 'profiles/pmc_traffic.json: ' + tr['source']
            else:
                tnote = ('PMC record made %.1f calls per step of %s, this run %.1f: populations differ, not used'
                         % (tr['calls_per_step'], dom, d['launches'] / steps))
        if '_per_step' in tj:
            ps_ = tj['_per_step']
            per_step = dict(pmc_gb=round(ps_['pmc_bytes'] / 1e9, 2), algorithmic_gb=round(ps_['algorithmic_bytes'] / 1e9, 2),
                            ratio=round(ps_['pmc_over_algorithmic'], 3), families=ps_['families'])
    mfma, msrc = {}, None  # MFMA-busy per family from the PMC pass of the same bench command (tools/pmc_mfma.py)
    mpath = os.path.join(ROOT, 'profiles', 'pmc_mfma.json')
    if os.path.exists(mpath):
        with open(mpath) as f:
            mj = json.load(f).get(cfg_name, {})
        mfma = {k: v['mfma_busy'] for k, v in mj.items()}
        msrc = next(iter(mj.values()))['source'] if mj else None
    return dict(bound='hbm' if hbm else 'mfma', kernel=f'dmy_{dom} (implicit-GEMM family, all launches of the roofline pass)',
                mfma_busy=mfma or None, mfma_busy_unit='SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), '
                'time-weighted per family; conv_3x3 = the k > 1 kernels', mfma_busy_source=msrc,
                achieved=round(achieved, 2), peak=peak, unit=unit, frac=round(troof / d['seconds'], 4),
                achieved_over_peak=round(achieved / peak, 4),
                traffic=traffic, traffic_unit='bytes/launch (HBM, PMC, same call population)', traffic_source=tsrc,
                traffic_note=tnote,
                traffic_over_algorithmic=round(traffic / (d['bytes'] / d['launches']), 3) if traffic else None,
                conv_traffic_per_step=per_step,
                algorithmic_bytes_per_launch=round(d['bytes'] / d['launches']),
                algorithmic_flops_per_launch=round(d['flops'] / d['launches']),
                launches=d['launches'], avg_launch_us=round(d['seconds'] / d['launches'] * 1e6, 2),
                troof_share={'mfma': round(d['troof_mfma'] / troof, 3), 'hbm': round(d['troof_hbm'] / troof, 3)},
                kernels={k: dict(launches=v['launches'], ms=round(v['seconds'] * 1e3 / steps, 3),
                                 tflops=round(v['flops'] / v['seconds'] / 1e12, 2),
                                 gbps=round(v['bytes'] / v['seconds'] / 1e9, 1),
                                 frac=round((v['troof_mfma'] + v['troof_hbm']) / v['seconds'], 4),
                                 **({'mfma_busy': mfma[k]} if k in mfma else {})) for k, v in ks.items()},
                conv_share_of_step=round(sum(v['seconds'] for v in ks.values()) / el_events, 3),
                measured_in='separate pass of the same %d steps with per-launch HIP events (%.1f ms/step there)'
                            % (steps, el_events * 1e3 / steps))


def run_config(name, a, world, rank, dev_idx, device, dtype, batch=0, cpu_seconds=15.0, fp8=False, light=False):
    """light: only the timed steps (no roofline pass, detect or CPU baseline) -- the bf16 twin of the fp8 config-5
    leg, for its step time"""
    from dmayolo.functional import KernelTimer
    from dmayolo.synthetic import images, targets, clustered_predictions
    from dmayolo.infer import GraphedDetector
    from dmayolo.trainer import Trainer
    from dmayolo.utils.general import non_max_suppression

    cfg = list(CONFIGS[name])
    if batch:
        cfg[3] = batch
    yml, nc, img, bs, _ = cfg
    torch.cuda.reset_peak_memory_stats(device)
    model = build(cfg, dtype, device, fp8=fp8)
    net = model
    # train.py:326 (find_unused_parameters when the model holds nn.MultiheadAttention)
    fu = any(isinstance(m, torch.nn.MultiheadAttention) for m in model.modules())
    if world > 1 and a.ddp == 'arena':  # buckets = slices of the gradient arena (dmayolo/ddp.py)
        from dmayolo.ddp import ArenaDDP
        net = ArenaDDP(model, bucket_cap_mb=a.bucket_mb, compress=None if a.grad_compress == 'none' else a.grad_compress,
                       find_unused_parameters=fu)
    elif world > 1:
        net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev_idx], output_device=dev_idx,
                                                        find_unused_parameters=fu)
    total_bs = bs * world
    tr = Trainer(model, model.hyp, total_bs, epochs=300, nb=-(-VISDRONE_TRAIN_IMAGES // total_bs), world_size=world,
                 rank=rank if world > 1 else -1, net=net)
    imgs = images(bs, img, seed=1 + rank, device=device)
    tg = targets(bs, nc, seed=1 + rank, device=device)

    model.train()
    for _ in range(a.warmup):
        tr.step(imgs, tg)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss, items = tr.step(imgs, tg)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if light:
        if world > 1:
            t = torch.tensor([el], device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t)
        res = dict(value=round(world * bs * a.steps / el, 2), ms_per_step=round(el / a.steps * 1e3, 3),
                   peak_hbm_gib=round(torch.cuda.max_memory_allocated(device) / 2 ** 30, 1))
        del tr, net, model, imgs, tg, loss, items
        gc.collect()
        torch.cuda.empty_cache()
        return res
    # roofline pass: the same K steps again with a HIP event pair around every implicit-GEMM launch on its stream
    # (functional.KernelTimer).  Kept out of the timed region: ~380 event records per yolov5s step cost ~6 % of the
    # step (3400 vs 3184 img/s measured), which would understate `value`.
    KernelTimer.enabled = True
    KernelTimer.records = []
    t1 = time.perf_counter()
    for _ in range(a.steps):
        tr.step(imgs, tg)
    torch.cuda.synchronize()
    el_events = time.perf_counter() - t1
    KernelTimer.enabled = False
    detail = {} if a.layer_report else None
    table = [] if a.launch_table else None
    ks = KernelTimer.summary(detail, PEAK_FLOPS[dtype], PEAK_BW, peak_flops_f8=PEAK_FLOPS['fp8'], table=table)
    if table is not None and rank == 0:
        write_launch_table(a.launch_table if name == a.config else a.launch_table.replace('.csv', f'_{name}.csv'),
                           table, ks, name)
    if detail and rank == 0:
        tot = sum(v[2] for v in detail.values())
        print(f'[{name}] kind        N    C    H    W    K  k s  launches  ms/step  TFLOP/s  share', file=sys.stderr)
        for (kind, tag), v in sorted(detail.items(), key=lambda kv: -kv[1][2]):
            print('%-10s %s %6d %8.3f %8.1f %6.3f' % (kind, ' '.join('%4d' % t for t in tag), v[0],
                  v[2] * 1e3 / a.steps, v[1] / v[2] / 1e12, v[2] / tot), file=sys.stderr)
    if world > 1:
        t = torch.tensor([el], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    assert torch.isfinite(loss).all(), 'non-finite loss'
    res = dict(value=round(world * bs * a.steps / el, 2), unit='images/s', ms_per_step=round(el / a.steps * 1e3, 3),
               config={'workload': f'{yml} train @{img} nc={nc}', 'model': yml, 'global_batch': total_bs, 'img': img,
                       'parallelism': f'dp{world}',
                       **({'grad_exchange': (a.ddp + ('' if a.ddp == 'torch' else ' bucket %g MB' % a.bucket_mb) +
                                             ('' if a.grad_compress == 'none' else ' ' + a.grad_compress))}
                          if world > 1 else {})},
               roofline=roofline(ks, a.steps, el_events, dtype, name),
               loss_items=[round(float(v), 5) for v in items], lr=[round(float(g['lr']), 8) for g in tr.optimizer.param_groups],
               loss_scale=tr.scaler.get_scale())

    if rank == 0 and not a.no_detect:
        # detect p50 (detect.py:175-243): bs1 uint8 on device -> forward -> NMS(0.25, 0.45, max_det 1000)
        ev = tr.ema.ema if tr.ema is not None else model
        ev.eval()
        x1 = images(1, img, seed=3, device=device)
        graphed = GraphedDetector(ev)

        def p50(fwd, n=60):
            lat = []
            for i in range(n):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                z, _ = fwd(x1)
                dets = non_max_suppression(z, 0.25, 0.45, max_det=1000)
                torch.cuda.synchronize()
                lat.append(time.perf_counter() - t1)
            lat = sorted(lat[10:])
            return z, dets, round(lat[len(lat) // 2] * 1e3, 3)

        def p50_graph(n=60):  # forward + NMS recorded in ONE graph, one host read of the keep counts (infer.py)
            lat = []
            for i in range(n):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                dets, (z, _) = graphed.detect(x1, 0.25, 0.45, max_det=1000)
                torch.cuda.synchronize()
                lat.append(time.perf_counter() - t1)
            lat = sorted(lat[10:])
            return z, dets, round(lat[len(lat) // 2] * 1e3, 3)

        with torch.no_grad():
            z, de, res['detect_eager_p50_ms'] = p50(ev)
            zg, dg, res['detect_graph_fwd_p50_ms'] = p50(graphed)  # graph-replayed forward, eager NMS
            zd, dd, res['detect_p50_ms'] = p50_graph()  # forward + NMS in one graph replay
            assert torch.equal(z, zg) and torch.equal(z, zd), 'graph replay differs from the eager forward'
            assert len(de) == len(dd) and all(torch.equal(a, b) for a, b in zip(de, dd)), 'graphed NMS differs'
            # NMS under load: random-init weights leave ~0 boxes above conf, so time NMS on Detect-shaped synthetic
            # predictions with 2,000 candidates (200 clusters x 10), alone and in the same timed loop as
            # the replayed forward (detect p50 as a loaded detector would see it)
            sp = clustered_predictions(1, z.shape[1], nc, device=device)
            nl, dl = [], []
            for i in range(40):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                non_max_suppression(sp, 0.25, 0.45, max_det=1000)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                graphed(x1)
                non_max_suppression(sp, 0.25, 0.45, max_det=1000)
                torch.cuda.synchronize()
                nl.append(t2 - t1)
                dl.append(time.perf_counter() - t2)
            nl, dl = sorted(nl[10:]), sorted(dl[10:])
            res['nms_2000cand_p50_ms'] = round(nl[len(nl) // 2] * 1e3, 3)
            res['detect_2000cand_p50_ms'] = round(dl[len(dl) // 2] * 1e3, 3)
    res['peak_hbm_gib'] = round(torch.cuda.max_memory_allocated(device) / 2 ** 30, 1)
    del tr, net, model, imgs, tg
    gc.collect()
    torch.cuda.empty_cache()
    res['cpu_baseline'] = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res['cpu_baseline'] = cpu_baseline(cfg, cpu_seconds)
    return res


def main():
    a = parse()
    if a.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn_ranks(a.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    ndev = torch.cuda.device_count()
    dev_idx = local % max(ndev, 1)
    torch.cuda.set_device(dev_idx)
    if world > 1:
        if a.backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev_idx))
        else:
            dist.init_process_group('gloo')
    device = torch.device('cuda', dev_idx)
    dtype = torch.bfloat16 if a.dtype == 'bf16' else torch.float32

    head = run_config(a.config, a, world, rank, dev_idx, device, dtype, a.batch, a.cpu_seconds, fp8=a.fp8)
    also = {}
    for name in [n for n in a.also.split(',') if n and n != 'none' and n != a.config]:
        assert name in CONFIGS, (name, list(CONFIGS))
        f8 = name == 'c5-1920' and dtype == torch.bfloat16  # BASELINE configs[4]: "fp8 MFMA conv"
        r = run_config(name, a, world, rank, dev_idx, device, dtype, 0, a.cpu_seconds, fp8=f8)
        if f8:
            b = run_config(name, a, world, rank, dev_idx, device, dtype, 0, fp8=False, light=True)
            r['dtype'] = 'bf16 storage, fp8 e4m3 forward convs'
            r['bf16_twin'] = dict(b, fp8_speedup=round(r['value'] / b['value'], 4))
        also['at_%d' % CONFIGS[name][2]] = dict(config_name=name, **r)

    if rank == 0:
        img = CONFIGS[a.config][2]
        line = {
            'metric': 'train images/sec (fwd+loss+bwd+optimizer, train.py batch loop) @%d; detect p50 ms incl. NMS' % img,
            'value': head.pop('value'), 'unit': head.pop('unit'), 'n_gpus': world, 'steps': a.steps,
            'warmup': a.warmup, 'ms_per_step': head.pop('ms_per_step'), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None,
            'dtype': ('bf16' if dtype == torch.bfloat16 else 'fp32') + (' (fp8 e4m3 forward convs)' if a.fp8 else ''),
            'data': 'synthetic (uint8 images seed 1+rank, 50 VisDrone-like targets/img; random-init weights)',
            'config': head.pop('config'), 'roofline': head.pop('roofline'), 'cpu_baseline': head.pop('cpu_baseline'),
            **head,
        }
        line.update(also)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
