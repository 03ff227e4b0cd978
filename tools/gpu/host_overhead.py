"""Host-side cost of one training step: time to enqueue (no sync) vs the synchronised step, plus a
cProfile of the enqueue path.  python tools/gpu/host_overhead.py [config] [batch]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'dma-yolo_amd'))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else 'v5s-640'
    cfg = list(bench.CONFIGS[cfgname])
    if len(sys.argv) > 2:
        cfg[3] = int(sys.argv[2])
    from dmayolo.optim import build_optimizer
    from dmayolo.synthetic import images, targets
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.utils.torch_utils import ModelEMA
    dev = torch.device('cuda')
    model = bench.build(cfg, torch.bfloat16, dev)
    hyp = model.hyp
    cl = ComputeLoss(model)
    bs = cfg[3]
    opt = build_optimizer(model, 'sgd', hyp['lr0'], hyp['momentum'], hyp['weight_decay'])
    ema = ModelEMA(model)
    imgs, tg = images(bs, cfg[2], device=dev), targets(bs, cfg[1], device=dev)
    step = lambda: bench.train_step(model, model, cl, opt, ema, imgs, tg, 1)  # noqa: E731
    model.train()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'{cfgname} bs{bs}: enqueue {1e3 * (t1 - t0) / n:.2f} ms/step, synchronised {1e3 * (t2 - t0) / n:.2f} ms/step')
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
