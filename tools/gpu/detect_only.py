"""Detect-path workload for profiling: bs1 uint8 image -> graphed eval forward + NMS (one graph), N iterations.
python tools/gpu/detect_only.py [config] [iters] [--eager | --graph-fwd]  (--graph-fwd: graphed forward, eager NMS)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]
import torch  # noqa: E402
import bench  # noqa: E402
from dmayolo.infer import GraphedDetector  # noqa: E402
from dmayolo.synthetic import images  # noqa: E402
from dmayolo.utils.general import non_max_suppression  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'dma-1536'
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
eager = '--eager' in sys.argv
gfwd = '--graph-fwd' in sys.argv
warm = '--warm' in sys.argv  # diagnostic: read every prepped inference weight before each timed call (L2 / MALL warm)
m = bench.build(list(bench.CONFIGS[cfg]), torch.bfloat16, torch.device('cuda', 0)).eval()
x = images(1, bench.CONFIGS[cfg][2], seed=3, device='cuda')
det = m if eager else GraphedDetector(m)
lat = []
wts = []
with torch.no_grad():
    for i in range(iters):
        if warm:
            if not wts:
                from dmayolo import functional as Fn
                specs = list(Fn._SPECS.values()) + [sp for _, d in Fn._PSPECS.values() for sp in d.values()]
                wts = [sp.wcache[1] for sp in specs if getattr(sp, 'wcache', None) is not None]
            for t in wts:
                t.view(-1)[::64].sum()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if eager or gfwd:
            z, _ = det(x)
            non_max_suppression(z, 0.25, 0.45, max_det=1000)
        else:
            det.detect(x, 0.25, 0.45, max_det=1000)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
lat = sorted(lat[10:])
print(f'{cfg} detect p50 {lat[len(lat) // 2] * 1e3:.3f} ms ({"eager" if eager else "graph fwd" if gfwd else "graph"}'
      f'{", weights warm: %d tensors" % len(wts) if warm else ""})')
