"""Per-layer conv times of the bs1 eval forward (eager, HIP events per launch via KernelTimer).
python tools/gpu/det_layers.py [config] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]
import torch  # noqa: E402
import bench  # noqa: E402
from dmayolo.functional import KernelTimer  # noqa: E402
from dmayolo.synthetic import images  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'dma-1536'
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
m = bench.build(list(bench.CONFIGS[cfg]), torch.bfloat16, torch.device('cuda', 0)).eval()
x = images(1, bench.CONFIGS[cfg][2], seed=3, device='cuda')
with torch.no_grad():
    for _ in range(3):
        m(x)
    torch.cuda.synchronize()
    KernelTimer.enabled = True
    for _ in range(iters):
        m(x)
    KernelTimer.enabled = False
    torch.cuda.synchronize()
agg = {}
for kind, fl, nb, e0, e1, tag in KernelTimer.records:
    a = agg.setdefault((kind, tag), [0, 0.0, fl, nb])
    a[0] += 1
    a[1] += e0.elapsed_time(e1) * 1e3
tot = sum(a[1] for a in agg.values()) / iters
print(f'total conv {tot:.1f} us / forward')
for (kind, tag), (n, us, fl, nb) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    per = us / n
    print(f'{kind:12s} {str(tag):34s} x{n / iters:4.1f} {per:7.1f} us {fl / per / 1e6:6.1f} TF/s {nb / per / 1e3:6.0f} GB/s '
          f'{us / iters:7.1f} us/fwd')
