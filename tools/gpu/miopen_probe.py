"""Where the first per-layer bench-shape test spends its time: the fp32 oracle model's forward + backward at a bench
shape, first and second call (MIOpen builds its kernels on first use of a conv configuration on a fresh box).
python tools/gpu/miopen_probe.py <config yaml> <img> <bs>"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd'), os.path.join(ROOT, 'tests')]
import torch  # noqa: E402
import yaml  # noqa: E402
from dmayolo.synthetic import images, CONFIGS  # noqa: E402
from oracle import nn as onn  # noqa: E402

yml, img, bs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
with open(os.path.join(CONFIGS, yml)) as f:
    cfg = yaml.safe_load(f)
torch.manual_seed(0)
ref = onn.bn_defaults(onn.Model(cfg, nc=10)).cuda().train()
x = images(bs, img, seed=1).cuda().float() / 255
for it in range(3):
    torch.cuda.synchronize()
    t = time.time()
    with torch.no_grad():
        ref(x)
    torch.cuda.synchronize()
    t1 = time.time()
    out = ref(x)
    sum(o.float().sum() for o in out).backward()
    torch.cuda.synchronize()
    print(f'{yml} {img} bs{bs} call {it}: no-grad forward {t1 - t:.2f} s, forward+backward {time.time() - t1:.2f} s '
          f'env MIOPEN_FIND_MODE={os.environ.get("MIOPEN_FIND_MODE")}', flush=True)
