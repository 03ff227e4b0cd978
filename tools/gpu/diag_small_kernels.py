"""Where the torch-side small kernels of a training step come from (copies, fills, adds): torch.profiler over one
DMA-YOLO-l step, every aten::copy_ / fill_ / zero_ / add / zeros op grouped by the innermost dmayolo source line.
python tools/gpu/diag_small_kernels.py [yaml] [img] [bs]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]
import torch  # noqa: E402
from torch.profiler import profile, ProfilerActivity  # noqa: E402
from dmayolo.models.yolo import Model  # noqa: E402
from dmayolo.trainer import Trainer  # noqa: E402
from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp, CONFIGS  # noqa: E402

yml = sys.argv[1] if len(sys.argv) > 1 else 'yolov5l-ca-sppfcspc-bifpn-scconv.yaml'
img = int(sys.argv[2]) if len(sys.argv) > 2 else 512
bs = int(sys.argv[3]) if len(sys.argv) > 3 else 4
torch.manual_seed(0)
m = Model(os.path.join(CONFIGS, yml), nc=10, act_dtype=torch.bfloat16).cuda().train()
m.hyp = scaled_hyp(HYP_VISDRONE, 10, img)
tr = Trainer(m, dict(m.hyp), 64, nb=100)
tr.i = 500
x, t = images(bs, img, seed=1, device='cuda'), targets(bs, 10, seed=1, device='cuda')
for _ in range(3):
    tr.step(x, t)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    tr.step(x, t)
    torch.cuda.synchronize()
agg = collections.Counter()
for ev in prof.events():
    if ev.name not in ('aten::copy_', 'aten::fill_', 'aten::zero_', 'aten::add', 'aten::add_', 'aten::zeros',
                       'aten::clone', 'aten::contiguous', 'aten::to', 'aten::_to_copy', 'aten::mul', 'aten::div_'):
        continue
    site = next((f for f in ev.stack if 'dmayolo' in f or 'bench' in f), ev.stack[0] if ev.stack else '?')
    agg[(ev.name, site.split('/')[-1][:90])] += 1
for (name, site), n in agg.most_common(40):
    print(f'{n:4d}  {name:18s} {site}')
