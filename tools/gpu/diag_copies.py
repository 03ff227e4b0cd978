"""Diagnostic: which host calls launch the runtime copy / fill / elementwise kernels of a yolov5s training step."""
import os, sys, collections
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]
import torch
import bench
from dmayolo.trainer import Trainer
from dmayolo import optim
from dmayolo.synthetic import images, targets

cfg = bench.CONFIGS['v5s-640']
m = bench.build(cfg, torch.bfloat16, torch.device('cuda', 0))
tr = Trainer(m, m.hyp, 64, nb=100)
x, t = images(64, 640, device='cuda'), targets(64, 10, device='cuda')
for _ in range(3):
    tr.step(x, t)
torch.cuda.synchronize()
misses = [0]
orig = optim._Table.__init__
def counting(self, *a, **k):
    misses[0] += 1
    orig(self, *a, **k)
optim._Table.__init__ = counting
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
    for _ in range(2):
        tr.step(x, t)
    torch.cuda.synchronize()
print('table misses in 2 steps:', misses[0])
ev = prof.key_averages(group_by_stack_n=6)
rows = [e for e in ev if e.key in ('aten::copy_', 'aten::clone', 'aten::fill_', 'aten::zero_', 'aten::add', 'aten::add_',
                                   'aten::to', 'aten::_to_copy', 'aten::mul', 'aten::zeros', 'aten::cat', 'aten::contiguous')]
rows.sort(key=lambda e: -e.count)
for e in rows[:30]:
    print(e.count // 2, e.key, ' <- ', ' | '.join(s for s in e.stack[:6] if 'dmayolo' in s or 'bench' in s or 'trainer' in s)[:400])
