"""Which objects accumulate across Trainer steps (memory-flat test diagnosis): per-step memory_allocated, then the
diff of live python objects by type and of live CUDA tensors by (shape, dtype) between step 3 and step 9."""
import collections
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]
import torch  # noqa: E402
from dmayolo.models.yolo import Model  # noqa: E402
from dmayolo.trainer import Trainer  # noqa: E402
from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp, CONFIGS  # noqa: E402

yaml = sys.argv[1] if len(sys.argv) > 1 else 'yolov5l-xs-tr-cbam-spp-bifpn.yaml'
img, bs = 256, 2
torch.manual_seed(0)
m = Model(os.path.join(CONFIGS, yaml), nc=10, act_dtype=torch.bfloat16).cuda().train()
m.hyp = scaled_hyp(HYP_VISDRONE, 10, img)
x = images(bs, img, seed=1, device='cuda')
t = targets(bs, 10, seed=1, device='cuda')
tr = Trainer(m, dict(m.hyp), 64, nb=100)
tr.i = 500


def snap():
    gc.collect()
    ty = collections.Counter(type(o).__name__ for o in gc.get_objects())
    ts = collections.Counter()
    for o in gc.get_objects():
        try:
            if torch.is_tensor(o) and o.is_cuda:
                ts[(tuple(o.shape), str(o.dtype))] += 1
        except Exception:
            pass
    return ty, ts


snaps = {}
for i in range(10):
    loss, _ = tr.step(x, t)
    del loss
    torch.cuda.synchronize()
    print(i, torch.cuda.memory_allocated(), flush=True)
    if i in (3, 9):
        snaps[i] = snap()
(a, ta), (b, tb) = snaps[3], snaps[9]
print('types grown:', {k: b[k] - a[k] for k in b if b[k] != a[k]})
print('tensors grown:', {k: tb[k] - ta[k] for k in tb if tb[k] != ta[k]})
