"""List the ATen ops a training step still dispatches (forward + loss + backward), with shapes and the module
stack of the forward ones -- to find stray elementwise kernels in the timed step.
python tools/gpu/diag_aten.py [config] [batch]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
import bench  # noqa: E402
from dmayolo.synthetic import images, targets  # noqa: E402
from dmayolo.utils.loss import ComputeLoss  # noqa: E402

SKIP = ('empty', 'view', 'as_strided', 'detach', '_to_copy', 'slice', 'select', 'permute', 'reshape', 'unsqueeze',
        'squeeze', 'expand', 'alias', 'split', 'unbind', 't.', 'transpose', 'lift_fresh', 'set_', 'zeros_like',
        'empty_like', 'new_empty', 'sym_', 'is_', 'size', 'stride', 'storage_offset', 'record_stream', '_unsafe_view')


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if not any(s in name for s in SKIP):
            shp = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor))
            dt = next((str(a.dtype).replace('torch.', '') for a in args if isinstance(a, torch.Tensor)), '')
            self.c[(name, dt, shp[:2])] += 1
        return func(*args, **(kwargs or {}))


cfg = sys.argv[1] if len(sys.argv) > 1 else 'dma-1536'
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
c = list(bench.CONFIGS[cfg])
m = bench.build(c, torch.bfloat16, torch.device('cuda', 0)).train()
cl = ComputeLoss(m)
x = images(bs, c[2], seed=1, device='cuda')
tg = targets(bs, c[1], seed=1, device='cuda')
for it in range(2):
    log = Log()
    with log:
        pred = m(x)
        loss, _ = cl(pred, tg)
        loss.backward()
    torch.cuda.synchronize()
print(f'{cfg} bs{bs}: ATen ops of one step (2nd iteration), largest first operand first')


def numel(shp):
    n = 1
    for d in (shp[0] if shp else ()):
        n *= d
    return n


for (name, dt, shp), n in sorted(log.c.items(), key=lambda kv: -numel(kv[0][2])):
    print(f'{n:4d}  {name:40s} {dt:9s} {shp}')
