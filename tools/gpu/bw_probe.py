"""HBM write / copy rates for the 1x1-conv analysis: fill (write only), copy, and the 1x1 conv shapes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'dma-yolo_amd'))
import torch


def t(fn, n=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


for nbytes in (302e6, 1.2e9):
    n = int(nbytes // 2)
    a = torch.empty(n, dtype=torch.bfloat16, device='cuda')
    b = torch.empty(n, dtype=torch.bfloat16, device='cuda')
    s = t(lambda: a.fill_(1.0))
    print(f'fill  {nbytes/1e6:.0f} MB: {nbytes / s / 1e12:.2f} TB/s write')
    s = t(lambda: b.copy_(a))
    print(f'copy  {nbytes/1e6:.0f} MB: {2 * nbytes / s / 1e12:.2f} TB/s (read + write)')
