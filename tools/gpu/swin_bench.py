"""Time the bf16 window-attention kernels (dmy_winattn_fwd / _bwd) at the DMA-YOLO-l @1536 bs32 C3STR shapes.
python tools/gpu/swin_bench.py  -> per shape: us per call and the algorithmic HBM rate (qkv + out / + dout + dqkv)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'dma-yolo_amd'))
import torch  # noqa: E402
from dmayolo.functional import call, ptr, stream  # noqa: E402


def bench(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for (B, H, W, nh) in [(32, 192, 192, 4), (32, 96, 96, 8), (32, 48, 48, 16)]:
    C = 32 * nh
    qkv = torch.randn(B, H, W, 3 * C, device='cuda').bfloat16()
    dout = torch.randn(B, H, W, C, device='cuda').bfloat16()
    table = torch.randn(225, nh, device='cuda') * 0.1
    o = torch.empty(B, H, W, C, dtype=torch.bfloat16, device='cuda')
    dq = torch.empty_like(qkv)
    G = call('dmy_winattn_bwd_groups', B, H, W, nh)
    part = torch.empty(G * nh * 225, device='cuda')
    dtab = torch.empty(225, nh, device='cuda')
    for shift in (0, 4):
        tf = bench(lambda: call('dmy_winattn_fwd', 1, ptr(qkv), ptr(table), ptr(o), B, H, W, C, nh, shift, C ** -0.5,
                                stream()))
        tb = bench(lambda: call('dmy_winattn_bwd', 1, ptr(qkv), ptr(dout), ptr(table), ptr(dq), ptr(part), ptr(dtab), B,
                                H, W, C, nh, shift, C ** -0.5, stream()))
        bf, bb = 2.0 * B * H * W * 4 * C, 2.0 * B * H * W * 7 * C
        print(f'winattn B{B} {H}x{W} C{C} nh{nh} shift{shift}: fwd {tf:8.1f} us {bf / tf / 1e3:6.0f} GB/s   '
              f'bwd {tb:8.1f} us {bb / tb / 1e3:6.0f} GB/s', flush=True)
