"""Time the LDS max-pool kernels (dmy_maxpool_fwd / _bwd, k = 5) at the SPPFCSPC shapes of DMA-YOLO-l @1536 bs32
(512 channels @48^2) and yolov5s @640 bs64 (256 @20^2), dense and as concat-buffer slices (pixel stride 4 C).
python tools/gpu/pool_micro.py  -> per shape: us per call and the algorithmic HBM rate."""
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


for (N, H, W, C) in [(32, 48, 48, 512), (64, 20, 20, 256), (32, 96, 96, 256)]:
    for mult in (1, 4):
        ps = C * mult
        x = torch.randn(N * H * W * ps, device='cuda').bfloat16()
        y = torch.empty(N * H * W * ps, device='cuda', dtype=torch.bfloat16)
        arg = torch.empty(N * H * W * C, device='cuda', dtype=torch.uint8)
        dx = torch.zeros(N * H * W * ps, device='cuda', dtype=torch.bfloat16)
        tf = bench(lambda: call('dmy_maxpool_fwd', 1, ptr(x), ps, ptr(y), ps, ptr(arg), N, H, W, C, 5, stream()))
        tb = bench(lambda: call('dmy_maxpool_bwd', 1, ptr(y), ps, ptr(arg), ptr(dx), ps, 1, N, H, W, C, 5, stream()))
        e = N * H * W * C
        print(f'maxpool k5 N{N} {H}x{W} C{C} pixel stride {ps}: fwd {tf:7.1f} us {5 * e / tf / 1e3:6.0f} GB/s   '
              f'bwd (acc) {tb:7.1f} us {7 * e / tb / 1e3:6.0f} GB/s', flush=True)
