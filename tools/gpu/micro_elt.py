"""Time the HBM-bound NHWC kernels in isolation and print achieved GB/s (algorithmic bytes).

python tools/gpu/micro_elt.py     (bf16; DMA-YOLO-l @1536 bs32 and yolov5s @640 bs64 shapes)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'dma-yolo_amd'))
import torch  # noqa: E402
from dmayolo.functional import call, ptr, stream  # noqa: E402


_SCRIBBLE = []


def bench_cold(fn, n=10):
    """each launch timed alone after a 512 MiB scribble evicted its operands from the Infinity Cache (MICRO_COLD=1:
    the state a layer of the training step finds them in)"""
    if not _SCRIBBLE:
        _SCRIBBLE.append(torch.empty(512 << 20, dtype=torch.uint8, device='cuda'))
    fn()
    tot = 0.0
    for _ in range(n):
        _SCRIBBLE[0].fill_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        tot += e0.elapsed_time(e1)
    return tot / n * 1e3


def bench(fn, n=10):
    if os.environ.get('MICRO_COLD'):
        return bench_cold(fn, n)
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def act(N, C, H, W, ps=None):
    ps = ps or C
    t = torch.randn(N, H, W, ps, device='cuda').bfloat16()
    return t, ps


def report(name, us, nbytes):
    print(f'{name:58s} {us:9.1f} us  {nbytes / us / 1e3:8.1f} GB/s', flush=True)


def main():
    dev = 'cuda'
    if os.environ.get('MICRO_BN_ONLY'):
        return bn(dev)
    for (N, C, H, W) in [(32, 1024, 48, 48), (64, 256, 20, 20)]:
        M = N * H * W
        for ps in (C, 4 * C):
            x, xps = act(N, C, H, W, ps)
            y, yps = act(N, C, H, W, ps)
            arg = torch.empty(M * C, dtype=torch.uint8, device=dev)
            us = bench(lambda: call('dmy_maxpool_fwd', 1, ptr(x), xps, ptr(y), yps, ptr(arg), N, H, W, C, 5, stream()))
            report(f'maxpool_fwd k5 N{N} C{C} {H}x{W} ps{ps}', us, M * C * 5)
            us = bench(lambda: call('dmy_maxpool_bwd', 1, ptr(y), yps, ptr(arg), ptr(x), xps, 0, N, H, W, C, 5, stream()))
            report(f'maxpool_bwd k5 N{N} C{C} {H}x{W} ps{ps}', us, M * C * 5)
    bn(dev)


def bn(dev):
    for (N, C, H, W) in [(32, 64, 768, 768), (32, 256, 96, 96), (32, 128, 192, 192), (64, 64, 160, 160),
                         (64, 32, 320, 320), (64, 128, 40, 40)]:
        M = N * H * W
        z, _ = act(N, C, H, W)
        y, _ = act(N, C, H, W)
        dy, _ = act(N, C, H, W)
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev)
        mu = torch.randn(C, device=dev)
        iv = torch.rand(C, device=dev) + 0.5
        P = call('dmy_bn_reduce_rows', 1, ptr(z), C, ptr(dy), C, M, C)
        pdb = torch.empty(P * C, device=dev)
        pdg = torch.empty(P * C, device=dev)
        us = bench(lambda: call('dmy_bn_act_fwd', 1, ptr(z), C, ptr(sc), ptr(sh), 1, None, 0, ptr(y), C, M, C, stream()))
        report(f'bn_act_fwd silu M{M} C{C}', us, 4 * M * C)
        us = bench(lambda: call('dmy_bn_bwd_reduce', 1, ptr(z), C, ptr(dy), C, ptr(sc), ptr(sh), ptr(mu), ptr(iv), 1,
                                M, C, ptr(pdb), ptr(pdg), stream()))
        report(f'bn_bwd_reduce silu M{M} C{C} (P={P})', us, 4 * M * C)
        us = bench(lambda: call('dmy_bn_bwd_apply', 1, ptr(z), C, ptr(dy), C, ptr(sc), ptr(sh), ptr(mu), ptr(iv), 1,
                                ptr(sc), ptr(sh), ptr(mu), ptr(y), C, M, C, stream()))
        report(f'bn_bwd_apply silu M{M} C{C}', us, 6 * M * C)
        us = bench(lambda: y.copy_(z))
        report(f'torch copy_ M{M} C{C}', us, 4 * M * C)


if __name__ == '__main__':
    main()
