"""A/B of the fused 1x1 Conv-BN-act backward (dmy_conv1x1_bwd_bn) against the three launches it replaces
(dmy_bn_bwd_apply + dmy_conv_dgrad + dmy_conv_wgrad_ex OIHW/zeroed), cold caches (tune_conv.bench_cold), on the 1x1
layers of DMA-YOLO-l @1536 bs32 and yolov5s @640 bs64 the kernel is built for.

python tools/gpu/bwd1x1_ab.py [acc: 0|1]
One line per shape: three-pass us (apply / dgrad / wgrad), fused us, speedup, fused HBM rate on algorithmic bytes.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'dma-yolo_amd'), os.path.join(ROOT, 'tools', 'gpu')]
import torch  # noqa: E402
from dmayolo.functional import call, ptr, stream  # noqa: E402
from tune_conv import bench_cold  # noqa: E402

# (N, C = fwd in = dx channels, H, W, K = fwd out = dz channels)
SHAPES = [(32, 512, 192, 192, 128), (32, 256, 96, 96, 256), (32, 128, 192, 192, 128), (32, 64, 384, 384, 64), (32, 128, 384, 384, 64),
          (32, 256, 192, 192, 128), (32, 256, 192, 192, 256), (32, 128, 384, 384, 128), (32, 128, 192, 192, 256),
          (64, 64, 160, 160, 64), (64, 128, 80, 80, 128), (64, 256, 40, 40, 256), (64, 128, 80, 80, 64),
          (32, 128, 192, 192, 512), (64, 256, 80, 80, 64)]


def main():
    acc = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    only = os.environ.get('B1_ONLY') == '1'  # profiling: the fused kernel alone (PMC passes)
    shapes = SHAPES if os.environ.get('B1_SET') != 'pmc' else [SHAPES[2], SHAPES[1], SHAPES[3], SHAPES[0]]
    print(f'accumulate={acc}: shape (N C H W K) | apply dgrad wgrad = 3-pass us | fused us | speedup | fused GB/s')
    for N, C, H, W, K in shapes:
        M = N * H * W
        g = torch.Generator(device='cuda').manual_seed(0)
        dy = (torch.randn(M, K, device='cuda', generator=g) * 0.1).bfloat16()
        z = torch.randn(M, K, device='cuda', generator=g).bfloat16()
        x = torch.randn(M, C, device='cuda', generator=g).bfloat16()
        wt = (torch.randn(C, K, device='cuda', generator=g) / K ** 0.5).bfloat16()
        dx = torch.randn(M, C, device='cuda', generator=g).bfloat16()
        dz = torch.empty(M, K, dtype=torch.bfloat16, device='cuda')
        dw = torch.zeros(K, C, device='cuda')
        co = [torch.rand(K, device='cuda', generator=g) + 0.5 for _ in range(7)]
        sc, sh, mu, inv, ca, cb, cc = [ptr(t) for t in co]
        if not call('dmy_conv1x1_bwd_bn_ok', M, K, C, K, C, C, ptr(dy), ptr(z), ptr(x), ptr(dx)):
            print(N, C, H, W, K, 'unsupported')
            continue

        def apply():
            call('dmy_bn_bwd_apply', 1, ptr(z), K, ptr(dy), K, sc, sh, mu, inv, 1, ca, cb, cc, ptr(dz), K, M, K,
                 stream())

        def dgrad():
            call('dmy_conv_dgrad', 1, ptr(dz), ptr(wt), ptr(dx), acc, N, H, W, C, C, K, 1, 1, 1, 0, H, W, K, stream())

        def wgrad():
            call('dmy_conv_wgrad_ex', 1, ptr(x), ptr(dz), ptr(dw), N, H, W, C, C, K, 1, 1, 1, 0, H, W, K, 3, stream())

        def fused():
            call('dmy_conv1x1_bwd_bn', ptr(dy), K, ptr(z), ptr(x), C, ptr(wt), sc, sh, mu, inv, 1, ca, cb, cc,
                 ptr(dx), C, acc, ptr(dw), None, 0, M, K, C, stream())

        ta, td, tw = (bench_cold(apply), bench_cold(dgrad), bench_cold(wgrad)) if not only else (0.0, 0.0, 0.0)
        tf = bench_cold(fused)
        nb = 2 * (2 * M * K + (2 + acc) * M * C + K * C) + 4 * K * C
        print(f'{N:3d} {C:4d} {H:4d} {W:4d} {K:4d} | {ta:7.1f} {td:7.1f} {tw:7.1f} = {ta + td + tw:7.1f} | '
              f'{tf:7.1f} | {(ta + td + tw) / tf:5.2f}x | {nb / tf / 1e3:6.0f}', flush=True)
        del dy, z, x, wt, dx, dz, dw, co
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
