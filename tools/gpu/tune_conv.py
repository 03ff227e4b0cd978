"""Time single conv launches (fwd / dgrad / wgrad, bf16) for a list of layer shapes.

python tools/gpu/tune_conv.py [shape-set]   (env knobs such as DMY_WGRAD_TARGET are read by the library)
Prints one line per (kind, shape): mean us over 20 launches and TFLOP/s.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'dma-yolo_amd'))
import torch  # noqa: E402
from dmayolo.functional import call, ptr, stream, prep_weight  # noqa: E402

SETS = {
    'dma': [(32, 256, 96, 96, 256, 3, 1), (32, 1024, 48, 48, 1024, 3, 1), (32, 128, 192, 192, 128, 3, 1),
            (32, 64, 768, 768, 64, 3, 1), (32, 64, 384, 384, 64, 3, 1), (32, 256, 96, 96, 256, 1, 1),
            (32, 512, 96, 96, 512, 3, 1), (32, 512, 192, 192, 128, 1, 1)],
    'narrow': [(64, 8, 640, 640, 32, 6, 2), (64, 64, 80, 80, 64, 3, 1), (64, 32, 160, 160, 32, 3, 1),
               (64, 32, 320, 320, 64, 3, 2), (64, 256, 80, 80, 64, 1, 1), (64, 64, 160, 160, 32, 1, 1)],
    'p1': [(32, 256, 96, 96, 256, 1, 1), (32, 512, 192, 192, 128, 1, 1), (32, 1024, 96, 96, 256, 1, 1),
           (32, 256, 192, 192, 128, 1, 1), (32, 1024, 48, 48, 512, 1, 1), (32, 512, 96, 96, 512, 1, 1),
           (64, 256, 40, 40, 128, 1, 1), (64, 512, 20, 20, 256, 1, 1)],
    'p1dma': [(32, 512, 192, 192, 128, 1, 1), (32, 128, 192, 192, 512, 1, 1), (32, 1024, 96, 96, 256, 1, 1),
              (32, 256, 96, 96, 256, 1, 1), (32, 128, 192, 192, 128, 1, 1), (32, 128, 384, 384, 128, 1, 1),
              (32, 2048, 48, 48, 1024, 1, 1), (32, 256, 96, 96, 1024, 1, 1), (32, 1280, 96, 96, 256, 1, 1)],
    's2': [(32, 64, 768, 768, 128, 3, 2), (32, 128, 384, 384, 256, 3, 2), (32, 256, 192, 192, 512, 3, 2),
           (64, 32, 320, 320, 64, 3, 2), (64, 64, 160, 160, 128, 3, 2), (64, 128, 80, 80, 256, 3, 2)],
    'c128': [(32, 128, 192, 192, 128, 3, 1), (32, 128, 384, 384, 128, 3, 1), (32, 512, 192, 192, 128, 1, 1),
             (32, 128, 192, 192, 128, 1, 1), (32, 128, 384, 384, 128, 1, 1), (8, 128, 240, 240, 128, 3, 1),
             (64, 128, 80, 80, 128, 3, 1), (64, 256, 80, 80, 128, 1, 1), (32, 256, 192, 192, 128, 1, 1)],
    'p1s': [(32, 128, 192, 192, 512, 1, 1), (32, 512, 192, 192, 128, 1, 1), (32, 256, 96, 96, 256, 1, 1),
            (32, 128, 192, 192, 128, 1, 1), (32, 64, 384, 384, 64, 1, 1), (32, 128, 384, 384, 64, 1, 1),
            (32, 64, 384, 384, 128, 1, 1), (32, 128, 192, 192, 384, 1, 1), (32, 256, 192, 192, 128, 1, 1),
            (32, 128, 192, 192, 256, 1, 1), (64, 64, 160, 160, 64, 1, 1), (64, 128, 80, 80, 128, 1, 1)],
    'q2h': [(32, 128, 384, 384, 256, 3, 2), (64, 128, 80, 80, 256, 3, 2), (8, 128, 480, 480, 256, 3, 2)],
    'q2r': [(32, 64, 768, 768, 128, 3, 2), (64, 64, 160, 160, 128, 3, 2), (8, 64, 960, 960, 128, 3, 2)],
    'q2s': [(64, 32, 320, 320, 64, 3, 2), (32, 32, 384, 384, 64, 3, 2), (16, 32, 640, 640, 64, 3, 2)],
    's2v5s': [(64, 256, 40, 40, 512, 3, 2), (64, 256, 40, 40, 256, 3, 2), (64, 128, 80, 80, 256, 3, 2), (64, 64, 160, 160, 128, 3, 2)],
    'stem': [(32, 16, 768, 768, 64, 3, 1), (64, 16, 320, 320, 32, 3, 1), (8, 16, 960, 960, 64, 3, 1)],
    # batch-1 1536 inference layers (dmy_conv_fwd_act path, 'infer' kind)
    'det': [(1, 256, 96, 96, 256, 1, 1), (1, 128, 192, 192, 128, 1, 1), (1, 128, 192, 192, 512, 1, 1),
            (1, 1024, 96, 96, 256, 1, 1), (1, 512, 192, 192, 128, 1, 1), (1, 256, 192, 192, 256, 1, 1),
            (1, 256, 96, 96, 1024, 1, 1), (1, 512, 96, 96, 512, 1, 1), (1, 1024, 48, 48, 1024, 1, 1),
            (1, 512, 48, 48, 512, 1, 1), (1, 128, 192, 192, 128, 3, 1), (1, 256, 96, 96, 256, 3, 1),
            (1, 64, 384, 384, 64, 3, 1), (1, 512, 48, 48, 512, 3, 1), (1, 128, 384, 384, 128, 1, 1)],
    'halo': [(32, 64, 768, 768, 64, 3, 1), (32, 64, 384, 384, 64, 3, 1), (8, 64, 256, 256, 64, 3, 1)],
    # the stride-2 layers of DMA-YOLO-l @1536 bs32 (SCConv k4 and the downsampling convs) and of yolov5s @640 bs64
    's2dma': [(32, 64, 768, 768, 128, 3, 2), (32, 128, 384, 384, 256, 3, 2), (32, 256, 192, 192, 512, 3, 2),
              (32, 512, 96, 96, 1024, 3, 2), (32, 256, 192, 192, 256, 3, 2), (64, 32, 320, 320, 64, 3, 2),
              (64, 64, 160, 160, 128, 3, 2), (64, 128, 80, 80, 256, 3, 2), (64, 256, 40, 40, 512, 3, 2)],
    # every >= 256-column GEMM view of DMA-YOLO-l @1536 bs32 on the 256 x 256 tiles (conv_fwd_w / conv_fwd_8p)
    'wide': [(32, 256, 96, 96, 256, 3, 1), (32, 512, 96, 96, 512, 3, 1), (32, 1024, 48, 48, 1024, 3, 1),
             (32, 512, 48, 48, 512, 3, 1), (32, 1024, 48, 48, 1024, 1, 1), (32, 2048, 48, 48, 1024, 1, 1),
             (32, 512, 96, 96, 512, 1, 1), (32, 256, 96, 96, 1024, 1, 1), (32, 256, 96, 96, 768, 1, 1),
             (32, 4096, 48, 48, 1024, 1, 1)],
    'one': [(32, 256, 96, 96, 256, 3, 1), (32, 1024, 48, 48, 1024, 3, 1)],
    # the k > 1 GEMM views of DMA-YOLO-l @1536 bs32 with >= 256 columns (wide / 288-row / quad tiles)
    'quad': [(32, 256, 96, 96, 256, 3, 1), (32, 512, 96, 96, 512, 3, 1), (32, 1024, 48, 48, 1024, 3, 1),
             (32, 512, 48, 48, 512, 3, 1), (32, 256, 192, 192, 256, 3, 1), (32, 128, 384, 384, 256, 3, 2),
             (32, 256, 192, 192, 512, 3, 2), (32, 256, 192, 192, 256, 3, 2), (32, 512, 96, 96, 1024, 3, 2),
             (32, 512, 96, 96, 512, 3, 2)],
    # the slowest batch-1 @1536 detect layers (round-5 trace): SPPFCSPC at 48^2, the s2 3x3 / 96^2 C3 layers
    'det48': [(1, 512, 48, 48, 512, 3, 1), (1, 2048, 48, 48, 512, 1, 1), (1, 1024, 48, 48, 512, 1, 1),
              (1, 1024, 48, 48, 1024, 1, 1), (1, 512, 96, 96, 1024, 3, 2), (1, 256, 96, 96, 256, 3, 1),
              (1, 256, 192, 192, 512, 3, 2), (1, 128, 384, 384, 256, 3, 2), (1, 64, 768, 768, 128, 3, 2)],
    'v5s': [(64, 128, 40, 40, 128, 3, 1), (64, 64, 80, 80, 64, 3, 1), (64, 256, 20, 20, 256, 3, 1),
            (64, 512, 20, 20, 256, 1, 1), (64, 32, 160, 160, 32, 3, 1), (64, 64, 160, 160, 32, 1, 1)],
}


_SCRIBBLE = []


def bench_cold(fn, n=10):
    """each launch timed alone after a 512 MiB scribble has pushed its operands out of the Infinity Cache and the
    L2s (the state a layer of the training step finds them in); mean us of the n launches"""
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


def bench_graph(fn, n=50):
    """n launches captured in one HIP graph and replayed: the GPU-side time per launch without the host launch cost
    (TUNE_GRAPH=1; the batch-1 shapes are otherwise CPU launch-bound under ~20 us)"""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return best


def bench(fn, n=20):
    if os.environ.get('TUNE_COLD'):
        return bench_cold(fn)
    if os.environ.get('TUNE_GRAPH'):
        return bench_graph(fn)
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else 'dma'
    kinds = (sys.argv[2] if len(sys.argv) > 2 else 'fwd,dgrad,wgrad').split(',')
    for (N, C, H, W, K, k, s) in SETS[which]:
        p = k // 2
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, C, H, W, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, K, OH, OW, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
        w = torch.randn(K, C, k, k, device='cuda') * 0.05
        wf, wt = prep_weight(w, torch.bfloat16, True)
        y = torch.empty_like(dy)
        dx = torch.empty_like(x)
        M = N * OH * OW
        P = call('dmy_conv_fwd_bn_rows', 1, ptr(x), ptr(wf), None, ptr(y), N, H, W, C, C, K, k, k, s, p, OH, OW, K)
        ps, pq = torch.empty(P * K, device='cuda'), torch.empty(P * K, device='cuda')
        dwo = torch.empty(K * C * k * k, device='cuda')
        fl = 2.0 * M * K * C * k * k
        by = 2.0 * (N * H * W * C + M * K)  # algorithmic bytes: the gathered tensor once + the output / dy once
        fns = {
            'fwd': lambda: call('dmy_conv_fwd', 1, ptr(x), ptr(wf), None, ptr(y), ptr(ps), ptr(pq), N, H, W, C, C, K, k,
                                k, s, p, OH, OW, K, stream()),
            'fwdnb': lambda: call('dmy_conv_fwd', 1, ptr(x), ptr(wf), None, ptr(y), None, None, N, H, W, C, C, K, k,
                                  k, s, p, OH, OW, K, stream()),
            'dgrad': lambda: call('dmy_conv_dgrad', 1, ptr(dy), ptr(wt), ptr(dx), 0, N, H, W, C, C, K, k, k, s, p, OH,
                                  OW, K, stream()),
            'wgrad': lambda: call('dmy_conv_wgrad', 1, ptr(x), ptr(dy), ptr(dwo), N, H, W, C, C, K, k, k, s, p, OH, OW,
                                  K, stream()),
        }
        if 'infer' in kinds:  # eval forward: BN scale / shift + SiLU epilogue, split-K workspace when the plan splits
            ne = call('dmy_conv_fwd_splitk_elems', 1, ptr(x), ptr(wf), ptr(y), N, H, W, C, C, K, k, k, s, p, OH, OW, K)
            wsi = torch.empty(max(ne, 1), device='cuda')
            sc, sh = torch.rand(K, device='cuda') + 0.5, torch.randn(K, device='cuda') * 0.1
            fns['infer'] = lambda: call('dmy_conv_fwd_act_ws', 1, ptr(x), ptr(wf), None, ptr(y), N, H, W, C, C, K, k, k,
                                        s, p, OH, OW, K, ptr(sc), ptr(sh), 1, None, 0, ptr(wsi), ne, stream())
        if 'wgrad_det' in kinds:  # deterministic form: split partials to a workspace, reduced in split order
            ne = call('dmy_conv_wgrad_ws_elems', 1, ptr(x), ptr(dy), N, H, W, C, C, K, k, k, s, p, OH, OW, K, 0)
            wsd = torch.empty(max(ne, 1), device='cuda')
            fns['wgrad_det'] = lambda: call('dmy_conv_wgrad_det', 1, ptr(x), ptr(dy), ptr(dwo), N, H, W, C, C, K, k, k, s,
                                            p, OH, OW, K, 0, ptr(wsd), ne, stream())
        if 'mm' in kinds and k == 1:  # vendor GEMM of the same 1x1 problem (torch.matmul -> hipBLASLt), a reference point only
            a2, b2 = x.permute(0, 2, 3, 1).reshape(-1, C), wf.view(K, C).t()
            y2 = torch.empty(a2.shape[0], K, dtype=torch.bfloat16, device='cuda')
            fns['mm'] = lambda: torch.matmul(a2, b2, out=y2)
        if 'copy' in kinds:  # calibration: a torch copy moving the same bytes as the 1x1 forward (read x, write y)
            xf_ = x.permute(0, 2, 3, 1).reshape(-1)
            yf_ = torch.empty(N * OH * OW * K, dtype=torch.bfloat16, device='cuda')
            n_ = min(xf_.numel(), yf_.numel())
            fns['copy'] = lambda: yf_[:n_].copy_(xf_[:n_])
        if 'fill' in kinds:  # calibration: write-only stream of the output's bytes
            yfl_ = torch.empty(N * OH * OW * K, dtype=torch.bfloat16, device='cuda')
            fns['fill'] = lambda: yfl_.fill_(1.0)
        if 'bcast' in kinds and k == 1 and K % C == 0:  # calibration: the 1x1 byte pattern (read x once, write y once)
            xb_ = x.permute(0, 2, 3, 1).reshape(-1, 1, C)
            yb_ = torch.empty(N * OH * OW, K // C, C, dtype=torch.bfloat16, device='cuda')
            fns['bcast'] = lambda: yb_.copy_(xb_.expand(-1, K // C, C))
        for kind in kinds:
            if (kind == 'mm' and k != 1) or kind not in fns:
                continue
            us = bench(fns[kind])
            print(f'{kind:6s} N{N} C{C} {H}x{W} K{K} k{k} s{s}: {us:9.1f} us {fl / us / 1e6:8.1f} TFLOP/s '
                  f'{by / us / 1e3:7.0f} GB/s', flush=True)


if __name__ == '__main__':
    main()
