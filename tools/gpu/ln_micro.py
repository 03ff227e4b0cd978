"""Graph-replayed GPU time of dmy_layernorm_fwd at the batch-1 C3STR sizes (and 32x of them) next to a plain copy of
the same bytes: is the bs1 LayerNorm time the kernel or the size?"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'dma-yolo_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tools', 'gpu'))
import torch  # noqa: E402
from dmayolo.functional import call, ptr, stream  # noqa: E402
from bw_small import graph_time  # noqa: E402

def main():
  for M, C in [(36864, 128), (9216, 256), (2304, 512), (32 * 36864, 128)]:
      x = torch.randn(M, C, device='cuda').bfloat16()
      y = torch.empty_like(x)
      w, b = torch.ones(C, device='cuda'), torch.zeros(C, device='cuda')
      mu, rs = torch.empty(M, device='cuda'), torch.empty(M, device='cuda')
      ln = graph_time(lambda: call('dmy_layernorm_fwd', 1, ptr(x), C, ptr(w), ptr(b), ptr(y), ptr(mu), ptr(rs), M, C,
                                   1e-5, stream()))
      cp = graph_time(lambda: y.copy_(x))
      mb = 2 * x.numel() * 2 / 1e6
      print(f'M={M:8d} C={C:4d} ({mb:6.1f} MB r+w): layernorm {ln:7.1f} us ({mb / ln * 1e3:6.0f} GB/s), copy {cp:6.1f} us',
            flush=True)


if __name__ == '__main__' and len(sys.argv) == 1:
    main()

if __name__ == '__main__' and len(sys.argv) > 1:  # plain launches of the first shape (for rocprofv3 --pmc)
    M, C = 36864, 128
    x = torch.randn(M, C, device='cuda').bfloat16()
    y = torch.empty_like(x)
    w, b = torch.ones(C, device='cuda'), torch.zeros(C, device='cuda')
    mu, rs = torch.empty(M, device='cuda'), torch.empty(M, device='cuda')
    for _ in range(int(sys.argv[1])):
        call('dmy_layernorm_fwd', 1, ptr(x), C, ptr(w), ptr(b), ptr(y), ptr(mu), ptr(rs), M, C, 1e-5, stream())
    torch.cuda.synchronize()
