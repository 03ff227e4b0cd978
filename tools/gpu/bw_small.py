"""Graph-replayed GPU time of plain device copies at batch-1 activation sizes: the floor a bs1 elementwise kernel
can reach on this box (compare with the per-launch times of the detect trace)."""
import torch

def graph_time(fn, n=50):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay(); torch.cuda.synchronize()
    best = 1e30
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return best

if __name__ == "__main__":
  for mb in (1.2, 4.7, 9.4, 18.9, 37.7, 75.5, 302):
      n = int(mb * 1e6 / 2)
      a = torch.empty(n, dtype=torch.bfloat16, device='cuda').normal_()
      b = torch.empty_like(a)
      us = graph_time(lambda: b.copy_(a))
      print(f'copy {mb:7.1f} MB: {us:8.1f} us  {2 * mb * 1e6 / us / 1e3:7.0f} GB/s (read + write)', flush=True)
