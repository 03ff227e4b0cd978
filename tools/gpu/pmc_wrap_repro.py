"""Product-free reproduction for the rocprofv3 --pmc SIGSEGV: only torch kernels, no dmayolo
library.  Launches `n` tiny elementwise kernels on one stream (default 40,000: more AQL packets than a 1 MiB HSA queue
ring holds, 16,384 x 64 B, several times over), printing progress.  Run under
rocprofv3 --kernel-trace --pmc FETCH_SIZE -- python tools/gpu/pmc_wrap_repro.py [n]"""
import sys

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40000
x = torch.zeros(1024, device='cuda')
for i in range(n):
    x.add_(1.0)
    if i % 5000 == 4999:
        torch.cuda.synchronize()
        print(f'{i + 1} kernels, x[0] = {float(x[0])}', flush=True)
torch.cuda.synchronize()
print('done', float(x[0]))
