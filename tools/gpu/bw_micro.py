"""HBM streaming rates of the BN elementwise kernels against plain copies, HIP events, warm (no cache flush: the
tensors are 4-8x the 256 MB Infinity Cache).  python tools/gpu/bw_micro.py [M] [C]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'dma-yolo_amd')]
import torch  # noqa: E402
from dmayolo.functional import call, ptr, stream  # noqa: E402
from dmayolo._lib import ACT_SILU  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 32 * 192 * 192
C = int(sys.argv[2]) if len(sys.argv) > 2 else 128
dev = 'cuda'
z = torch.randn(M, C, device=dev).bfloat16()
dy = torch.randn(M, C, device=dev).bfloat16()
y = torch.empty_like(z)
f = lambda: torch.rand(C, device=dev) + 0.5  # noqa: E731
sc, sh, mu, inv, ca, cb, cc = f(), f(), f(), f(), f(), f(), f()
P = call('dmy_bn_reduce_rows', 1, ptr(z), C, ptr(dy), C, M, C)
pdb, pdg = torch.empty(P * C, device=dev), torch.empty(P * C, device=dev)
E = M * C * 2


def t(fn, n=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


cases = [
    ('torch copy_ (r+w)', lambda: y.copy_(z), 2 * E),
    ('torch add (2r+w)', lambda: torch.add(z, dy, out=y), 3 * E),
    ('bn_act_fwd (r+w)', lambda: call('dmy_bn_act_fwd', 1, ptr(z), C, ptr(sc), ptr(sh), ACT_SILU, None, 0, ptr(y), C, M,
                                      C, stream()), 2 * E),
    ('bn_bwd_reduce (2r)', lambda: call('dmy_bn_bwd_reduce', 1, ptr(z), C, ptr(dy), C, ptr(sc), ptr(sh), ptr(mu),
                                        ptr(inv), ACT_SILU, M, C, ptr(pdb), ptr(pdg), stream()), 2 * E),
    ('bn_bwd_apply (2r+w)', lambda: call('dmy_bn_bwd_apply', 1, ptr(z), C, ptr(dy), C, ptr(sc), ptr(sh), ptr(mu),
                                         ptr(inv), ACT_SILU, ptr(ca), ptr(cb), ptr(cc), ptr(y), C, M, C, stream()), 3 * E),
]
print(f'M={M} C={C} ({E / 1e6:.0f} MB per tensor)')
for name, fn, byt in cases:
    us = t(fn)
    print(f'{name:22s} {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s')
