import sys, torch
sys.path.insert(0, 'tests'); sys.path.insert(0, 'dma-yolo_amd'); sys.path.insert(0, '.')
from gpu_util import product_modules, run_case, rel_err
from test_oracle_golden import MODS
for name in ('c3tr_a', 'c3tr_b'):
    fx, res = run_case(name, product_modules(), 'cuda', dtype=torch.bfloat16)
    _, r32 = run_case(name, product_modules(), 'cuda', dtype=torch.float32)
    _, ref = run_case(name, MODS, 'cpu')
    gmax = max(float(b.norm()) for b in ref['gp'].values())
    print(name, 'out', rel_err(res['out'][0], ref['out'][0]), 'gin', rel_err(res['gin'][0], ref['gin'][0]), 'gmax', gmax)
    for k, b in ref['gp'].items():
        e16 = float((res['gp'][k] - b).norm()) / max(float(b.norm()), 1e-2 * gmax)
        e32 = float((r32['gp'][k] - b).norm()) / max(float(b.norm()), 1e-2 * gmax)
        print(f'  {k:32s} norm {float(b.norm()):9.4f}  bf16 {e16:.4f}  fp32 {e32:.2e}')
