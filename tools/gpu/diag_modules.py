"""Diagnostic: tests/module_parity.py's layer-by-layer parity at a bench shape, printed (product | emulation per
column; see that module).

python tools/gpu/diag_modules.py <yaml> <img> <bs> [layer ids, comma-separated | all] [product: bf16 | fp8 | fp32]
(DIAG_FP16=1: also the fp16 autocast emulation per layer)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd'), os.path.join(ROOT, 'tests')]
from module_parity import layer_parity, fmt  # noqa: E402

if __name__ == '__main__':
    yml, img, bs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    only = [int(v) for v in sys.argv[4].split(',')] if len(sys.argv) > 4 and sys.argv[4] != 'all' else None
    prod = sys.argv[5] if len(sys.argv) > 5 else 'bf16'
    print(f'{yml} @{img} bs{bs}: layer type | output rel prod emu | dx rel prod emu | dx norm prod emu | params rel '
          f'prod emu | params norm prod emu | worst param (rel prod / emu)', flush=True)
    print(f'product: {prod}', flush=True)
    for i, name, row in layer_parity(yml, img, bs, only, fp16=os.environ.get('DIAG_FP16') == '1', prod=prod):
        print(fmt(i, name, row), flush=True)
