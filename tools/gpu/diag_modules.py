"""Diagnostic: tests/module_parity.py's layer-by-layer parity at a bench shape, printed (product | emulation per
column; see that module).

python tools/gpu/diag_modules.py <yaml> <img> <bs> [layer ids, comma-separated]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd'), os.path.join(ROOT, 'tests')]
from module_parity import layer_parity, fmt  # noqa: E402

if __name__ == '__main__':
    yml, img, bs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    only = [int(v) for v in sys.argv[4].split(',')] if len(sys.argv) > 4 else None
    print(f'{yml} @{img} bs{bs}: layer type | dx rel prod emu | dx norm prod emu | params rel prod emu | params norm '
          f'prod emu | worst param (rel prod / emu)', flush=True)
    for i, name, row in layer_parity(yml, img, bs, only):
        print(fmt(i, name, row), flush=True)
