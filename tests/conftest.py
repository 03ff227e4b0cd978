import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'dma-yolo_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)
# The GPU tests' fp32 oracle / emulation runs use torch convolutions (MIOpen).  On a fresh box MIOpen's default find
# mode compiles kernels for every new conv configuration: ~100 s per bench-shape model (config 5 @1920 bs2: 80.6 s of
# its first forward + backward, 1.8 s with FAST; profiles/r06/miopen_probe.log).  FAST picks from its heuristics without
# that search; the oracle is fp32 either way (TF32 off) and every GPU bound is a tolerance, not a bit pattern.
os.environ.setdefault('MIOPEN_FIND_MODE', 'FAST')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU and the built HIP library')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason='no GPU in this container')
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)
