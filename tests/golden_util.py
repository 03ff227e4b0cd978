"""Helpers to load tests/golden/*.npz fixtures (captured from the reference by tools/gen_golden.py)."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


class Fixture:
    def __init__(self, name):
        self.name = name
        self.z = np.load(os.path.join(GOLDEN, f'{name}.npz'), allow_pickle=False)
        self.meta = json.loads(str(self.z['meta'])) if 'meta' in self.z.files else {}

    def t(self, key, dtype=None):
        v = torch.from_numpy(np.array(self.z[key]))
        if dtype is not None:
            v = v.to(dtype)
        elif v.dtype == torch.float16:
            v = v.float()
        return v

    def group(self, prefix):
        n = len(prefix) + 1
        return {k[n:]: self.t(k) for k in self.z.files if k.startswith(prefix + '.')}

    def seq(self, prefix):
        g = self.group(prefix)
        return [g[str(i)] for i in range(len(g))]

    def has(self, key):
        return key in self.z.files


def golden_names(prefix):
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith(prefix) and f.endswith('.npz'))


def load_sd(mod, sd):
    """Load a golden state_dict, keeping the module's own dtype for integer buffers."""
    own = mod.state_dict()
    fixed = {}
    for k, v in sd.items():
        fixed[k] = v.to(own[k].dtype) if k in own else v
    missing, unexpected = mod.load_state_dict(fixed, strict=False)
    assert not unexpected, unexpected
    assert not [k for k in missing if not k.endswith('num_batches_tracked')], missing
