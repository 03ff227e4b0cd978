"""Checkpoint files: the reference's ckpt dict (train.py:515-522) with the model /
EMA entries stored as state_dicts, plus attempt_load (models/experimental.py:113-153) and intersect_dicts
(utils/torch_utils.py:156-158).

The reference pickles whole nn.Module objects ('model': deepcopy(de_parallel(model)).half()).  Loading
such a file executes the pickled class references, so this build never reads one with a pickle-capable
loader: it writes and reads state_dicts only (torch.load(..., weights_only=True)), whose keys are the
reference's own `model.{i}.…` (Model / parse_model keep the layer numbering and parameter names).  A
reference .pt is converted once, on a machine that trusts it, with
`torch.save(torch.load(pt)['model'].float().state_dict(), sd_path)`; load_weights() then takes sd_path.
"""
from datetime import datetime

import torch

from ..models.yolo import Model


def intersect_dicts(da, db, exclude=()):
    """utils/torch_utils.py:156-158: entries of da whose key is in db with the same shape, minus `exclude`."""
    return {k: v for k, v in da.items() if k in db and not any(x in k for x in exclude) and v.shape == db[k].shape}


def save_checkpoint(path, model, ema=None, optimizer=None, epoch=-1, best_fitness=0.0, half=True):
    """train.py:515-522 with state_dicts in 'model' / 'ema' (fp16 as the reference's .half(); BN counters
    and other integer buffers keep their dtype)."""
    def sd(m):
        m = m.module if hasattr(m, 'module') else m
        return {k: (v.detach().half() if half and v.is_floating_point() else v.detach()).cpu()
                for k, v in m.state_dict().items()}

    ckpt = {'epoch': epoch,
            'best_fitness': float(best_fitness) if best_fitness is not None else None,
            'model': sd(model),
            'ema': sd(ema.ema) if ema is not None else None,
            'updates': ema.updates if ema is not None else 0,
            'optimizer': optimizer.state_dict() if optimizer is not None else None,
            'wandb_id': None,
            'date': datetime.now().isoformat(),
            'yaml': (model.module if hasattr(model, 'module') else model).yaml}
    torch.save(ckpt, path)
    return ckpt


def load_weights(model, path_or_sd, exclude=(), key='model'):
    """Transfer weights into `model` as train.py:148-156 does (intersect_dicts on matching keys / shapes);
    returns the number of tensors loaded.  `path_or_sd`: a state_dict, or a file holding one or a ckpt dict
    written by save_checkpoint (read with weights_only=True).  From a ckpt dict the `key` entry is taken:
    'model' as the reference's pretrained / resume path (train.py:148-156: ckpt['model']); attempt_load
    passes 'ema' (models/experimental.py:128)."""
    sd = path_or_sd
    if not isinstance(sd, dict):
        sd = torch.load(sd, map_location='cpu', weights_only=True)
    if isinstance(sd.get('model'), dict):  # a ckpt dict, not a bare state_dict
        sd = sd[key] if sd.get(key) is not None else sd['model']
    sd = {k: v.float() if v.is_floating_point() else v for k, v in sd.items()}
    csd = intersect_dicts(sd, model.state_dict(), exclude=exclude)
    model.load_state_dict(csd, strict=False)
    return len(csd)


def attempt_load(path, device='cuda', fuse=True, act_dtype=torch.float32):
    """models/experimental.py:113-153 for one save_checkpoint file: rebuild the Model from the stored yaml,
    load 'ema' if present else 'model' (fp32), fuse BN into the YAML Conv layers, eval mode."""
    ckpt = torch.load(path, map_location='cpu', weights_only=True)
    model = Model(ckpt['yaml'], act_dtype=act_dtype)
    load_weights(model, ckpt, key='ema')  # ckpt['ema'] or ckpt['model'] (experimental.py:128)
    model = model.to(device)
    if fuse:
        model.fuse()
    return model.eval()
