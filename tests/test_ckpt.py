"""Checkpoint files (dmayolo/utils/ckpt.py): the reference's own state_dicts (captured in
tests/golden by tools/gen_golden.py) load into this build's Model with every key and shape matching, and
save_checkpoint / attempt_load round-trip through weights_only files.  CPU only (no kernels run)."""
import os

import torch

from golden_util import Fixture, load_sd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model(name):
    from dmayolo.models.yolo import Model
    fx = Fixture(name)
    return fx, Model(fx.meta['yaml'], nc=fx.meta['nc'])


def test_reference_state_dicts_load_with_full_key_coverage():
    from dmayolo.utils.ckpt import load_weights
    for name in ('model_v5s', 'model_dma', 'model_c5'):
        fx, m = _model(name)
        ref = fx.group('sd')
        mine = m.state_dict()
        assert set(ref) == set(mine), (name, sorted(set(ref) ^ set(mine))[:5])
        n = load_weights(m, ref)
        assert n == len(ref)
        for k, v in m.state_dict().items():
            torch.testing.assert_close(v.float(), ref[k].float(), rtol=0, atol=0)


def test_save_checkpoint_attempt_load_round_trip(tmp_path):
    from dmayolo.utils.ckpt import save_checkpoint, attempt_load, load_weights
    fx, m = _model('model_v5s')
    load_sd(m, fx.group('sd'))
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9)
    p = str(tmp_path / 'last.pt')
    ckpt = save_checkpoint(p, m, optimizer=opt, epoch=3, best_fitness=0.25)
    assert set(ckpt) >= {'epoch', 'best_fitness', 'model', 'ema', 'updates', 'optimizer', 'wandb_id', 'date'}
    got = torch.load(p, map_location='cpu', weights_only=True)
    assert got['epoch'] == 3 and got['model']['model.0.conv.weight'].dtype == torch.float16
    m2 = attempt_load(p, device='cpu', fuse=False)
    for k, v in m.state_dict().items():
        if v.is_floating_point():
            torch.testing.assert_close(m2.state_dict()[k], v.half().float(), rtol=0, atol=0)
    _, m3 = _model('model_v5s')
    assert load_weights(m3, p, exclude=('anchor',)) == len([k for k in m3.state_dict() if 'anchor' not in k])
    fused = attempt_load(p, device='cpu', fuse=True)
    assert not any(hasattr(mm, 'bn') for mm in fused.model if type(mm).__name__ == 'Conv')


def test_load_weights_takes_model_entry_attempt_load_takes_ema(tmp_path):
    """train.py:148-156 transfers ckpt['model']; attempt_load (experimental.py:128) prefers ckpt['ema']."""
    from dmayolo.utils.ckpt import save_checkpoint, attempt_load, load_weights
    from dmayolo.utils.torch_utils import ModelEMA
    fx, m = _model('model_v5s')
    load_sd(m, fx.group('sd'))
    ema = ModelEMA(m)
    with torch.no_grad():
        for q in ema.ema.parameters():
            q.add_(1.0)
    p = str(tmp_path / 'last.pt')
    save_checkpoint(p, m, ema=ema, half=False)
    _, m2 = _model('model_v5s')
    load_weights(m2, p)
    k = 'model.0.conv.weight'
    torch.testing.assert_close(m2.state_dict()[k], m.state_dict()[k], rtol=0, atol=0)
    m3 = attempt_load(p, device='cpu', fuse=False)
    torch.testing.assert_close(m3.state_dict()[k], ema.ema.state_dict()[k], rtol=0, atol=0)
