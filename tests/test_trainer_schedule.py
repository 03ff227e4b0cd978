"""CPU: dmayolo.trainer.Trainer's host-side schedule (warmup interpolation of accumulate / lr / momentum, LambdaLR
one_cycle or linear, weight-decay scaling, Adam's inherited 3e-4) against the loop restatement in oracle/train.py
(train.py:189-235, 345, 352, 408-422, 466-468).  No kernels run: the Trainer is built on a CPU model and only its
schedule is stepped."""
import os

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs', 'yolov5n.yaml')


@pytest.mark.parametrize('adam,linear,bs,nb', [(False, False, 16, 400), (True, False, 32, 300),
                                               (False, True, 64, 700), (False, False, 256, 25)])
def test_trainer_schedule_matches_reference_loop(adam, linear, bs, nb):
    from dmayolo.models.yolo import Model
    from dmayolo.trainer import Trainer
    from dmayolo.synthetic import HYP_VISDRONE, scaled_hyp
    from oracle.train import schedule
    torch.manual_seed(0)
    m = Model(CFG, nc=10)
    m.hyp = scaled_hyp(HYP_VISDRONE, 10, 640)
    hyp0 = dict(m.hyp)
    epochs = 30
    tr = Trainer(m, m.hyp, bs, epochs=epochs, nb=nb, adam=adam, linear_lr=linear, ema=False, amp=False)
    n = 3 * nb + 1200
    ref = schedule(hyp0, bs, epochs, nb, n, adam=adam, linear_lr=linear)
    assert tr.optimizer.param_groups[1]['weight_decay'] == pytest.approx(ref[0][4], rel=1e-12)
    for ni, acc, lrs, mom, _ in ref:
        if ni > 0 and ni % nb == 0:
            tr.epoch_end()
        assert tr.ni == ni
        tr.warmup(ni)
        assert tr.accumulate == acc, ni
        got = [g['lr'] for g in tr.optimizer.param_groups]
        assert got == pytest.approx(lrs, rel=1e-12, abs=1e-15), (ni, got, lrs)
        if mom is not None:
            assert all(g['momentum'] == pytest.approx(mom, rel=1e-12) for g in tr.optimizer.param_groups), ni
        else:
            assert all('momentum' not in g for g in tr.optimizer.param_groups)
        tr.i += 1
