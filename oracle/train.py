"""ORACLE (test infrastructure only; never imported by the product): the reference's optimisation schedule restated
with plain Python loops, for checking dmayolo.trainer.Trainer's host-side schedule logic.

Follows train.py:189-192 (nbs = 64, accumulate = max(round(nbs / batch_size), 1), weight_decay scaled by
batch_size * accumulate / nbs), 216-222 (SGD: every group starts at lr0; Adam: Adam(g0, lr=3e-4) so all three
groups inherit lr 3e-4 as their initial lr), 231-235 (linear lf or one_cycle(1, lrf, epochs), utils/general.py:
460-462), 235 + 352 (LambdaLR constructed -- lr = initial_lr * lf(0) -- then last_epoch reset to start_epoch - 1),
345 (nw = max(round(warmup_epochs * nb), 1000)), 408-422 (warmup: np.interp of accumulate, of each group's lr from
warmup_bias_lr (group 2) / 0.0 to initial_lr * lf(epoch), of momentum from warmup_momentum to momentum) and 466-468
(scheduler.step() at each epoch end: last_epoch += 1, lr = initial_lr * lf(last_epoch)).

Parity: the reference's train.py cannot run in this container (dataset, network); this restatement is pinned by
the reference lines above and by torch's LambdaLR / numpy.interp semantics, not by a reference run.
"""
import math


def _interp(x, xp, fp):
    """numpy.interp for two points, x in [xp0, xp1]"""
    if x <= xp[0]:
        return float(fp[0])
    if x >= xp[1]:
        return float(fp[1])
    return float(fp[0]) + (x - xp[0]) * (float(fp[1]) - float(fp[0])) / (xp[1] - xp[0])


def schedule(hyp, batch_size, epochs, nb, n_iters, adam=False, linear_lr=False, nbs=64):
    """[(ni, accumulate, [lr g0, g1, g2], momentum or None, weight_decay g1)] for ni in range(n_iters), each the value
    in force when batch ni is optimised."""
    accumulate = max(round(nbs / batch_size), 1)
    wd = hyp['weight_decay'] * batch_size * accumulate / nbs
    if linear_lr:
        lf = lambda x: (1 - x / (epochs - 1)) * (1.0 - hyp['lrf']) + hyp['lrf']  # noqa: E731
    else:
        lf = lambda x: ((1 - math.cos(x * math.pi / epochs)) / 2) * (hyp['lrf'] - 1) + 1  # noqa: E731
    initial = [3e-4] * 3 if adam else [hyp['lr0']] * 3
    lrs = [v * lf(0) for v in initial]  # LambdaLR.__init__ performs step 0
    last_epoch = -1  # train.py:352 with start_epoch = 0
    mom = None if adam else hyp['momentum']
    nw = max(round(hyp['warmup_epochs'] * nb), 1000)
    out = []
    for ni in range(n_iters):
        epoch = ni // nb
        if ni > 0 and ni % nb == 0:  # epoch end: scheduler.step()
            last_epoch += 1
            lrs = [v * lf(last_epoch) for v in initial]
        if ni <= nw:
            accumulate = max(1, round(_interp(ni, [0, nw], [1, nbs / batch_size])))
            lrs = [_interp(ni, [0, nw], [hyp['warmup_bias_lr'] if j == 2 else 0.0, initial[j] * lf(epoch)])
                   for j in range(3)]
            if not adam:
                mom = _interp(ni, [0, nw], [hyp['warmup_momentum'], hyp['momentum']])
        out.append((ni, accumulate, list(lrs), mom, wd))
    return out
