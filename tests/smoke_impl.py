"""Body of __graft_entry__.smoke(): tiny DMA-YOLO train step + eval + NMS on cuda:0 vs the oracle."""
import copy

import torch


def tiny_yaml():
    return dict(nc=4, depth_multiple=0.33, width_multiple=0.125,
                anchors=[[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [116, 90, 156, 198, 373, 326]],
                backbone=[[-1, 1, 'Conv', [64, 6, 2, 2]], [-1, 1, 'SCConv', [128, 2]], [-1, 3, 'C3', [128]],
                          [-1, 1, 'Conv', [256, 3, 2]], [-1, 1, 'C3', [256]], [-1, 1, 'Conv', [512, 3, 2]],
                          [-1, 1, 'CA', [512]], [-1, 1, 'SPPFCSPC', [512]]],
                head=[[-1, 1, 'Conv', [256, 1, 1]], [-1, 1, 'nn.Upsample', [None, 2, 'nearest']],
                      [[-1, 4], 1, 'AdConcat2', [1]], [-1, 1, 'C3', [256, False]],
                      [-1, 1, 'Conv', [128, 1, 1]], [-1, 1, 'nn.Upsample', [None, 2, 'nearest']],
                      [[-1, 2], 1, 'AdConcat2', [1]], [-1, 1, 'C3', [128, False]],
                      [-1, 1, 'Conv', [128, 3, 2]], [[-1, 11, 4], 1, 'AdConcat3', [1]], [-1, 1, 'C3', [256, False]],
                      [-1, 1, 'Conv', [256, 3, 2]], [[-1, 7], 1, 'AdConcat2', [1]], [-1, 1, 'C3', [512, False]],
                      [[15, 18, 21], 1, 'Detect', ['nc', 'anchors']]])


def run_smoke():
    from dmayolo.models.yolo import Model
    from dmayolo.utils.loss import ComputeLoss
    from dmayolo.utils.general import non_max_suppression
    from dmayolo.optim import build_optimizer
    from oracle import nn as onn
    from oracle.loss import compute_loss
    from oracle.general import non_max_suppression as onms

    assert torch.cuda.is_available(), 'smoke() needs cuda:0'
    torch.manual_seed(0)
    yml = tiny_yaml()
    m = Model(copy.deepcopy(yml), nc=4)
    ref = onn.bn_defaults(onn.Model(copy.deepcopy(yml), nc=4))
    ref.load_state_dict(m.state_dict())
    hyp = dict(box=0.05, obj=1.0 * (64 / 640) ** 2, cls=0.5 * 4 / 80, cls_pw=1.0, obj_pw=1.0, anchor_t=4.0,
               fl_gamma=0.0, label_smoothing=0.0)
    m.hyp = hyp
    m = m.cuda().train()
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (2, 3, 64, 64), generator=g, dtype=torch.uint8)
    tg = torch.cat([torch.tensor([[0, 1, .5, .5, .2, .3], [1, 3, .3, .6, .1, .1], [1, 0, .8, .2, .3, .2]])], 0)
    p = m(imgs.cuda())
    loss, items = ComputeLoss(m)(p, tg.cuda())
    loss.backward()
    ref.train()
    pr = ref(imgs.float() / 255)
    lr_, ir_ = compute_loss(pr, tg, m.model[-1].anchors.cpu(), hyp, 4)
    for a, b in zip(p, pr):
        torch.testing.assert_close(a.detach().float().cpu(), b.detach(), rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(loss.detach().cpu(), lr_.detach(), rtol=2e-3, atol=1e-5)
    opt = build_optimizer(m)
    opt.step()
    assert all(torch.isfinite(q).all() for q in m.parameters())
    m.eval()
    with torch.no_grad():
        z, _ = m(imgs.cuda())
    out = non_max_suppression(z, 0.001, 0.6, multi_label=True)
    oref = onms(z.cpu(), 0.001, 0.6, multi_label=True)
    for a, b in zip(out, oref):
        assert torch.equal(a.cpu(), b)
    print(f'smoke ok: loss={float(loss):.5f} items={items.tolist()} det={[o.shape[0] for o in out]}')
