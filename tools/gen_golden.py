"""Generate golden vectors from the reference's own PyTorch-CPU path (in-container only).

Run:  cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tools/gen_golden.py
Writes small .npz fixtures into /root/repo/tests/golden/.  The reference code itself never
leaves this container: only inputs, state_dicts and outputs are stored.

Each module fixture stores (keys):
  meta          JSON string (module name, ctor args, shapes, flags)
  in.<i>        input tensors
  sd.<k>        state_dict BEFORE the train-mode forward (params + buffers)
  gup.<i>       upstream gradient used for backward (loss = sum(out * gup))
  out.<i>       train-mode outputs
  gin.<i>       d loss / d input
  gp.<k>        d loss / d param
  sd_after.<k>  buffers after the train-mode forward (BN running stats)
  eout.<i>      eval-mode outputs (from the BEFORE state)
"""
import json
import math
import os
import sys
from copy import deepcopy

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ref_stubs  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden')
os.makedirs(OUT, exist_ok=True)
Y = ref_stubs.install()
import models.common as C  # noqa: E402  (reference)
import utils.loss as L  # noqa: E402
import utils.general as G  # noqa: E402
import utils.metrics as M  # noqa: E402
from utils.torch_utils import initialize_weights, fuse_conv_and_bn  # noqa: E402

torch.set_num_threads(8)


def npy(t):
    return t.detach().cpu().numpy().copy()  # copy: never alias module buffers that are reloaded later


def randomize_bn(mod, gen):
    for m in mod.modules():
        if isinstance(m, nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.copy_(torch.rand(m.weight.shape, generator=gen) + 0.5)
                m.bias.copy_(torch.randn(m.bias.shape, generator=gen) * 0.1)
                m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=gen) * 0.1)
                m.running_var.copy_(torch.rand(m.running_var.shape, generator=gen) + 0.5)
        if isinstance(m, nn.LayerNorm):
            with torch.no_grad():
                m.weight.copy_(torch.rand(m.weight.shape, generator=gen) + 0.5)
                m.bias.copy_(torch.randn(m.bias.shape, generator=gen) * 0.1)
        if isinstance(m, C.WindowAttention):
            with torch.no_grad():
                m.relative_position_bias_table.copy_(
                    torch.randn(m.relative_position_bias_table.shape, generator=gen) * 0.5)
        if isinstance(m, (C.AdConcat2, C.AdConcat3)):
            with torch.no_grad():
                m.w.copy_(torch.rand(m.w.shape, generator=gen) + 0.5)
        if isinstance(m, C.DropPath):
            m.drop_prob = 0.0  # deterministic: SURVEY §0.6 (DropPath forced off in fixtures)
        if isinstance(m, nn.Dropout):
            m.p = 0.0  # TransformerLayer dropout (common.py:328): deterministic fixtures


def module_case(name, mod, inputs, meta, seed=0, eval_too=True, list_input=False):
    gen = torch.Generator().manual_seed(seed + 1000)
    initialize_weights(mod)  # BN eps 1e-3 / momentum 0.03 (utils/torch_utils.py:161-170)
    randomize_bn(mod, gen)
    sd0 = {k: v.clone() for k, v in mod.state_dict().items()}
    ins = [x.clone().requires_grad_(True) for x in inputs]
    mod.train()
    out = mod(ins if list_input else ins[0])
    outs = list(out) if isinstance(out, (list, tuple)) else [out]
    gups = [torch.randn(o.shape, generator=gen) for o in outs]
    loss = sum((o * g).sum() for o, g in zip(outs, gups))
    mod.zero_grad()
    loss.backward()
    d = {'meta': json.dumps(meta)}
    for i, x in enumerate(inputs):
        d[f'in.{i}'] = npy(x)
    for k, v in sd0.items():
        d[f'sd.{k}'] = npy(v)
    for i, (o, g) in enumerate(zip(outs, gups)):
        d[f'out.{i}'] = npy(o)
        d[f'gup.{i}'] = npy(g)
    for i, x in enumerate(ins):
        d[f'gin.{i}'] = npy(x.grad)
    for k, p in mod.named_parameters():
        if p.grad is not None:
            d[f'gp.{k}'] = npy(p.grad)
    for k, v in mod.state_dict().items():
        if k not in dict(mod.named_parameters()):
            d[f'sd_after.{k}'] = npy(v)
    if eval_too:
        mod.load_state_dict(sd0)
        mod.eval()
        with torch.no_grad():
            eo = mod(inputs if list_input else inputs[0])
        eos = list(eo) if isinstance(eo, (list, tuple)) else [eo]
        for i, o in enumerate(eos):
            if isinstance(o, torch.Tensor):
                d[f'eout.{i}'] = npy(o)
    np.savez_compressed(os.path.join(OUT, f'{name}.npz'), **d)
    print('wrote', name, sum(v.nbytes for k, v in d.items() if k != 'meta') / 1e6, 'MB')


def rnd(*shape, seed=0, scale=1.0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)) * scale


def gen_modules():
    torch.manual_seed(0)
    # 1. Conv (YAML-level cspcm.Conv; identical forward to common.Conv)
    for (c1, c2, k, s, p, hw, tag) in [(16, 32, 1, 1, None, 12, 'k1s1'), (16, 24, 3, 1, None, 12, 'k3s1'),
                                       (16, 32, 3, 2, None, 13, 'k3s2'), (3, 16, 6, 2, 2, 16, 'k6s2p2'),
                                       (8, 16, 3, 2, None, 10, 'k3s2b')]:
        torch.manual_seed(1)
        m = Y.Conv(c1, c2, k, s, p)
        module_case(f'conv_{tag}', m, [rnd(2, c1, hw, hw + 2, seed=2)],
                    dict(module='Conv', args=[c1, c2, k, s, p]))
    # forward_fuse (partial fuse semantics, yolo.py:315-323)
    torch.manual_seed(1)
    m = Y.Conv(16, 32, 3, 1)
    gen = torch.Generator().manual_seed(5)
    initialize_weights(m)
    randomize_bn(m, gen)
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    m.eval()
    x = rnd(2, 16, 10, 10, seed=3)
    m.conv = fuse_conv_and_bn(m.conv, m.bn)
    with torch.no_grad():
        o = m.act(m.conv(x))
    np.savez_compressed(os.path.join(OUT, 'conv_fuse.npz'), meta=json.dumps(dict(module='Conv', args=[16, 32, 3, 1])),
                        **{'in.0': npy(x), 'eout.0': npy(o), 'fw': npy(m.conv.weight), 'fb': npy(m.conv.bias)},
                        **{f'sd.{k}': npy(v) for k, v in sd0.items()})
    # 2. Bottleneck / C3
    for sc in (True, False):
        torch.manual_seed(2)
        module_case(f'bottleneck_{int(sc)}', C.Bottleneck(16, 16, sc), [rnd(2, 16, 8, 8, seed=4)],
                    dict(module='Bottleneck', args=[16, 16, sc]))
        torch.manual_seed(2)
        module_case(f'c3_{int(sc)}', C.C3(16, 32, 2, sc), [rnd(2, 16, 8, 8, seed=4)],
                    dict(module='C3', args=[16, 32, 2, sc]))
    # 3. SCConv
    torch.manual_seed(3)
    module_case('scconv_sq', C.SCConv(16, 32, 2), [rnd(2, 16, 32, 32, seed=5)], dict(module='SCConv', args=[16, 32, 2]))
    torch.manual_seed(3)
    module_case('scconv_rect', C.SCConv(16, 32, 2), [rnd(1, 16, 40, 24, seed=6)], dict(module='SCConv', args=[16, 32, 2]))
    torch.manual_seed(3)
    module_case('scconv_odd', C.SCConv(8, 16, 2), [rnd(1, 8, 18, 22, seed=6)], dict(module='SCConv', args=[8, 16, 2]))
    # 4. CoorAttention / C3CA
    torch.manual_seed(4)
    module_case('ca', C.CoorAttention(32, 32), [rnd(2, 32, 12, 10, seed=7)], dict(module='CoorAttention', args=[32, 32]))
    torch.manual_seed(4)
    module_case('c3ca', C.C3CA(32, 32, 1, False), [rnd(2, 32, 8, 8, seed=8)], dict(module='C3CA', args=[32, 32, 1, False]))
    torch.manual_seed(4)
    module_case('c3ca_sc', C.C3CA(32, 32, 2, True), [rnd(2, 32, 8, 8, seed=8)], dict(module='C3CA', args=[32, 32, 2, True]))
    # 5. SPPF / SPPFCSPC
    torch.manual_seed(5)
    module_case('sppf', C.SPPF(32, 32, 5), [rnd(2, 32, 9, 9, seed=9)], dict(module='SPPF', args=[32, 32, 5]))
    torch.manual_seed(5)
    module_case('sppfcspc', C.SPPFCSPC(32, 32), [rnd(2, 32, 9, 9, seed=9)], dict(module='SPPFCSPC', args=[32, 32]))
    # 6. Upsample + AdConcat
    torch.manual_seed(6)
    module_case('upsample', nn.Upsample(None, 2, 'nearest'), [rnd(2, 8, 5, 6, seed=10)],
                dict(module='Upsample', args=[None, 2, 'nearest']))
    torch.manual_seed(6)
    module_case('adconcat2', C.AdConcat2(1), [rnd(2, 8, 6, 6, seed=11), rnd(2, 16, 6, 6, seed=12)],
                dict(module='AdConcat2', args=[1]), list_input=True)
    torch.manual_seed(6)
    module_case('adconcat3', C.AdConcat3(1), [rnd(2, 8, 6, 6, seed=11), rnd(2, 16, 6, 6, seed=12),
                                              rnd(2, 8, 6, 6, seed=13)], dict(module='AdConcat3', args=[1]),
                list_input=True)
    torch.manual_seed(6)
    module_case('concat', C.Concat(1), [rnd(2, 8, 6, 6, seed=11), rnd(2, 16, 6, 6, seed=12)],
                dict(module='Concat', args=[1]), list_input=True)
    # 7. Swin
    for (c, heads, shift, h, w, tag) in [(64, 2, 0, 16, 16, 's0_16'), (64, 2, 4, 16, 16, 's4_16'),
                                         (64, 2, 4, 20, 20, 's4_20'), (32, 1, 4, 12, 20, 's4_12x20'),
                                         (64, 2, 0, 20, 12, 's0_20x12')]:
        torch.manual_seed(7)
        m = C.SwinTransformerLayer(c, num_heads=heads, window_size=8, shift_size=shift)
        module_case(f'swin_{tag}', m, [rnd(1, c, h, w, seed=14, scale=0.5)],
                    dict(module='SwinTransformerLayer', args=[c, heads, 8, shift]))
    for (hh, ww, tag) in [(24, 24, '24'), (24, 16, '24x16'), (16, 24, '16x24')]:
        m = C.SwinTransformerLayer(32, num_heads=1, window_size=8, shift_size=4)
        x = torch.zeros(1, ww, hh, 32)
        mask = m.create_mask(x, hh, ww)
        np.savez_compressed(os.path.join(OUT, f'swinmask_{tag}.npz'), meta=json.dumps(dict(H=hh, W=ww)),
                            mask=npy(mask))
    # 8. config-5 modules (yolov5l-xs-tr-cbam-spp-bifpn.yaml): SPP variants, CBAM
    for (k, tag) in [((5, 9, 13), 'k5913'), ((3, 5, 7), 'k357')]:
        torch.manual_seed(17)
        module_case(f'spp_{tag}', C.SPP(32, 32, k), [rnd(2, 32, 11, 9, seed=18)], dict(module='SPP', args=[32, 32, list(k)]))
    for (c, hw, tag) in [(32, (10, 12), 'c32'), (64, (7, 5), 'c64')]:
        torch.manual_seed(19)
        module_case(f'cbam_{tag}', C.CBAM(c, c), [rnd(2, c, *hw, seed=20)], dict(module='CBAM', args=[c, c]))
    torch.manual_seed(8)
    module_case('c3str', C.C3STR(64, 64, 3, False), [rnd(1, 64, 16, 16, seed=15, scale=0.5)],
                dict(module='C3STR', args=[64, 64, 3, False]))
    torch.manual_seed(8)
    module_case('c3str_pad', C.C3STR(128, 128, 2, False), [rnd(1, 128, 12, 10, seed=16, scale=0.5)],
                dict(module='C3STR', args=[128, 128, 2, False]))


def gen_detect():
    torch.manual_seed(9)
    anchors = [[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [116, 90, 156, 198, 373, 326]]
    d = Y.Detect(10, anchors, [16, 32, 64])
    d.stride = torch.tensor([8., 16., 32.])
    d.anchors /= d.stride.view(-1, 1, 1)
    xs = [rnd(2, 16, 8, 8, seed=20), rnd(2, 32, 4, 4, seed=21), rnd(2, 64, 2, 2, seed=22)]
    sd0 = {k: v.clone() for k, v in d.state_dict().items()}
    d.train()
    outs = d([x.clone() for x in xs])
    d.eval()
    with torch.no_grad():
        z, _ = d([x.clone() for x in xs])
    dd = {'meta': json.dumps(dict(module='Detect', nc=10, anchors=anchors, ch=[16, 32, 64], stride=[8, 16, 32]))}
    for i, x in enumerate(xs):
        dd[f'in.{i}'] = npy(x)
    for k, v in sd0.items():
        dd[f'sd.{k}'] = npy(v)
    for i, o in enumerate(outs):
        dd[f'out.{i}'] = npy(o)
    dd['eout.0'] = npy(z)
    np.savez_compressed(os.path.join(OUT, 'detect.npz'), **dd)
    print('wrote detect')


def synth_targets(n_img, nt_per, nc, seed, edge=True):
    g = torch.Generator().manual_seed(seed)
    rows = []
    for b in range(n_img):
        nt = nt_per
        cls = torch.randint(0, nc, (nt,), generator=g).float()
        xy = torch.rand(nt, 2, generator=g) * 0.9 + 0.05
        wh = torch.exp(torch.rand(nt, 2, generator=g) * (math.log(0.3) - math.log(0.005)) + math.log(0.005))
        rows.append(torch.cat([torch.full((nt, 1), float(b)), cls[:, None], xy, wh], 1))
    t = torch.cat(rows, 0)
    if edge:  # targets at the image border exercise the in-place clamp (loss.py:265-272)
        t = torch.cat([t, torch.tensor([[0, 1, 0.0, 0.0, 0.05, 0.05], [0, 2, 1.0, 1.0, 0.1, 0.08],
                                        [n_img - 1, 0, 0.999, 0.001, 0.02, 0.04],
                                        [n_img - 1, 3, 0.5, 0.5, 0.5, 0.6]])], 0)
    return t


class _FakeDet:
    pass


def gen_loss():
    anchors = [[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [116, 90, 156, 198, 373, 326]]
    for hypname, nc, img in [('VisDrone', 10, 256), ('scratch', 80, 128)]:
        import yaml
        hyp = yaml.safe_load(open(f'/root/reference/data/hyps/hyp.{hypname}.yaml'))
        nl = 3
        hyp['box'] *= 3 / nl
        hyp['cls'] *= nc / 80 * 3 / nl
        hyp['obj'] *= (img / 640) ** 2 * 3 / nl
        hyp['label_smoothing'] = 0.0
        torch.manual_seed(10)
        model = Y.Model('/root/reference/models/yolov5n.yaml', nc=nc)
        model.hyp = hyp
        det = model.model[-1]
        bs = 2
        p = [rnd(bs, 3, img // s, img // s, nc + 5, seed=30 + i) for i, s in enumerate((8, 16, 32))]
        targets = synth_targets(bs, 12, nc, seed=31)
        cl = L.ComputeLoss(model)
        tcls, tbox, indices, anch = cl.build_targets(p, targets)
        pp = [x.clone().requires_grad_(True) for x in p]
        loss, items = cl(pp, targets)
        loss.backward()
        d = {'meta': json.dumps(dict(hyp=hyp, nc=nc, img=img, anchors=anchors, stride=[8, 16, 32])),
             'targets': npy(targets), 'anchors': npy(det.anchors), 'loss': npy(loss), 'items': npy(items)}
        for i in range(3):
            d[f'p.{i}'] = npy(p[i])
            d[f'gp.{i}'] = npy(pp[i].grad)
            d[f'tcls.{i}'] = npy(tcls[i])
            d[f'tbox.{i}'] = npy(tbox[i])
            d[f'anch.{i}'] = npy(anch[i])
            for j, nm in enumerate('b a gj gi'.split()):
                d[f'{nm}.{i}'] = npy(indices[i][j])
        np.savez_compressed(os.path.join(OUT, f'loss_{hypname}.npz'), **d)
        print('wrote loss', hypname)


def gen_siou():
    g = torch.Generator().manual_seed(40)
    n = 256
    b1 = torch.cat([torch.rand(n, 2, generator=g) * 4, torch.rand(n, 2, generator=g) * 3 + 0.05], 1)
    b2 = torch.cat([torch.rand(n, 2, generator=g) * 4, torch.rand(n, 2, generator=g) * 3 + 0.05], 1)
    b2[:8, :2] = b1[:8, :2] + 1e-3 * torch.randn(8, 2, generator=g)  # near-coincident centres
    b2[8:16, 0] = b1[8:16, 0]  # sin_alpha exactly 1 on one side
    b1r = b1.clone().requires_grad_(True)
    iou = M.bbox_iou(b1r.T, b2, x1y1x2y2=False, SIoU=True)
    iou.sum().backward()
    np.savez_compressed(os.path.join(OUT, 'siou.npz'), b1=npy(b1), b2=npy(b2), iou=npy(iou), g=npy(b1r.grad))
    # plain IoU / box_iou
    bx1 = torch.cat([b1[:, :2] - b1[:, 2:] / 2, b1[:, :2] + b1[:, 2:] / 2], 1)
    bx2 = torch.cat([b2[:, :2] - b2[:, 2:] / 2, b2[:, :2] + b2[:, 2:] / 2], 1)
    np.savez_compressed(os.path.join(OUT, 'box_iou.npz'), a=npy(bx1[:40]), b=npy(bx2[:50]),
                        iou=npy(M.box_iou(bx1[:40], bx2[:50])))
    print('wrote siou')


def gen_nms():
    cases = []
    g = torch.Generator().manual_seed(50)

    def clustered(n_img, A, nc, n_clusters, per, seed, quant=False):
        gg = torch.Generator().manual_seed(seed)
        pred = torch.zeros(n_img, A, nc + 5)
        pred[..., :2] = torch.rand(n_img, A, 2, generator=gg) * 600
        pred[..., 2:4] = torch.rand(n_img, A, 2, generator=gg) * 40 + 2
        pred[..., 4] = torch.rand(n_img, A, generator=gg) * 0.2  # mostly below conf
        pred[..., 5:] = torch.rand(n_img, A, nc, generator=gg)
        for b in range(n_img):
            idx = torch.randperm(A, generator=gg)[:n_clusters * per]
            cen = torch.rand(n_clusters, 2, generator=gg) * 600
            wh = torch.rand(n_clusters, 2, generator=gg) * 60 + 10
            for ci in range(n_clusters):
                ii = idx[ci * per:(ci + 1) * per]
                pred[b, ii, :2] = cen[ci] + torch.randn(per, 2, generator=gg) * 3
                pred[b, ii, 2:4] = wh[ci] * (1 + 0.1 * torch.randn(per, 2, generator=gg))
                pred[b, ii, 4] = torch.rand(per, generator=gg) * 0.7 + 0.3
        if quant:  # score ties
            pred[..., 4] = (pred[..., 4] * 8).round() / 8
            pred[..., 5:] = (pred[..., 5:] * 4).round() / 4
        return pred

    specs = [
        ('nms_detect', clustered(2, 3000, 10, 40, 10, 51), dict(conf_thres=0.25, iou_thres=0.45, max_det=1000)),
        ('nms_val', clustered(2, 3000, 10, 40, 10, 52), dict(conf_thres=0.001, iou_thres=0.6, multi_label=True,
                                                            max_det=300)),
        ('nms_ties', clustered(2, 2000, 4, 30, 8, 53, quant=True), dict(conf_thres=0.25, iou_thres=0.45)),
        ('nms_ties_ml', clustered(1, 2000, 4, 30, 8, 54, quant=True), dict(conf_thres=0.1, iou_thres=0.5,
                                                                          multi_label=True)),
        ('nms_agnostic', clustered(1, 2000, 10, 30, 8, 55), dict(conf_thres=0.25, iou_thres=0.45, agnostic=True)),
        ('nms_classes', clustered(1, 2000, 10, 30, 8, 56), dict(conf_thres=0.25, iou_thres=0.45, classes=[1, 3, 7])),
        ('nms_empty', clustered(2, 500, 10, 0, 0, 57), dict(conf_thres=0.5, iou_thres=0.45)),
        ('nms_nc1', clustered(1, 1500, 1, 20, 8, 58), dict(conf_thres=0.25, iou_thres=0.45, multi_label=True)),
    ]
    # >30k candidates: multi-label over many boxes to exercise the max_nms cut
    big = clustered(1, 12000, 5, 400, 25, 59)
    big[..., 4] = torch.rand(1, 12000, generator=g) * 0.5 + 0.5
    specs.append(('nms_big', big, dict(conf_thres=0.001, iou_thres=0.6, multi_label=True, max_det=300)))
    class _NoClock:  # the reference's 10 s wall-clock guard (general.py:651,721) is not part of the contract
        @staticmethod
        def time():
            return 0.0
    G.time = _NoClock
    for name, pred, kw in specs:
        out = G.non_max_suppression(pred.clone(), **kw)
        d = {'meta': json.dumps(kw), 'pred': npy(pred)}
        for i, o in enumerate(out):
            d[f'out.{i}'] = npy(o)
        np.savez_compressed(os.path.join(OUT, f'{name}.npz'), **d)
        print('wrote', name, [o.shape[0] for o in out])


def small_yaml(src, gw, gd, overrides=None):
    import yaml
    d = yaml.safe_load(open(src))
    d['width_multiple'] = gw
    d['depth_multiple'] = gd
    for i, args in (overrides or {}).items():
        layers = d['backbone'] + d['head']
        layers[i][3] = args
    return d


def gen_models():
    # whole-model forward/backward at small width, fp16-rounded weights so fixtures stay small
    cfgs = [
        ('model_v5s', small_yaml('/root/reference/models/yolov5s.yaml', 0.125, 0.33), 10, 64, 2),
        ('model_dma', small_yaml('/root/reference/models/yolov5l-ca-sppfcspc-bifpn-scconv.yaml', 0.125, 0.33,
                                 {18: [512, False], 21: [512, False], 24: [1024, False]}), 10, 128, 2),
    ]
    for name, yml, nc, img, bs in cfgs:
        torch.manual_seed(11)
        model = Y.Model(deepcopy(yml), nc=nc)
        gen = torch.Generator().manual_seed(12)
        randomize_bn(model, gen)
        with torch.no_grad():
            for k, v in model.state_dict().items():
                if v.dtype.is_floating_point:
                    v.copy_(v.half().float())
        sd0 = {k: v.clone() for k, v in model.state_dict().items()}
        x = torch.rand(bs, 3, img, img, generator=torch.Generator().manual_seed(13))
        model.train()
        outs = model(x)
        gups = [torch.randn(o.shape, generator=gen) * 0.1 for o in outs]
        loss = sum((o * g).sum() for o, g in zip(outs, gups))
        loss.backward()
        d = {'meta': json.dumps(dict(yaml=yml, nc=nc, img=img)), 'in.0': npy(x)}
        for k, v in sd0.items():
            d[f'sd.{k}'] = v.half().numpy() if v.dtype.is_floating_point else npy(v)
        for i, (o, g) in enumerate(zip(outs, gups)):
            d[f'out.{i}'] = npy(o)
            d[f'gup.{i}'] = npy(g)
        params = dict(model.named_parameters())
        for k in list(params)[:6] + list(params)[-6:]:
            d[f'gp.{k}'] = npy(params[k].grad)
        d['gnorm'] = np.array([float(p.grad.norm()) if p.grad is not None else 0.0 for p in params.values()],
                              dtype=np.float64)
        d['pnames'] = np.array(list(params.keys()))
        model.load_state_dict(sd0)
        model.eval()
        with torch.no_grad():
            z, _ = model(x)
        d['eout.0'] = npy(z)
        np.savez_compressed(os.path.join(OUT, f'{name}.npz'), **d)
        print('wrote', name, sum(v.nbytes for k, v in d.items() if k != 'meta') / 1e6, 'MB')


def gen_optim():
    """One SGD (nesterov) and one Adam step with the reference's param grouping (train.py:197-222) + EMA."""
    from torch.optim import SGD, Adam
    from utils.torch_utils import ModelEMA
    yml = dict(nc=3, depth_multiple=1.0, width_multiple=1.0,
               anchors=[[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [116, 90, 156, 198, 373, 326]],
               backbone=[[-1, 1, 'Conv', [8, 3, 2]], [-1, 1, 'Conv', [16, 3, 2]], [-1, 1, 'C3', [16]],
                         [-1, 1, 'Conv', [32, 3, 2]], [-1, 1, 'C3STR', [64, False]], [-1, 1, 'Conv', [32, 3, 2]]],
               head=[[-1, 1, 'nn.Upsample', [None, 2, 'nearest']], [[-1, 4], 1, 'AdConcat2', [1]],
                     [-1, 1, 'Conv', [16, 1, 1]], [[2, 8, 5], 1, 'Detect', ['nc', 'anchors']]])
    torch.manual_seed(14)
    model = Y.Model(deepcopy(yml), nc=10)
    names = {id(p): k for k, p in model.named_parameters()}
    g0, g1, g2 = [], [], []
    for v in model.modules():
        if hasattr(v, 'bias') and isinstance(v.bias, nn.Parameter):
            g2.append(v.bias)
        if isinstance(v, nn.BatchNorm2d):
            g0.append(v.weight)
        elif hasattr(v, 'weight') and isinstance(v.weight, nn.Parameter):
            g1.append(v.weight)
        elif isinstance(v, (C.AdConcat2, C.AdConcat3)) and isinstance(v.w, nn.Parameter):
            g1.append(v.w)
    groups = {'g0': [names[id(p)] for p in g0], 'g1': [names[id(p)] for p in g1], 'g2': [names[id(p)] for p in g2]}
    # deterministic grads
    gen = torch.Generator().manual_seed(15)
    grads = {k: torch.randn(p.shape, generator=gen) * 0.01 for k, p in model.named_parameters()}
    d = {'meta': json.dumps(dict(groups=groups, yaml=yml))}
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    for k, v in sd0.items():
        d[f'sd.{k}'] = npy(v)
    for k, v in grads.items():
        d[f'grad.{k}'] = npy(v)
    for kind in ('sgd', 'adam'):
        model.load_state_dict(sd0)
        g0p = [dict(model.named_parameters())[n] for n in groups['g0']]
        g1p = [dict(model.named_parameters())[n] for n in groups['g1']]
        g2p = [dict(model.named_parameters())[n] for n in groups['g2']]
        lr, mom, wd = 0.01, 0.937, 0.0005
        if kind == 'adam':
            opt = Adam(g0p, lr=3e-4, betas=(mom, 0.999))
        else:
            opt = SGD(g0p, lr=lr, momentum=mom, nesterov=True)
        opt.add_param_group({'params': g1p, 'weight_decay': wd})
        opt.add_param_group({'params': g2p})
        for j, grp in enumerate(opt.param_groups):
            grp['lr'] = [0.001, 0.002, 0.05][j]
            if 'momentum' in grp:
                grp['momentum'] = 0.8
        for step in range(2):
            for k, p in model.named_parameters():
                p.grad = grads[k].clone() * (1 + step)
            opt.step()
        for k, p in model.named_parameters():
            d[f'{kind}.{k}'] = npy(p)
    # EMA over state_dict incl. BN buffers (torch_utils.py:329-339)
    model.load_state_dict(sd0)
    ema = ModelEMA(model)
    with torch.no_grad():
        for p in model.parameters():
            p.add_(0.1)
        for m in model.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.running_mean.add_(0.2)
    ema.update(model)
    ema.update(model)
    for k, v in ema.ema.state_dict().items():
        d[f'ema.{k}'] = npy(v)
    np.savez_compressed(os.path.join(OUT, 'optim.npz'), **d)
    print('wrote optim', sum(v.nbytes for k, v in d.items() if k != 'meta') / 1e6, 'MB')


def gen_tal():
    """anchor-free TAL path: TaskAlignedAssigner, ComputeLoss_TAL (+ grads), TDetect, space_to_depth,
    and the CASPD_ODRTA (TDetect) model's parameter layout."""
    from utils.tal_assign import TaskAlignedAssigner
    import utils.tal as T
    import models.detect_t as DT
    import yaml
    shapes, strides = [(8, 8), (4, 4), (2, 2)], [8, 16, 32]
    img = 64
    # 1. assigner on crafted crowded inputs (several gts claim the same anchors; one padded gt row)
    for tag, nc, seed in [('a', 5, 40), ('b', 3, 41)]:
        g = torch.Generator().manual_seed(seed)
        B, n = 2, 5
        pts, st = [], []
        for (h, w), s_ in zip(shapes, strides):
            ys, xs = torch.meshgrid(torch.arange(h) + 0.5, torch.arange(w) + 0.5, indexing='ij')
            pts.append(torch.stack((xs.reshape(-1), ys.reshape(-1)), 1) * s_)
            st.append(torch.full((h * w, 1), float(s_)))
        pts, st = torch.cat(pts), torch.cat(st)
        A = pts.shape[0]
        c = torch.rand(B, n, 2, generator=g) * 48 + 8
        wh = torch.rand(B, n, 2, generator=g) * 30 + 6
        gboxes = torch.cat((c - wh / 2, c + wh / 2), -1)
        labels = torch.randint(0, nc, (B, n, 1), generator=g).float()
        gmask = torch.ones(B, n, 1)
        gboxes[1, -1] = 0
        labels[1, -1] = 0
        gmask[1, -1] = 0
        scores = torch.rand(B, A, nc, generator=g) * 0.9 + 0.05
        pc = pts[None] + torch.randn(B, A, 2, generator=g) * 4
        pwh = torch.rand(B, A, 2, generator=g) * 30 + 4
        pboxes = torch.cat((pc - pwh / 2, pc + pwh / 2), -1)
        asg = TaskAlignedAssigner(topk=10, num_classes=nc, alpha=0.5, beta=6.0)
        tl, tb, ts, fg = asg(scores, pboxes, pts, labels, gboxes, gmask)
        np.savez_compressed(os.path.join(OUT, f'tal_assign_{tag}.npz'), meta=json.dumps(dict(nc=nc)),
                            scores=npy(scores), pboxes=npy(pboxes), pts=npy(pts), labels=npy(labels),
                            gboxes=npy(gboxes), gmask=npy(gmask), t_lab=npy(tl), t_box=npy(tb), t_sc=npy(ts),
                            fg=npy(fg))
        print('wrote tal_assign', tag, int(fg.sum()))
    # 2. ComputeLoss_TAL with gradients w.r.t. the TDetect training outputs
    hyp = yaml.safe_load(open('/root/reference/data/hyps/hyp.VisDrone.yaml'))
    for tag, nc, seed in [('a', 10, 42), ('b', 4, 43)]:
        B = 2
        det = DT.TDetect(nc=nc, ch=(16, 16, 16))
        det.stride = torch.tensor([8.0, 16.0, 32.0])

        class _M(nn.Module):
            def __init__(self):
                super().__init__()
                self.model = nn.Sequential(det)
        m = _M()
        m.hyp = hyp
        A = sum(h * w for h, w in shapes)
        g = torch.Generator().manual_seed(seed)
        feats = [torch.zeros(B, nc + 64, h, w) for h, w in shapes]
        pdist = torch.randn(B, 64, A, generator=g) * 1.5
        pcls = torch.randn(B, nc, A, generator=g) - 2.0
        targets = synth_targets(B, 6, nc, seed=seed + 100)
        targets[:, 4:6] = targets[:, 4:6].clamp(0.08, 0.6)   # boxes of a few cells on the 64-px image
        cl = T.ComputeLoss_TAL(m)
        pd_, pc_ = pdist.clone().requires_grad_(True), pcls.clone().requires_grad_(True)
        loss, items = cl((feats, pd_, pc_), targets)
        loss.backward()
        np.savez_compressed(os.path.join(OUT, f'tal_loss_{tag}.npz'),
                            meta=json.dumps(dict(nc=nc, hyp=hyp, strides=[8, 16, 32], shapes=shapes)),
                            pdist=npy(pdist), pcls=npy(pcls), targets=npy(targets), loss=npy(loss), items=npy(items),
                            g_pdist=npy(pd_.grad), g_pcls=npy(pc_.grad))
        print('wrote tal_loss', tag, npy(items))
    # 3. TDetect head forward / backward / eval (list input, tuple output flattened)
    torch.manual_seed(44)
    det = DT.TDetect(nc=6, ch=(16, 32))
    det.stride = torch.tensor([8.0, 16.0])
    det.bias_init()
    gen = torch.Generator().manual_seed(45)
    initialize_weights(det)
    randomize_bn(det, gen)
    sd0 = {k: v.clone() for k, v in det.state_dict().items()}
    xs = [rnd(2, 16, 8, 10, seed=46), rnd(2, 32, 4, 5, seed=47)]
    ins = [x.clone().requires_grad_(True) for x in xs]
    det.train()
    lvl, box, cls = det(list(ins))
    outs = list(lvl) + [box, cls]
    gups = [torch.randn(o.shape, generator=gen) for o in outs]
    sum((o * gg).sum() for o, gg in zip(outs, gups)).backward()
    d = {'meta': json.dumps(dict(module='TDetect', args=[6, [16, 32]], stride=[8.0, 16.0]))}
    for i, x in enumerate(xs):
        d[f'in.{i}'] = npy(x)
        d[f'gin.{i}'] = npy(ins[i].grad)
    for k, v in sd0.items():
        d[f'sd.{k}'] = npy(v)
    for i, (o, gg) in enumerate(zip(outs, gups)):
        d[f'out.{i}'] = npy(o)
        d[f'gup.{i}'] = npy(gg)
    for k, p_ in det.named_parameters():
        if p_.grad is not None:
            d[f'gp.{k}'] = npy(p_.grad)
    det.load_state_dict(sd0)
    det.eval()
    with torch.no_grad():
        y, _ = det([x.clone() for x in xs])
    d['eout.0'] = npy(y)
    np.savez_compressed(os.path.join(OUT, 'tdetect.npz'), **d)
    print('wrote tdetect')
    # 4. space_to_depth
    x = rnd(2, 8, 6, 10, seed=48)
    np.savez_compressed(os.path.join(OUT, 'space_to_depth.npz'), **{'in.0': npy(x), 'out.0': npy(C.space_to_depth()(x))})
    # 5. CASPD_ODRTA (TDetect, P2-P5) parameter layout
    torch.manual_seed(49)
    model = Y.Model('/root/reference/models/CASPD_ODRTA.yaml', nc=10)
    sd = model.state_dict()
    np.savez_compressed(os.path.join(OUT, 'model_caspd_layout.npz'),
                        meta=json.dumps(dict(yaml='CASPD_ODRTA.yaml', nc=10,
                                             nparams=sum(p.numel() for p in model.parameters()),
                                             stride=[float(s_) for s_ in model.stride],
                                             shapes={k: list(v.shape) for k, v in sd.items()})))
    print('wrote model_caspd_layout', sum(p.numel() for p in model.parameters()))


def gen_c5():
    """Config-5 (yolov5l-xs-tr-cbam-spp-bifpn.yaml) extras: C3TR (global MHSA, common.py:184-189, 312-355)
    at a small head dim (4) and at head dim 32, and a whole small-width config-5 model (4-level Detect
    with the `anchors: 4` placeholder anchors, yolo.py:432-436)."""
    torch.manual_seed(21)
    module_case('c3tr_a', C.C3TR(32, 32, 2), [rnd(2, 32, 5, 7, seed=22)], dict(module='C3TR', args=[32, 32, 2]))
    torch.manual_seed(23)
    module_case('c3tr_b', C.C3TR(256, 256, 1, False), [rnd(2, 256, 9, 10, seed=24, scale=0.5)],
                dict(module='C3TR', args=[256, 256, 1, False]))
    torch.manual_seed(25)
    yml = small_yaml('/root/reference/models/yolov5l-xs-tr-cbam-spp-bifpn.yaml', 0.125, 0.33)
    model = Y.Model(deepcopy(yml), nc=3)
    gen = torch.Generator().manual_seed(26)
    randomize_bn(model, gen)
    with torch.no_grad():
        for k, v in model.state_dict().items():
            if v.dtype.is_floating_point:
                v.copy_(v.half().float())
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    x = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(27))
    model.train()
    outs = model(x)
    gups = [torch.randn(o.shape, generator=gen) * 0.1 for o in outs]
    loss = sum((o * g).sum() for o, g in zip(outs, gups))
    loss.backward()
    d = {'meta': json.dumps(dict(yaml=yml, nc=3, img=128)), 'in.0': npy(x)}
    for k, v in sd0.items():
        d[f'sd.{k}'] = v.half().numpy() if v.dtype.is_floating_point else npy(v)
    for i, (o, g) in enumerate(zip(outs, gups)):
        d[f'out.{i}'] = npy(o)
        d[f'gup.{i}'] = npy(g)
    params = dict(model.named_parameters())
    for k in list(params)[:6] + list(params)[-6:]:
        d[f'gp.{k}'] = npy(params[k].grad)
    d['gnorm'] = np.array([float(p.grad.norm()) if p.grad is not None else 0.0 for p in params.values()],
                          dtype=np.float64)
    d['pnames'] = np.array(list(params.keys()))
    model.load_state_dict(sd0)
    model.eval()
    with torch.no_grad():
        z, _ = model(x)
    d['eout.0'] = npy(z)
    np.savez_compressed(os.path.join(OUT, 'model_c5.npz'), **d)
    print('wrote model_c5', sum(v.nbytes for k, v in d.items() if k != 'meta') / 1e6, 'MB',
          sum(p.numel() for p in model.parameters()), 'params')
    # full-size parameter layout (nc=3): never-optimized in_proj params, shapes, strides
    torch.manual_seed(28)
    full = Y.Model('/root/reference/models/yolov5l-xs-tr-cbam-spp-bifpn.yaml', nc=3)
    sd = full.state_dict()
    np.savez_compressed(os.path.join(OUT, 'model_c5_layout.npz'),
                        meta=json.dumps(dict(yaml='yolov5l-xs-tr-cbam-spp-bifpn.yaml', nc=3,
                                             nparams=sum(p.numel() for p in full.parameters()),
                                             stride=[float(s_) for s_ in full.stride],
                                             anchors=full.model[-1].anchors.tolist(),
                                             shapes={k: list(v.shape) for k, v in sd.items()})))
    print('wrote model_c5_layout', sum(p.numel() for p in full.parameters()))


if __name__ == '__main__':
    which = sys.argv[1:] or ['modules', 'detect', 'loss', 'siou', 'nms', 'models', 'optim']
    for w in which:
        globals()[f'gen_{w}']()
