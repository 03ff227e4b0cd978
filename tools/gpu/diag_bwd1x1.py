"""Which 1x1 Conv-BN-act backwards of a model take the fused kernel (bwd1x1.hip) and why the others do not: one train
step at a small resolution with functional._bwd1x1 wrapped, one line per 1x1 train-BN layer.
python tools/gpu/diag_bwd1x1.py [yaml] [img] [bs]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]
import torch  # noqa: E402
from dmayolo import functional as fn  # noqa: E402
from dmayolo.models.yolo import Model  # noqa: E402
from dmayolo.trainer import Trainer  # noqa: E402
from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp, CONFIGS  # noqa: E402

yml = sys.argv[1] if len(sys.argv) > 1 else 'yolov5l-ca-sppfcspc-bifpn-scconv.yaml'
img = int(sys.argv[2]) if len(sys.argv) > 2 else 256
bs = int(sys.argv[3]) if len(sys.argv) > 3 else 2
orig = fn._bwd1x1
seen = collections.Counter()


def wrapped(ctx, dy, dps, x, xps, wt, z, scale, shift, mean, invstd, ca, cb, cc, N, C, H, W, K, k, s, p, M):
    r = orig(ctx, dy, dps, x, xps, wt, z, scale, shift, mean, invstd, ca, cb, cc, N, C, H, W, K, k, s, p, M)
    if k == 1 and ctx.train_bn:
        why = 'fused' if r is not None else ','.join(n for n, c in (
            ('needs_dx', not ctx.needs_input_grad[0]), ('needs_dw', not ctx.needs_input_grad[1]),
            ('wt', wt is None), ('s2d', bool(ctx.s2d)), ('cp', ctx.cp != C), ('dtype', dy.dtype != torch.bfloat16),
            ('stride', s != 1 or p != 0)) if c) or \
            f'ok-query (K {K} C {C} dps {dps} xps {xps} sink {ctx.xsink is not None})'
        seen[(K, C, why)] += 1
    return r


fn._bwd1x1 = wrapped
torch.manual_seed(0)
m = Model(os.path.join(CONFIGS, yml), nc=10, act_dtype=torch.bfloat16).cuda().train()
m.hyp = scaled_hyp(HYP_VISDRONE, 10, img)
tr = Trainer(m, dict(m.hyp), 64, nb=100)
tr.step(images(bs, img, seed=1, device='cuda'), targets(bs, 10, seed=1, device='cuda'))
torch.cuda.synchronize()
for (K, C, why), n in sorted(seen.items()):
    print(f'K {K:5d} C {C:5d} x{n:3d}: {why}')
