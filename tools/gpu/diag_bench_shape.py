"""Diagnostic: per-parameter gradient agreement of the bf16 product vs the fp32 oracle at a bench shape."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd'), os.path.join(ROOT, 'tests')]
import torch, yaml
from dmayolo.models.yolo import Model
from dmayolo.utils.loss import ComputeLoss
from dmayolo.synthetic import images, targets, HYP_VISDRONE, scaled_hyp, CONFIGS
from oracle import nn as onn
from oracle.loss import compute_loss
yml, img, bs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
dt = torch.float32 if len(sys.argv) > 4 and sys.argv[4] == 'fp32' else torch.bfloat16
torch.set_num_threads(16)
nc = 10
torch.manual_seed(0)
m = Model(os.path.join(CONFIGS, yml), nc=nc, act_dtype=dt)
ref = onn.bn_defaults(onn.Model(yaml.safe_load(open(os.path.join(CONFIGS, yml))), nc=nc))
ref.load_state_dict(m.state_dict())
for mod in m.modules():
    if type(mod).__name__ == 'SwinTransformerLayer':
        mod.drop_path = torch.nn.Identity()
for mod in ref.modules():
    if hasattr(mod, 'drop_prob'):
        mod.drop_prob = 0.0
hyp = scaled_hyp(HYP_VISDRONE, nc, img, 3)
m.hyp = hyp
m = m.cuda().train(); ref.train()
x = images(bs, img, seed=1); t = targets(bs, nc, seed=1)
p = m(x.cuda()); loss, items = ComputeLoss(m)(p, t.cuda()); loss.backward()
pr = ref(x.float() / 255); lr_, ir_ = compute_loss(pr, t, m.model[-1].anchors.cpu(), hyp, nc); lr_.backward()
pp, pq = dict(m.named_parameters()), dict(ref.named_parameters())
rows = []
for k in pq:
    if pq[k].grad is None: continue
    a = pp[k].grad.double().cpu().flatten(); b = pq[k].grad.double().flatten()
    cos = float(a @ b / (a.norm() * b.norm() + 1e-300))
    rows.append((float(b.norm()), k, cos, float((a - b).norm() / (b.norm() + 1e-300)), float(a.norm())))
rows.sort(reverse=True)
tot = sum(r[0] ** 2 for r in rows)
print('loss', float(loss), float(lr_), 'items', items.tolist(), ir_.tolist())
print('top by ref grad norm: norm share, param, cos, relerr, |a|/|b|')
for r in rows[:25]:
    print('%.4f %-40s cos %.4f rel %.3e ratio %.4f' % (r[0] ** 2 / tot, r[1], r[2], r[3], r[4] / (r[0] + 1e-300)))
print('worst cos among params with >0.1% of the squared norm:')
for r in sorted([r for r in rows if r[0] ** 2 / tot > 1e-3], key=lambda r: r[2])[:15]:
    print('%.4f %-40s cos %.4f rel %.3e ratio %.4f' % (r[0] ** 2 / tot, r[1], r[2], r[3], r[4] / (r[0] + 1e-300)))
lids = sorted({int(k.split('.')[1]) for k in pq if pq[k].grad is not None})


def lnorm(pg, lid):
    return float(torch.cat([pg[k].grad.double().flatten().cpu() for k in pq
                            if pq[k].grad is not None and int(k.split('.')[1]) == lid]).norm())


print('per-layer gradient norm product / fp32 oracle: ' + ' '.join(f'{lid}:{lnorm(pp, lid) / lnorm(pq, lid):.3f}'
                                                                for lid in lids))
