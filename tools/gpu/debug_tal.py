"""Dump the TAL assigner intermediates (workspace) for a golden case."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'dma-yolo_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import torch  # noqa: E402
from golden_util import Fixture  # noqa: E402
from dmayolo.functional import call, ptr, stream  # noqa: E402
from dmayolo.models.tdetect import level_arrays  # noqa: E402

fx = Fixture('tal_loss_a')
meta = fx.meta
pd, pc, t = fx.t('pdist').cuda(), fx.t('pcls').cuda(), fx.t('targets').cuda()
B, _, A = pd.shape
nc = meta['nc']
nt = t.shape[0]
cap = nt
nbytes = call('dmy_tal_workspace_bytes', B, A, cap)
ws = torch.zeros(nbytes, dtype=torch.uint8, device='cuda')
G = torch.empty(B, A, 64 + nc, device='cuda')
loss, items = torch.empty(1, device='cuda'), torch.empty(3, device='cuda')
nl, H, W, S, keep = level_arrays(meta['shapes'], meta['strides'])
sb, sc = pd.stride(), pc.stride()
call('dmy_tal_loss', 0, ptr(pd), sb[0], sb[1], sb[2], ptr(pc), sc[0], sc[1], sc[2], B, nc, nl, H, W, S, ptr(t), nt,
     0.5, 6.0, float(meta['hyp']['cls_pw']), ptr(ws), ptr(G), ptr(loss), ptr(items), stream())
torch.cuda.synchronize()
off = 0


def take(nb, dt):
    global off
    v = ws[off:off + nb].view(dt)
    off += (nb + 255) // 256 * 256
    return v


gt = take(4 * B * cap * 5, torch.float32).view(B, cap, 5)
cnt = take(4 * B, torch.int32)
cand = take(4 * B * cap * 10, torch.int32).view(B, cap, 10)
nclaim = take(4 * B * A, torch.int32).view(B, A)
owner = take(4 * B * A, torch.int32).view(B, A)
metric = take(4 * B * A, torch.float32).view(B, A)
norm = take(4 * B * A, torch.float32).view(B, A)
am = take(4 * B * cap, torch.int32)
ao = take(4 * B * cap, torch.int32)
pbox = take(16 * B * A, torch.float32).view(B, A, 4)
acc = take(16, torch.float32)
print('nbytes', nbytes, 'used', off)
print('cnt', cnt.tolist(), 'acc', acc.tolist(), 'loss', loss.item(), 'items', items.tolist(), 'ref', fx.t('items').tolist())
print('gt0', gt[0, :4].tolist())
print('cand0', cand[0, :4].tolist())
print('nclaim0 nonzero', nclaim[0].nonzero().flatten().tolist())
print('pbox0', pbox[0, :3].tolist())
