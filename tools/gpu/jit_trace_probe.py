"""Probe: does the reference logger's torch.jit.trace(de_parallel(model), imgs[0:1], strict=False)
(utils/loggers/__init__.py:86, at the first batch when plots are on) run on the product model?"""
import os, sys, warnings
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]
import torch
from dmayolo.models.yolo import Model
from dmayolo.synthetic import images
m = Model(os.path.join(ROOT, 'dma-yolo_amd', 'dmayolo', 'configs', 'yolov5s.yaml'), nc=10, act_dtype=torch.bfloat16).cuda()
m.train()
x = images(2, 256, device='cuda')
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter('always')
    try:
        tr = torch.jit.trace(m, x[0:1], strict=False)
        print('trace OK;', len(w), 'warnings; first:', str(w[0].message)[:200] if w else '')
        kinds = {}
        for n in tr.inlined_graph.nodes():
            kinds[n.kind()] = kinds.get(n.kind(), 0) + 1
        print(sorted(kinds.items(), key=lambda kv: -kv[1])[:12])
    except Exception as e:
        print('trace FAILED:', type(e).__name__, str(e)[:600])
