"""CPU: the drop-in Model/parse_model builds the reference YAMLs with identical state_dict keys,
shapes and parameter counts (the plugin boundary, models/yolo.py:353-478)."""
import os

import pytest
import torch
import yaml

from golden_util import Fixture

YAMLS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'dma-yolo_amd', 'dmayolo', 'configs')


@pytest.mark.parametrize('name', ['model_v5s', 'model_dma'])
def test_state_dict_matches_reference(name):
    from dmayolo.models.yolo import Model
    fx = Fixture(name)
    m = Model(fx.meta['yaml'], nc=fx.meta['nc'])
    sd = m.state_dict()
    ref = fx.group('sd')
    assert set(sd) == set(ref), set(sd) ^ set(ref)
    for k, v in ref.items():
        assert tuple(sd[k].shape) == tuple(v.shape), k


@pytest.mark.parametrize('cfg,nc,params', [('yolov5s.yaml', 10, 7046599), ('yolov5n.yaml', 80, 1872157),
                                           ('yolov5l-ca-sppfcspc-bifpn-scconv.yaml', 10, 81276228)])
def test_param_counts(cfg, nc, params):
    from dmayolo.models.yolo import Model
    m = Model(os.path.join(YAMLS, cfg), nc=nc)
    assert sum(p.numel() for p in m.parameters()) == params
    det = m.model[-1]
    assert det.stride.tolist() == [8.0, 16.0, 32.0]
    # BN defaults applied (utils/torch_utils.py:161-170)
    bns = [b for b in m.modules() if type(b) is torch.nn.BatchNorm2d]
    assert bns and all(b.eps == 1e-3 and b.momentum == 0.03 for b in bns)


def test_optimizer_groups_match_reference():
    from dmayolo.models.yolo import Model
    from dmayolo.optim import param_groups
    fx = Fixture('optim')
    groups = fx.meta['groups']
    m = Model(fx.meta['yaml'], nc=3)
    names = {id(p): k for k, p in m.named_parameters()}
    g0, g1, g2 = param_groups(m)
    assert [names[id(p)] for p in g0] == groups['g0']
    assert [names[id(p)] for p in g1] == groups['g1']
    assert [names[id(p)] for p in g2] == groups['g2']


def test_caspd_tdetect_layout_matches_reference():
    """CASPD_ODRTA (space_to_depth + C3CA + TDetect P2-P5): parameter count, state_dict shapes, strides."""
    from dmayolo.models.yolo import Model
    fx = Fixture('model_caspd_layout')
    m = Model(os.path.join(YAMLS, 'CASPD_ODRTA.yaml'), nc=fx.meta['nc'])
    sd = m.state_dict()
    ref = fx.meta['shapes']
    assert set(sd) == set(ref), set(sd) ^ set(ref)
    for k, v in ref.items():
        assert list(sd[k].shape) == v, k
    assert sum(p.numel() for p in m.parameters()) == fx.meta['nparams']
    assert [float(s) for s in m.stride] == fx.meta['stride']
