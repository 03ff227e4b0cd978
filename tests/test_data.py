"""CPU: the data path (dmayolo.data; utils/datasets.py:95-121, 370-373, 376-656, 659-675, 884-935 and
utils/augmentations.py:92-123).  Letterbox geometry is pinned by the reference's own detect log
(tutorial.ipynb:474-475: bus.jpg 1080x810 -> 640x480, zidane.jpg 720x1280 -> 384x640 at --img 640); the cv2
resamplers are restated (cv2 absent) and checked against their defining properties; the dataset / collate path is
checked end to end on a synthetic images/ + labels/ tree."""
import os

import numpy as np
import pytest
import torch


def test_letterbox_shapes_match_reference_detect_log():
    from dmayolo.data import letterbox
    for (h, w), exp in (((1080, 810), (640, 480)), ((720, 1280), (384, 640))):
        im = np.full((h, w, 3), 7, dtype=np.uint8)
        out, ratio, (dw, dh) = letterbox(im, 640, stride=32, auto=True)
        assert out.shape[:2] == exp, (h, w, out.shape)
    out, ratio, (dw, dh) = letterbox(np.zeros((720, 1280, 3), np.uint8), 640, auto=False)
    assert out.shape[:2] == (640, 640) and ratio == (0.5, 0.5) and (dw, dh) == (0.0, 140.0)
    assert (out[:140] == 114).all() and (out[-140:] == 114).all() and (out[140:500] == 0).all()
    out, ratio, _ = letterbox(np.zeros((100, 300, 3), np.uint8), (640, 640), auto=False, scaleFill=True)
    assert out.shape[:2] == (640, 640) and ratio == (640 / 300, 640 / 100)
    out, ratio, _ = letterbox(np.zeros((100, 300, 3), np.uint8), 640, auto=False, scaleup=False)
    assert out.shape[:2] == (640, 640) and ratio == (1.0, 1.0)


def test_resize_linear_properties():
    from dmayolo.data import resize_linear
    g = np.random.default_rng(0)
    im = g.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    assert np.array_equal(resize_linear(im, 53, 37), im)
    const = np.full((20, 30, 3), 200, dtype=np.uint8)
    assert (resize_linear(const, 47, 13) == 200).all()
    # against float bilinear (half-pixel centres, edge clamp): within one grey level
    out = resize_linear(im, 80, 61).astype(np.float64)
    ys = np.clip((np.arange(61) + 0.5) * 37 / 61 - 0.5, 0, None)
    xs = np.clip((np.arange(80) + 0.5) * 53 / 80 - 0.5, 0, None)
    y0 = np.minimum(np.floor(ys).astype(int), 36)
    x0 = np.minimum(np.floor(xs).astype(int), 52)
    fy, fx = ys - y0, xs - x0
    y1, x1 = np.minimum(y0 + 1, 36), np.minimum(x0 + 1, 52)
    f = im.astype(np.float64)
    ref = ((f[y0][:, x0] * (1 - fx)[None, :, None] + f[y0][:, x1] * fx[None, :, None]) * (1 - fy)[:, None, None]
           + (f[y1][:, x0] * (1 - fx)[None, :, None] + f[y1][:, x1] * fx[None, :, None]) * fy[:, None, None])
    assert np.abs(out - ref).max() <= 1.0


def test_resize_area_integer_factor_is_block_mean():
    from dmayolo.data import resize_area
    g = np.random.default_rng(1)
    im = g.integers(0, 256, (40, 60, 3), dtype=np.uint8)
    out = resize_area(im, 20, 10)
    mean = im.astype(np.float64).reshape(10, 4, 20, 3, 3).mean((1, 3))
    assert np.abs(out - mean).max() <= 0.5 + 1e-6
    out2 = resize_area(im, 25, 16).astype(np.float64)  # non-integer factor: a weighted box average
    assert out2.min() >= im.min() and out2.max() <= im.max()
    flat = np.full((40, 60, 3), 93, dtype=np.uint8)
    assert (resize_area(flat, 25, 16) == 93).all()


def _tree(root, sizes, nc=4, seed=0):
    from PIL import Image
    g = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, 'images'))
    os.makedirs(os.path.join(root, 'labels'))
    for i, (h, w) in enumerate(sizes):
        im = np.full((h, w, 3), 40, dtype=np.uint8)
        rows = []
        for _ in range(3):
            bw, bh = g.uniform(0.1, 0.3), g.uniform(0.1, 0.3)
            x, y = g.uniform(bw / 2, 1 - bw / 2), g.uniform(bh / 2, 1 - bh / 2)
            c = int(g.integers(0, nc))
            im[int((y - bh / 2) * h):int((y + bh / 2) * h), int((x - bw / 2) * w):int((x + bw / 2) * w)] = (200, 60 * c, 30)
            rows.append(f'{c} {x:.6f} {y:.6f} {bw:.6f} {bh:.6f}')
        Image.fromarray(im).save(os.path.join(root, 'images', f'im{i}.png'))
        if i != 1:  # image 1 has no label file (missing -> empty labels)
            with open(os.path.join(root, 'labels', f'im{i}.txt'), 'w') as f:
                f.write('\n'.join(rows + rows[:1]) + '\n')  # a duplicate row: removed as verify_image_label does


@pytest.mark.parametrize('rect', [False, True])
def test_dataset_and_collate(tmp_path, rect):
    from dmayolo.data import create_dataloader, img2label_paths
    sizes = [(480, 640), (300, 500), (640, 360), (200, 200), (700, 400)]
    _tree(str(tmp_path), sizes)
    assert img2label_paths([os.path.join('a', 'images', 'x.png')]) == [os.path.join('a', 'labels', 'x.txt')]
    loader, ds = create_dataloader(str(tmp_path / 'images'), 320, 2, 32, rect=rect, workers=0)
    seen = 0
    for imgs, targets, paths, shapes in loader:
        assert imgs.dtype == torch.uint8 and imgs.shape[1] == 3
        assert imgs.shape[2] % 32 == 0 and imgs.shape[3] % 32 == 0
        if not rect:
            assert imgs.shape[2:] == (320, 320)
        assert targets.shape[1] == 6 and (targets[:, 0] < imgs.shape[0]).all()
        assert ((targets[:, 2:] > 0) & (targets[:, 2:] <= 1)).all()
        for b in range(imgs.shape[0]):
            t = targets[targets[:, 0] == b]
            name = os.path.basename(paths[b])
            assert len(t) == (0 if name == 'im1.png' else 3)  # duplicate row removed; missing label file -> empty
            H, W = imgs.shape[2:]
            (h0, w0), ((gh, gw), (padw, padh)) = shapes[b]
            for row in t:  # every box sits on its painted rectangle after letterboxing
                x, y = float(row[2]) * W, float(row[3]) * H
                assert tuple(imgs[b, :, int(y), int(x)].tolist())[0] == 200, (name, row)
        seen += imgs.shape[0]
    assert seen == len(sizes)


def test_deferred_mosaic_spec_composes_to_the_same_canvas(tmp_path):
    """mosaic_canvas in gpu_compose mode (decoded images + rectangles, no pixel work) composed by compose_cpu equals
    the canvas the direct path builds under the same random draws, and carries the same labels"""
    import random
    from PIL import Image
    from dmayolo.data import LoadImagesAndLabels
    from dmayolo.augment import mosaic_canvas, compose_cpu, MosaicSpec
    from dmayolo.synthetic import HYP_VISDRONE
    (tmp_path / 'images').mkdir()
    (tmp_path / 'labels').mkdir()
    rng = np.random.default_rng(5)
    for i in range(6):
        w, h = int(rng.integers(90, 230)), int(rng.integers(80, 200))
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(tmp_path / 'images' / f'{i}.png')
        (tmp_path / 'labels' / f'{i}.txt').write_text('0 0.5 0.5 0.2 0.3')
    ds = LoadImagesAndLabels(str(tmp_path / 'images'), img_size=128, batch_size=4, augment=True, hyp=dict(HYP_VISDRONE))
    for idx in range(6):
        random.seed(idx)
        ds.gpu_compose = False
        c1, l1 = mosaic_canvas(ds, idx)
        random.seed(idx)
        ds.gpu_compose = True
        sp, l2 = mosaic_canvas(ds, idx)
        assert isinstance(sp, MosaicSpec) and sp.shape == c1.shape
        assert np.array_equal(compose_cpu(sp), c1) and np.array_equal(l1, l2)

