"""CPU: the training augmentation path (dmayolo.augment; utils/augmentations.py + datasets.py load_mosaic).

No cv2 here and the reference import is refused, so OpenCV's outputs cannot be fixtures; pinned
instead: exact known answers of the fixed-point warp (identity, integer and half-pixel shifts, the 114 border), the
warp against an independent float bilinear sampler (scipy.ndimage.map_coordinates) to one grey level, the HSV
conversions on known colours and against colorsys, the geometry of random_perspective / load_mosaic by drawing
the labelled boxes into the images and checking where they land, and run-to-run reproducibility under the seeds
the reference's RNG calls consume."""
import colorsys
import os
import random

import numpy as np
import pytest
import torch

from dmayolo import augment as A


def _img(h=48, w=64, seed=0):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def test_warp_affine_identity_and_integer_shift():
    im = _img()
    assert np.array_equal(A.warp_affine(im, [[1, 0, 0], [0, 1, 0]], (64, 48)), im)
    out = A.warp_affine(im, [[1, 0, 5], [0, 1, -3]], (64, 48))  # dst(x, y) = src(x - 5, y + 3)
    assert np.array_equal(out[:45, 5:], im[3:, :59])
    assert (out[:, :5] == 114).all() and (out[45:] == 114).all()


def test_warp_affine_half_pixel_is_rounded_average():
    im = _img()
    out = A.warp_affine(im, [[1, 0, -0.5], [0, 1, 0]], (64, 48)).astype(int)  # dst(x) = src(x + 0.5)
    ref = (im[:, :-1].astype(int) + im[:, 1:].astype(int) + 1) >> 1
    assert np.array_equal(out[:, :-1], ref)


def test_warp_affine_matches_float_bilinear():
    from scipy.ndimage import map_coordinates
    yy0, xx0 = np.mgrid[0:96, 0:80].astype(np.float64)  # smooth: <= ~6 levels per pixel
    im = np.stack([127 + 120 * np.sin(xx0 / 9 + c) * np.cos(yy0 / 11 - c) for c in range(3)], -1).astype(np.uint8)
    M = A.rotation_matrix_2d(17.0, 1.13)
    M[:, 2] += (20.0, -7.0)
    out = A.warp_affine(im, M, (80, 96)).astype(int)
    Mi = np.linalg.inv(np.vstack([M, [0, 0, 1]]))
    yy, xx = np.mgrid[0:96, 0:80].astype(np.float64)
    sx = Mi[0, 0] * xx + Mi[0, 1] * yy + Mi[0, 2]
    sy = Mi[1, 0] * xx + Mi[1, 1] * yy + Mi[1, 2]
    inside = (sx >= 0) & (sx <= 78) & (sy >= 0) & (sy <= 94)
    for c in range(3):
        ref = map_coordinates(im[..., c].astype(np.float64), [sy, sx], order=1, mode='constant', cval=114.0)
        # 1/32-pixel coordinates (<= 1/64 px error) and 15-bit weights, then rounding: within ~1 level
        assert np.abs(out[..., c] - ref)[inside].max() <= 1.0
        assert np.abs(out[..., c] - ref)[inside].mean() < 0.35


def test_warp_perspective_reduces_to_affine():
    # the two paths round the 1/32-px source coordinate differently (affine: via 1/1024 fixed point, perspective:
    # round(x * 32 / w)), so compare on a smooth image where 1/32 px moves a value by < 1 level
    yy0, xx0 = np.mgrid[0:40, 0:40].astype(np.float64)
    im = np.stack([127 + 120 * np.sin(xx0 / 7 + c) * np.cos(yy0 / 8) for c in range(3)], -1).astype(np.uint8)
    M = np.eye(3)
    M[:2] = A.rotation_matrix_2d(9.0, 0.9)
    M[:2, 2] = (4.0, 6.0)
    a = A.warp_affine(im, M[:2], (40, 40)).astype(int)
    p = A.warp_perspective(im, M, (40, 40)).astype(int)
    Mi = np.linalg.inv(M)
    sx = Mi[0, 0] * xx0 + Mi[0, 1] * yy0 + Mi[0, 2]
    sy = Mi[1, 0] * xx0 + Mi[1, 1] * yy0 + Mi[1, 2]
    inside = (sx >= 1) & (sx <= 38) & (sy >= 1) & (sy <= 38)  # away from the border-value blend
    d = np.abs(a - p)[inside]
    assert d.max() <= 1 and (d > 0).mean() < 0.1
    assert (a[~inside] == p[~inside]).mean() > 0.9


@pytest.mark.parametrize('bgr,hsv', [((255, 0, 0), (120, 255, 255)), ((0, 0, 255), (0, 255, 255)),
                                     ((0, 255, 0), (60, 255, 255)), ((128, 128, 128), (0, 0, 128)),
                                     ((0, 0, 0), (0, 0, 0)), ((255, 255, 0), (90, 255, 255))])
def test_hsv_known_colours(bgr, hsv):
    px = np.array([[bgr]], dtype=np.uint8)
    assert tuple(A.bgr2hsv(px)[0, 0]) == hsv
    assert tuple(A.hsv2bgr(np.array([[hsv]], dtype=np.uint8))[0, 0]) == bgr


def test_hsv_against_colorsys_and_round_trip():
    im = _img(32, 32, seed=5)
    hsv = A.bgr2hsv(im).astype(int)
    for (y, x) in [(0, 0), (3, 7), (10, 20), (31, 31), (15, 2)]:
        b, g, r = im[y, x] / 255.0
        h, s, v = colorsys.rgb_to_hsv(r, g, b)
        assert abs(hsv[y, x, 2] - round(v * 255)) <= 1 and abs(hsv[y, x, 1] - round(s * 255)) <= 1
        dh = abs(hsv[y, x, 0] - h * 180) % 180
        assert min(dh, 180 - dh) <= 1.0
    back = A.hsv2bgr(A.bgr2hsv(im)).astype(int)
    # 8-bit HSV quantises hue to 2 degrees: bright saturated pixels come back within a few levels
    assert np.abs(back - im.astype(int)).mean() < 2.0


def test_random_perspective_identity_and_labels_follow_the_image():
    im = np.zeros((120, 160, 3), np.uint8)
    t = np.array([[1, 20.0, 30.0, 60.0, 70.0], [2, 90.0, 10.0, 150.0, 50.0]])
    for _, x1, y1, x2, y2 in t:
        im[int(y1):int(y2), int(x1):int(x2)] = 255
    out, t2 = A.random_perspective(im.copy(), t.copy(), degrees=0, translate=0, scale=0, shear=0)
    assert np.array_equal(out, im) and np.allclose(t2, t)
    random.seed(11)
    out, t2 = A.random_perspective(im.copy(), t.copy(), degrees=25, translate=0.1, scale=0.3, shear=5)
    assert len(t2)
    for _, x1, y1, x2, y2 in t2:  # the warped box bounds its warped rectangle (rotation makes it looser)
        xi, yi, xa, ya = int(np.ceil(x1)), int(np.ceil(y1)), int(x2), int(y2)
        patch = out[yi:ya, xi:xa, 0]
        assert patch.size and (patch > 200).mean() > 0.45
    bright = out[..., 0] > 200
    covered = np.zeros_like(bright)
    for _, x1, y1, x2, y2 in t2:
        covered[max(int(y1) - 1, 0):int(y2) + 2, max(int(x1) - 1, 0):int(x2) + 2] = True
    assert bright[~covered].sum() == 0


def _dataset(tmp_path, n=6, size=(200, 150)):
    from PIL import Image
    (tmp_path / 'images').mkdir()
    (tmp_path / 'labels').mkdir()
    rng = np.random.default_rng(0)
    for i in range(n):
        w, h = size
        im = np.zeros((h, w, 3), np.uint8)
        rows = []
        for _ in range(3):
            bw, bh = rng.uniform(0.15, 0.3), rng.uniform(0.15, 0.3)
            cx, cy = rng.uniform(bw / 2 + 0.02, 1 - bw / 2 - 0.02), rng.uniform(bh / 2 + 0.02, 1 - bh / 2 - 0.02)
            x1, y1, x2, y2 = (cx - bw / 2) * w, (cy - bh / 2) * h, (cx + bw / 2) * w, (cy + bh / 2) * h
            im[int(np.ceil(y1)):int(y2), int(np.ceil(x1)):int(x2)] = 255
            rows.append(f'{int(rng.integers(0, 3))} {cx:.6f} {cy:.6f} {bw:.6f} {bh:.6f}')
        Image.fromarray(im).save(tmp_path / 'images' / f'{i}.png')
        (tmp_path / 'labels' / f'{i}.txt').write_text('\n'.join(rows))
    return str(tmp_path / 'images')


def _hyp(**kw):
    from dmayolo.synthetic import HYP_VISDRONE
    h = dict(HYP_VISDRONE)
    h.update(kw)
    return h


def test_training_dataset_mosaic_labels_on_their_objects(tmp_path):
    from dmayolo.data import LoadImagesAndLabels
    collate_fn = LoadImagesAndLabels.collate_fn
    path = _dataset(tmp_path)
    # no colour / flip / mixup noise: the objects stay white on black (114 grey where the canvas shows)
    ds = LoadImagesAndLabels(path, img_size=128, batch_size=4, augment=True,
                             hyp=_hyp(hsv_h=0, hsv_s=0, hsv_v=0, fliplr=0, mixup=0))
    assert ds.mosaic
    random.seed(0)
    np.random.seed(0)
    batch = [ds[i] for i in range(4)]
    imgs, targets, _, shapes = collate_fn(batch)
    assert imgs.shape == (4, 3, 128, 128) and imgs.dtype == torch.uint8 and shapes == (None,) * 4
    assert targets.shape[1] == 6 and len(targets) > 0
    assert (targets[:, 2:] >= 0).all() and (targets[:, 2:] <= 1).all()
    for b, c, x, y, w, h in targets.tolist():
        x1, y1, x2, y2 = (x - w / 2) * 128, (y - h / 2) * 128, (x + w / 2) * 128, (y + h / 2) * 128
        patch = imgs[int(b), 0, int(np.ceil(y1)):int(y2), int(np.ceil(x1)):int(x2)]
        if patch.numel() >= 16:
            assert (patch > 200).float().mean() > 0.5


def test_training_dataset_reproducible_and_flips(tmp_path):
    from dmayolo.data import LoadImagesAndLabels
    path = _dataset(tmp_path)
    ds = LoadImagesAndLabels(path, img_size=128, batch_size=4, augment=True, hyp=_hyp())
    outs = []
    for _ in range(2):
        random.seed(3)
        np.random.seed(3)
        outs.append([ds[i] for i in range(3)])
    for a, b in zip(*outs):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    # left-right flip mirrors the labels' x
    ds2 = LoadImagesAndLabels(path, img_size=128, batch_size=4, augment=True,
                              hyp=_hyp(mosaic=0, hsv_h=0, hsv_s=0, hsv_v=0, fliplr=1.0, degrees=0, scale=0))
    ds3 = LoadImagesAndLabels(path, img_size=128, batch_size=4, augment=True,
                              hyp=_hyp(mosaic=0, hsv_h=0, hsv_s=0, hsv_v=0, fliplr=0.0, degrees=0, scale=0))
    random.seed(5)
    im2, l2, _, _ = ds2[1]
    random.seed(5)
    im3, l3, _, _ = ds3[1]
    assert torch.equal(im2, im3.flip(-1))
    assert torch.allclose(l2[:, 2], 1 - l3[:, 2], atol=1e-6) and torch.allclose(l2[:, 3:], l3[:, 3:])


def test_mixup_blends_and_concatenates():
    np.random.seed(0)
    a, b = np.full((8, 8, 3), 200, np.uint8), np.full((8, 8, 3), 100, np.uint8)
    la, lb = np.ones((2, 5)), np.zeros((3, 5))
    im, lab = A.mixup(a, la, b, lb)
    assert 130 <= int(im[0, 0, 0]) <= 170 and lab.shape == (5, 5)


def test_aug_desc_layout_matches_library():
    """the host-built descriptor (augment.AUG_DESC) has the C struct's size (the library loads without a GPU)"""
    from dmayolo._lib import call
    assert call('dmy_aug_desc_bytes') == A.AUG_DESC.itemsize == 984
    assert A.AUG_DESC.fields['lut'][1] == 984 - 768 and A.AUG_DESC.fields['mix_r'][1] == 160
