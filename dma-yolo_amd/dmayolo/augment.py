"""Training augmentation of the data path: utils/augmentations.py (augment_hsv 48-62,
random_perspective 125-212, mixup 271-276, box_candidates 279-284) and utils/datasets.py load_mosaic (680-734).

cv2 is absent from this image, so the three OpenCV operations these use are restated on the host in numpy,
following OpenCV's 8-bit code paths:
  * warpAffine / warpPerspective, INTER_LINEAR, BORDER_CONSTANT (imgwarp.cpp): the inverse map in 1/32-pixel
    fixed point (AB_BITS = 10, INTER_BITS = 5, round_delta 16; perspective: X = round(x' * 32 / w)), then remap's
    bilinear tap with the 15-bit coefficient table (initInterTab2D: float products rounded to short, the largest /
    smallest entry corrected so every 2x2 set sums to 32768) and (v + 2^14) >> 15; a tap outside the image takes
    the border value, a pixel whose 2x2 window lies wholly outside is the border value.
  * cvtColor BGR2HSV (8U, hrange 180): the integer algorithm (hsv_shift 12, sdiv / hdiv tables).
  * cvtColor HSV2BGR (8U): s, v scaled by 1/255 in float32, the float sector formula, x255 and round-half-even.
Pixel values are therefore unpinned against OpenCV itself (no cv2, and the reference import is refused,
DESIGN.md §4); the geometry (matrices, mosaic placement, label transforms, candidate filter) follows the
reference line by line and draws from Python's `random` / numpy's global RNG in the reference's order.
"""
import math
import random

import numpy as np

BORDER = 114


# ------------------------------------------------------------------ cv2 restatements

def _round_half_even(x):
    return np.rint(x)  # cvRound / saturate_cast<int>(double): round half to even


def _bilinear_tab():
    """initInterTab2D for INTER_LINEAR: [32 * 32, 4] int32 coefficients (y-major: ty * 32 + tx)"""
    tab = np.zeros((32 * 32, 4), dtype=np.int64)
    for ty in range(32):
        fy = np.float32(ty) * np.float32(1.0 / 32)
        vy = (np.float32(1) - fy, fy)
        for tx in range(32):
            fx = np.float32(tx) * np.float32(1.0 / 32)
            vx = (np.float32(1) - fx, fx)
            it = [int(_round_half_even(np.float32(vy[k1] * vx[k2]) * np.float32(32768))) for k1 in (0, 1) for k2 in (0, 1)]
            diff = sum(it) - 32768
            if diff:
                mk = min(range(4), key=lambda k: (it[k], k))  # first minimum / maximum in scan order
                Mk = max(range(4), key=lambda k: (it[k], -k))
                if diff < 0:
                    it[Mk] -= diff
                else:
                    it[mk] -= diff
            tab[ty * 32 + tx] = it
    return tab


_TAB = None


def _remap_bilinear(im, X, Y, border=BORDER):
    """remap with 5-bit fractional fixed-point coordinates X, Y (int64 arrays of the destination shape)"""
    global _TAB
    if _TAB is None:
        _TAB = _bilinear_tab()
    H, W = im.shape[:2]
    sx, sy = X >> 5, Y >> 5
    w = _TAB[(Y & 31) * 32 + (X & 31)]  # [h, w, 4]
    src = im.astype(np.int64)
    C = im.shape[2]
    acc = np.zeros(X.shape + (C,), dtype=np.int64)
    for k, (dy, dx) in enumerate(((0, 0), (0, 1), (1, 0), (1, 1))):
        yy, xx = sy + dy, sx + dx
        inside = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        v = np.where(inside[..., None], src[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)], border)
        acc += v * w[..., k:k + 1]
    out = np.clip((acc + (1 << 14)) >> 15, 0, 255).astype(np.uint8)
    outside = (sx >= W) | (sx + 1 < 0) | (sy >= H) | (sy + 1 < 0)
    out[outside] = border
    return out


def affine_inverse(M):
    """warpAffine's inversion of the forward 2x3 map (imgwarp.cpp): (A11, A12, B1, A21, A22, B2)"""
    M = np.asarray(M, dtype=np.float64).reshape(2, 3)
    D = M[0, 0] * M[1, 1] - M[0, 1] * M[1, 0]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = M[1, 1] * D, M[0, 0] * D
    i01, i10 = -M[0, 1] * D, -M[1, 0] * D
    b1 = -A11 * M[0, 2] - i01 * M[1, 2]
    b2 = -i10 * M[0, 2] - A22 * M[1, 2]
    return A11, i01, b1, i10, A22, b2


def warp_affine(im, M, dsize, border=BORDER):
    """cv2.warpAffine(im, M (2x3, forward), dsize=(w, h), borderValue=(border,) * 3), INTER_LINEAR"""
    A11, i01, b1, i10, A22, b2 = affine_inverse(M)
    w, h = dsize
    x = np.arange(w, dtype=np.float64)
    y = np.arange(h, dtype=np.float64)
    adelta = _round_half_even(A11 * x * 1024).astype(np.int64)
    bdelta = _round_half_even(i10 * x * 1024).astype(np.int64)
    X0 = _round_half_even((i01 * y + b1) * 1024).astype(np.int64) + 16
    Y0 = _round_half_even((A22 * y + b2) * 1024).astype(np.int64) + 16
    X = (X0[:, None] + adelta[None, :]) >> 5
    Y = (Y0[:, None] + bdelta[None, :]) >> 5
    return _remap_bilinear(im, X, Y, border)


def warp_perspective(im, M, dsize, border=BORDER):
    """cv2.warpPerspective(im, M (3x3, forward), dsize=(w, h), borderValue=(border,) * 3), INTER_LINEAR"""
    Mi = np.linalg.inv(np.asarray(M, dtype=np.float64))
    w, h = dsize
    xx, yy = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
    W_ = Mi[2, 0] * xx + Mi[2, 1] * yy + Mi[2, 2]
    W_ = np.where(W_ != 0, 32.0 / np.where(W_ != 0, W_, 1.0), 0.0)
    fX = np.clip((Mi[0, 0] * xx + Mi[0, 1] * yy + Mi[0, 2]) * W_, -2 ** 31, 2 ** 31 - 1)
    fY = np.clip((Mi[1, 0] * xx + Mi[1, 1] * yy + Mi[1, 2]) * W_, -2 ** 31, 2 ** 31 - 1)
    return _remap_bilinear(im, _round_half_even(fX).astype(np.int64), _round_half_even(fY).astype(np.int64), border)


def rotation_matrix_2d(angle, scale, center=(0.0, 0.0)):
    """cv2.getRotationMatrix2D(center, angle (deg), scale)"""
    a = angle * math.pi / 180
    alpha, beta = math.cos(a) * scale, math.sin(a) * scale
    cx, cy = center
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy], [-beta, alpha, beta * cx + (1 - alpha) * cy]])


def _hsv_tables():
    i = np.arange(256, dtype=np.float64)
    with np.errstate(divide='ignore'):
        sdiv = np.where(i > 0, _round_half_even((255 << 12) / np.where(i > 0, i, 1)), 0).astype(np.int64)
        hdiv = np.where(i > 0, _round_half_even((180 << 12) / (6 * np.where(i > 0, i, 1))), 0).astype(np.int64)
    return sdiv, hdiv


_SDIV, _HDIV = _hsv_tables()


def bgr2hsv(im):
    """cv2.cvtColor(im, cv2.COLOR_BGR2HSV) for uint8 (H in [0, 180))"""
    b, g, r = (im[..., k].astype(np.int64) for k in range(3))
    v = np.maximum(np.maximum(b, g), r)
    vmin = np.minimum(np.minimum(b, g), r)
    diff = v - vmin
    vr = np.where(v == r, -1, 0)
    vg = np.where(v == g, -1, 0)
    s = (diff * _SDIV[v] + (1 << 11)) >> 12
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + (~vg & (r - g + 4 * diff))))
    h = (h * _HDIV[diff] + (1 << 11)) >> 12
    h = h + np.where(h < 0, 180, 0)
    return np.stack([h, s, v], -1).astype(np.uint8)


_SECTOR = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])


def hsv2bgr(hsv):
    """cv2.cvtColor(hsv, cv2.COLOR_HSV2BGR) for uint8 (float32 sector formula, x255, round half to even)"""
    f32 = np.float32
    h = hsv[..., 0].astype(f32) * f32(6.0 / 180)
    s = hsv[..., 1].astype(f32) * f32(1.0 / 255)
    v = hsv[..., 2].astype(f32) * f32(1.0 / 255)
    h = np.where(h < 0, h + 6, np.where(h >= 6, h - 6, h)).astype(f32)
    sector = np.floor(h).astype(np.int64)
    h = (h - sector.astype(f32)).astype(f32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    h = np.where(bad, f32(0), h)
    one = f32(1)
    tab = np.stack([v, v * (one - s), v * (one - s * h), v * (one - s * (one - h))], -1).astype(f32)
    idx = _SECTOR[sector]  # [..., 3] -> (b, g, r) table slots
    bgr = np.take_along_axis(tab, idx, -1)
    bgr = np.where((s == 0)[..., None], v[..., None], bgr).astype(f32)
    return np.clip(_round_half_even(bgr * f32(255)), 0, 255).astype(np.uint8)


# ------------------------------------------------------------------ augmentations (utils/augmentations.py)

def hsv_luts(hgain=0.5, sgain=0.5, vgain=0.5):
    """augmentations.py:50-58: the random gains (one numpy uniform(-1, 1, 3) draw) -> the hue / sat / val LUTs
    (uint8 [3, 256]); None when every gain is 0 (no draw, as the reference)"""
    if not (hgain or sgain or vgain):
        return None
    r = np.random.uniform(-1, 1, 3) * [hgain, sgain, vgain] + 1  # random gains
    x = np.arange(0, 256, dtype=r.dtype)
    return np.stack([((x * r[0]) % 180).astype(np.uint8), np.clip(x * r[1], 0, 255).astype(np.uint8),
                     np.clip(x * r[2], 0, 255).astype(np.uint8)])


def apply_hsv(im, luts):
    """augmentations.py:59-62: BGR -> HSV -> LUTs -> BGR, in place"""
    hsv = bgr2hsv(im)
    hsv = np.stack([luts[0][hsv[..., 0]], luts[1][hsv[..., 1]], luts[2][hsv[..., 2]]], -1)
    im[...] = hsv2bgr(hsv)


def augment_hsv(im, hgain=0.5, sgain=0.5, vgain=0.5):
    """augmentations.py:48-62, in place on a BGR uint8 image"""
    luts = hsv_luts(hgain, sgain, vgain)
    if luts is not None:
        apply_hsv(im, luts)


def box_candidates(box1, box2, wh_thr=2, ar_thr=20, area_thr=0.1, eps=1e-16):
    """augmentations.py:279-284: boxes (4, n) before / after the warp that survive it"""
    w1, h1 = box1[2] - box1[0], box1[3] - box1[1]
    w2, h2 = box2[2] - box2[0], box2[3] - box2[1]
    ar = np.maximum(w2 / (h2 + eps), h2 / (w2 + eps))
    return (w2 > wh_thr) & (h2 > wh_thr) & (w2 * h2 / (w1 * h1 + eps) > area_thr) & (ar < ar_thr)


def perspective_matrix(shape, degrees=10, translate=.1, scale=.1, shear=10, perspective=0.0, border=(0, 0)):
    """augmentations.py:129-163: the forward 3x3 map of random_perspective for an image of `shape` (h, w, ...),
    drawing from Python's `random` in the reference's order (perspective x2, angle, scale, shear x2,
    translation x2).  -> (M, s, (width, height), changed)"""
    height = shape[0] + border[0] * 2
    width = shape[1] + border[1] * 2
    C = np.eye(3)
    C[0, 2] = -shape[1] / 2
    C[1, 2] = -shape[0] / 2
    P = np.eye(3)
    P[2, 0] = random.uniform(-perspective, perspective)
    P[2, 1] = random.uniform(-perspective, perspective)
    R = np.eye(3)
    a = random.uniform(-degrees, degrees)
    s = random.uniform(1 - scale, 1 + scale)
    R[:2] = rotation_matrix_2d(a, s)
    S = np.eye(3)
    S[0, 1] = math.tan(random.uniform(-shear, shear) * math.pi / 180)
    S[1, 0] = math.tan(random.uniform(-shear, shear) * math.pi / 180)
    T = np.eye(3)
    T[0, 2] = random.uniform(0.5 - translate, 0.5 + translate) * width
    T[1, 2] = random.uniform(0.5 - translate, 0.5 + translate) * height
    M = T @ S @ R @ P @ C  # right to left
    changed = (border[0] != 0) or (border[1] != 0) or (M != np.eye(3)).any()
    return M, s, (width, height), changed


def warp_labels(targets, M, s, size, perspective=0.0):
    """augmentations.py:176-210 for box labels: corners through M, enclosing boxes clipped, box_candidates"""
    n = len(targets)
    if not n:
        return targets
    width, height = size
    xy = np.ones((n * 4, 3))
    xy[:, :2] = targets[:, [1, 2, 3, 4, 1, 4, 3, 2]].reshape(n * 4, 2)  # x1y1, x2y2, x1y2, x2y1
    xy = xy @ M.T
    xy = (xy[:, :2] / xy[:, 2:3] if perspective else xy[:, :2]).reshape(n, 8)
    x = xy[:, [0, 2, 4, 6]]
    y = xy[:, [1, 3, 5, 7]]
    new = np.concatenate((x.min(1), y.min(1), x.max(1), y.max(1))).reshape(4, n).T
    new[:, [0, 2]] = new[:, [0, 2]].clip(0, width)
    new[:, [1, 3]] = new[:, [1, 3]].clip(0, height)
    i = box_candidates(box1=targets[:, 1:5].T * s, box2=new.T, area_thr=0.10)
    targets = targets[i]
    targets[:, 1:5] = new[i]
    return targets


def warp_image(im, M, size, perspective, changed=True):
    if not changed:
        return im
    return warp_perspective(im, M, size) if perspective else warp_affine(im, M[:2], size)


def random_perspective(im, targets=(), degrees=10, translate=.1, scale=.1, shear=10, perspective=0.0, border=(0, 0)):
    """augmentations.py:125-212 for box labels (targets [n, 5] = cls, x1, y1, x2, y2 in pixels)"""
    M, s, size, changed = perspective_matrix(im.shape, degrees, translate, scale, shear, perspective, border)
    return warp_image(im, M, size, perspective, changed), warp_labels(targets, M, s, size, perspective)


def mixup(im, labels, im2, labels2):
    """augmentations.py:271-276"""
    r = np.random.beta(32.0, 32.0)  # mixup ratio, alpha = beta = 32
    im = (im * r + im2 * (1 - r)).astype(np.uint8)
    return im, np.concatenate((labels, labels2), 0)


def mosaic_canvas(ds, index):
    """datasets.py:680-724: 4-image mosaic on a 2s x 2s canvas (border 114) around a random centre, labels to
    pixel xyxy, clipped to the canvas.  copy_paste is a no-op here: it needs polygon segments, which box-label
    datasets do not have (datasets.py:902-911).  -> (canvas HWC BGR uint8, labels [n, 5])"""
    from .data import xywhn2xyxy
    labels4 = []
    s = ds.img_size
    yc, xc = (int(random.uniform(-x, 2 * s + x)) for x in ds.mosaic_border)  # mosaic centre
    indices = [index] + random.choices(ds.indices, k=3)
    random.shuffle(indices)
    img4 = None
    deferred = getattr(ds, 'gpu_compose', False)  # a MosaicSpec for dmy_mosaic_compose instead of the pixels
    quads = []
    for i, idx in enumerate(indices):
        img, _, (h, w) = ds.load_image_raw(idx) if deferred else ds.load_image(idx)
        if i == 0:  # top left
            if not deferred:
                img4 = np.full((s * 2, s * 2, img.shape[2]), BORDER, dtype=np.uint8)
            x1a, y1a, x2a, y2a = max(xc - w, 0), max(yc - h, 0), xc, yc
            x1b, y1b, x2b, y2b = w - (x2a - x1a), h - (y2a - y1a), w, h
        elif i == 1:  # top right
            x1a, y1a, x2a, y2a = xc, max(yc - h, 0), min(xc + w, s * 2), yc
            x1b, y1b, x2b, y2b = 0, h - (y2a - y1a), min(w, x2a - x1a), h
        elif i == 2:  # bottom left
            x1a, y1a, x2a, y2a = max(xc - w, 0), yc, xc, min(s * 2, yc + h)
            x1b, y1b, x2b, y2b = w - (x2a - x1a), 0, w, min(y2a - y1a, h)
        else:  # bottom right
            x1a, y1a, x2a, y2a = xc, yc, min(xc + w, s * 2), min(s * 2, yc + h)
            x1b, y1b, x2b, y2b = 0, 0, min(w, x2a - x1a), min(y2a - y1a, h)
        if deferred:
            quads.append((img, (h, w), (x1a, y1a, x2a, y2a, x1b, y1b)))
        else:
            img4[y1a:y2a, x1a:x2a] = img[y1b:y2b, x1b:x2b]
        padw, padh = x1a - x1b, y1a - y1b
        labels = ds.labels[idx].copy()
        if labels.size:
            labels[:, 1:] = xywhn2xyxy(labels[:, 1:], w, h, padw, padh)
        labels4.append(labels)
    labels4 = np.concatenate(labels4, 0)
    np.clip(labels4[:, 1:], 0, 2 * s, out=labels4[:, 1:])
    return (MosaicSpec(2 * s, quads) if deferred else img4), labels4


class MosaicSpec:
    """a mosaic canvas not yet composed: its side S2 and per quadrant (decoded RGB image tensor, resized (h, w), canvas
    rectangle (x1a, y1a, x2a, y2a) and source offset (x1b, y1b) in the resized image).  compose_cpu() / the GPU
    (render_batch_gpu -> dmy_mosaic_compose) turn it into the uint8 BGR canvas of datasets.py:680-724."""
    __slots__ = ('S2', 'quads')

    def __init__(self, S2, quads):
        self.S2, self.quads = S2, quads

    @property
    def shape(self):
        return (self.S2, self.S2, 3)


def compose_cpu(spec):
    """host restatement of the mosaic canvas from a MosaicSpec (resize_linear + placement, as mosaic_canvas)"""
    from .data import resize_linear
    img4 = np.full((spec.S2, spec.S2, 3), BORDER, dtype=np.uint8)
    for img, (h, w), (x1a, y1a, x2a, y2a, x1b, y1b) in spec.quads:
        img = np.ascontiguousarray(np.asarray(img)[:, :, ::-1])  # RGB -> BGR, as _read_bgr
        im = resize_linear(img, w, h) if img.shape[:2] != (h, w) else img
        img4[y1a:y2a, x1a:x2a] = im[y1b:y1b + (y2a - y1a), x1b:x1b + (x2a - x1a)]
    return img4


def _canvas(img):
    return compose_cpu(img) if isinstance(img, MosaicSpec) else img


MOSAIC_QUAD = np.dtype([('src', '<u8'), ('xt', '<u8'), ('yt', '<u8'), ('H0', '<i4'), ('W0', '<i4'), ('h', '<i4'),
                        ('w', '<i4'), ('x1a', '<i4'), ('y1a', '<i4'), ('x2a', '<i4'), ('y2a', '<i4'), ('x1b', '<i4'),
                        ('y1b', '<i4'), ('rgb', '<i4'), ('pad1', '<i4')])
MOSAIC_DESC = np.dtype([('dst', '<u8'), ('S2', '<i4'), ('pad', '<i4'), ('q', MOSAIC_QUAD, (4,))])


def _resize_table(dst, src):
    """[4, dst] int32: source index 0 / 1 and 11-bit weights of cv2 INTER_LINEAR along one axis (data._linear_coeffs;
    identity when no resize)"""
    from .data import _linear_coeffs
    if dst == src:
        i = np.arange(dst)
        return np.stack([i, i, np.full(dst, 2048), np.zeros(dst, np.int64)]).astype(np.int32)
    return np.stack(_linear_coeffs(dst, src)).astype(np.int32)


def compose_batch_gpu(specs, device, keep):
    """compose every MosaicSpec of a batch on `device` with ONE dmy_mosaic_compose launch; -> device canvases
    (uint8 [S2, S2, 3] tensors, kept alive through `keep` until the stream has used them)"""
    import torch
    from ._lib import call, ptr
    from .functional import stream
    assert call('dmy_mosaic_desc_bytes') == MOSAIC_DESC.itemsize, 'MosaicDesc layout mismatch'

    def up(a):
        t = (a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))).to(device, non_blocking=True)
        keep.append(t)
        return t.data_ptr()

    d = np.zeros(len(specs), dtype=MOSAIC_DESC)
    outs = []
    for n, sp in enumerate(specs):
        out = torch.empty((sp.S2, sp.S2, 3), dtype=torch.uint8, device=device)
        outs.append(out)
        d[n]['dst'], d[n]['S2'] = out.data_ptr(), sp.S2
        for k, (img, (h, w), (x1a, y1a, x2a, y2a, x1b, y1b)) in enumerate(sp.quads):
            q = d[n]['q'][k]
            q['src'], q['H0'], q['W0'], q['h'], q['w'] = up(img), img.shape[0], img.shape[1], h, w
            q['xt'], q['yt'] = up(_resize_table(w, img.shape[1])), up(_resize_table(h, img.shape[0]))
            q['rgb'] = 1  # load_image_raw's channel order: the kernel writes BGR
            q['x1a'], q['y1a'], q['x2a'], q['y2a'], q['x1b'], q['y1b'] = x1a, y1a, x2a, y2a, x1b, y1b
    descs = torch.from_numpy(d.view(np.uint8)).to(device)
    keep.append(descs)
    call('dmy_mosaic_compose', ptr(descs), len(specs), max(sp.S2 for sp in specs), stream())
    keep.extend(outs)
    return outs


def mosaic_warp(ds, index):
    """the mosaic canvas plus its random_perspective draw (datasets.py:726-734) WITHOUT resampling the image:
    -> (canvas, M, (width, height), perspective, changed, warped labels)"""
    img4, labels4 = mosaic_canvas(ds, index)
    hyp = ds.hyp
    M, s, size, changed = perspective_matrix(img4.shape, hyp['degrees'], hyp['translate'], hyp['scale'], hyp['shear'],
                                             hyp['perspective'], ds.mosaic_border)
    return img4, M, size, hyp['perspective'], changed, warp_labels(labels4, M, s, size, hyp['perspective'])


def load_mosaic(ds, index):
    """datasets.py:680-734"""
    img4, M, size, persp, changed, labels = mosaic_warp(ds, index)
    return warp_image(img4, M, size, persp, changed), labels


# ------------------------------------------------------------------ the GPU tail (csrc/augment.hip)

AUG_DESC = np.dtype([('src', '<u8'), ('src2', '<u8'), ('m', '<f8', 9), ('m2', '<f8', 9), ('mix_r', '<f8'),
                     ('H', '<i4'), ('W', '<i4'), ('H2', '<i4'), ('W2', '<i4'), ('persp', '<i4'), ('persp2', '<i4'),
                     ('copy', '<i4'), ('copy2', '<i4'), ('flipud', '<i4'), ('fliplr', '<i4'), ('use_lut', '<i4'),
                     ('pad_', '<i4'), ('lut', 'u1', (3, 256))])


def _inverse9(M, persp):
    if persp:
        return np.linalg.inv(np.asarray(M, dtype=np.float64)).reshape(9)
    m = np.zeros(9)
    m[:6] = affine_inverse(np.asarray(M)[:2])
    return m


def render_cpu(rec):
    """the host tail of one record (datasets.py:552-622 after the draws): warp, mixup, HSV, flips -> HWC BGR"""
    img = warp_image(_canvas(rec['img']), rec['M'], rec['size'], rec['persp'], rec['changed'])
    if rec['mix'] is not None:
        img2, M2, persp2, changed2, r = rec['mix']
        img = (img * r + warp_image(_canvas(img2), M2, rec['size'], persp2, changed2) * (1 - r)).astype(np.uint8)
    if rec['luts'] is not None:
        img = np.ascontiguousarray(img)
        apply_hsv(img, rec['luts'])
    if rec['flipud']:
        img = np.flipud(img)
    if rec['fliplr']:
        img = np.fliplr(img)
    return img


def render_batch_gpu(recs, device):
    """the same tail for a batch of records in ONE kernel (dmy_augment_batch): uint8 [B, 3, H, W] RGB on `device`
    (every record's output size must agree: mosaic s x s, or one rect / letterbox batch shape)"""
    import torch
    from ._lib import call, ptr
    from .functional import stream
    assert call('dmy_aug_desc_bytes') == AUG_DESC.itemsize, 'AugDesc layout mismatch'
    W, H = recs[0]['size']
    assert all(tuple(r['size']) == (W, H) for r in recs), 'one output size per batch'
    keep = []  # device canvases live until the kernel has run (stream-ordered frees)
    specs = [r['img'] for r in recs if isinstance(r['img'], MosaicSpec)] + \
        [r['mix'][0] for r in recs if r['mix'] is not None and isinstance(r['mix'][0], MosaicSpec)]
    composed = dict(zip(map(id, specs), compose_batch_gpu(specs, device, keep))) if specs else {}

    def up(a):
        if isinstance(a, MosaicSpec):
            t = composed[id(a)]
            return t.data_ptr()
        t = torch.from_numpy(np.ascontiguousarray(a)).to(device, non_blocking=True)
        keep.append(t)
        return t.data_ptr()

    d = np.zeros(len(recs), dtype=AUG_DESC)
    for i, r in enumerate(recs):
        img = r['img']
        d[i]['src'], d[i]['H'], d[i]['W'] = up(img), img.shape[0], img.shape[1]
        d[i]['persp'], d[i]['copy'] = int(bool(r['persp'])), int(not r['changed'])
        d[i]['m'] = _inverse9(r['M'], r['persp'])
        if r['mix'] is not None:
            img2, M2, persp2, changed2, mr = r['mix']
            d[i]['src2'], d[i]['H2'], d[i]['W2'] = up(img2), img2.shape[0], img2.shape[1]
            d[i]['persp2'], d[i]['copy2'] = int(bool(persp2)), int(not changed2)
            d[i]['m2'] = _inverse9(M2, persp2)
            d[i]['mix_r'] = mr
        if r['luts'] is not None:
            d[i]['use_lut'] = 1
            d[i]['lut'] = r['luts']
        d[i]['flipud'], d[i]['fliplr'] = int(r['flipud']), int(r['fliplr'])
    descs = torch.from_numpy(d.view(np.uint8)).to(device)
    out = torch.empty((len(recs), 3, H, W), dtype=torch.uint8, device=device)
    call('dmy_augment_batch', ptr(descs), len(recs), ptr(out), H, W, stream())
    keep.append(descs)
    return out
