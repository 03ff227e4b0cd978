"""Data path: images + YOLO label files -> the reference's batch format
(uint8 [N, 3, H, W] RGB, targets [nt, 6] = (img, cls, x, y, w, h) normalised, paths, shapes), feeding
Model.to_input (uint8 -> /255 on the GPU, train.py:402 / val.py:199) and val.run.

Follows utils/datasets.py: img2label_paths (370-373), the label checks of verify_image_label (884-935),
LoadImagesAndLabels (376-656: the val / detect path load_image 659-675 -> letterbox with the rect batch shape ->
labels to pixel xyxy -> back to clipped normalised xywh -> HWC BGR to CHW RGB; with augment=True the training
path of 552-622: 4-mosaic + random_perspective with probability hyp['mosaic'], mixup, else letterbox +
random_perspective, then HSV, up-down / left-right flips -- dmayolo.augment), collate_fn (624-629),
create_dataloader (95-121, DistributedSampler under DDP), and letterbox (utils/augmentations.py:92-123).  cv2 is
absent from this image (and from the reference's import path here), so the resamplers it uses are restated on the
host in numpy: cv2.INTER_LINEAR for 8-bit images in OpenCV's fixed-point form (11-bit coefficients,
(v + 2^21) >> 22), cv2.INTER_AREA as the exact box-filter average (round to nearest), and warpAffine / cvtColor
HSV in dmayolo.augment; pixel values are therefore unpinned against cv2 (letterbox geometry is pinned by the
reference's own detect log, tutorial.ipynb:474-475).  Albumentations (optional in the reference, absent here) is
a no-op as in the reference without the package.
"""
import glob
import math
import os
import random
from pathlib import Path

import numpy as np
import torch

IMG_FORMATS = ('bmp', 'jpg', 'jpeg', 'png', 'tif', 'tiff', 'dng', 'webp', 'mpo')  # datasets.py:37


# ------------------------------------------------------------------ resamplers (cv2 restatements)

def _linear_coeffs(dst, src):
    """cv2 resize INTER_LINEAR source index / 11-bit fixed-point weights along one axis (imgwarp resizeGeneric_)"""
    scale = src / dst
    f = (np.arange(dst, dtype=np.float64) + 0.5) * scale - 0.5
    f = f.astype(np.float32)
    s = np.floor(f).astype(np.int64)
    fx = f - s
    lo = s < 0
    s[lo], fx[lo] = 0, 0.0
    hi = s >= src - 1
    s[hi], fx[hi] = src - 1, 0.0
    a1 = np.rint(fx * 2048).astype(np.int64)  # saturate_cast<short>(cbuf[k] * INTER_RESIZE_COEF_SCALE)
    a0 = np.rint((1.0 - fx) * 2048).astype(np.int64)
    s1 = np.minimum(s + 1, src - 1)
    return s, s1, a0, a1


def resize_linear(im, w, h):
    """cv2.resize(im, (w, h), interpolation=cv2.INTER_LINEAR) for uint8 HWC: horizontal pass
    D = S[x0] * a0 + S[x1] * a1 (int), vertical pass (b0 * b0' + b1 * b1' + 2^21) >> 22, saturated"""
    H0, W0 = im.shape[:2]
    if (H0, W0) == (h, w):
        return im.copy()
    xs0, xs1, a0, a1 = _linear_coeffs(w, W0)
    ys0, ys1, b0, b1 = _linear_coeffs(h, H0)
    src = im.astype(np.int64)
    rows = src[:, xs0] * a0[None, :, None] + src[:, xs1] * a1[None, :, None]  # [H0, w, C]
    v = rows[ys0] * b0[:, None, None] + rows[ys1] * b1[:, None, None]
    return np.clip((v + (1 << 21)) >> 22, 0, 255).astype(np.uint8)


def _area_weights(dst, src):
    """[dst, src] box-filter overlap weights of INTER_AREA (each row sums to 1)"""
    scale = src / dst
    wmat = np.zeros((dst, src), dtype=np.float64)
    for d in range(dst):
        f0, f1 = d * scale, (d + 1) * scale
        i0, i1 = int(math.floor(f0)), min(int(math.ceil(f1)), src)
        for i in range(i0, i1):
            wmat[d, i] = min(f1, i + 1) - max(f0, i)
        wmat[d] /= scale
    return wmat


def resize_area(im, w, h):
    """cv2.resize(..., interpolation=cv2.INTER_AREA) for a downscale: box-filter average, rounded to nearest"""
    H0, W0 = im.shape[:2]
    if W0 % w == 0 and H0 % h == 0:  # integer factors: cv2's ResizeAreaFast, integer block sum * (1 / area)
        fy, fx = H0 // h, W0 // w
        s = im.astype(np.int64).reshape(h, fy, w, fx, -1).sum((1, 3))
        return np.clip(np.rint(s.astype(np.float32) * np.float32(1.0 / (fy * fx))), 0, 255).astype(np.uint8)
    wx, wy = _area_weights(w, W0), _area_weights(h, H0)
    v = np.einsum('yi,ijc->yjc', wy, im.astype(np.float64))
    v = np.einsum('xj,yjc->yxc', wx, v)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def letterbox(im, new_shape=(640, 640), color=(114, 114, 114), auto=True, scaleFill=False, scaleup=True, stride=32):
    """utils/augmentations.py:92-123: resize (keep aspect) and pad to a stride multiple; returns (im, ratio, (dw, dh))"""
    shape = im.shape[:2]  # current shape [height, width]
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = min(new_shape[0] / shape[0], new_shape[1] / shape[1])
    if not scaleup:  # only scale down, do not scale up (for better val mAP)
        r = min(r, 1.0)
    ratio = r, r  # width, height ratios
    new_unpad = int(round(shape[1] * r)), int(round(shape[0] * r))
    dw, dh = new_shape[1] - new_unpad[0], new_shape[0] - new_unpad[1]  # wh padding
    if auto:  # minimum rectangle
        dw, dh = np.mod(dw, stride), np.mod(dh, stride)
    elif scaleFill:  # stretch
        dw, dh = 0.0, 0.0
        new_unpad = (new_shape[1], new_shape[0])
        ratio = new_shape[1] / shape[1], new_shape[0] / shape[0]
    dw /= 2  # divide padding into 2 sides
    dh /= 2
    if shape[::-1] != new_unpad:  # resize
        im = resize_linear(im, new_unpad[0], new_unpad[1])
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    out = np.empty((im.shape[0] + top + bottom, im.shape[1] + left + right, im.shape[2]), dtype=np.uint8)
    out[...] = np.asarray(color, dtype=np.uint8)
    out[top:top + im.shape[0], left:left + im.shape[1]] = im
    return out, ratio, (dw, dh)


# ------------------------------------------------------------------ labels / boxes

def img2label_paths(img_paths):
    """utils/datasets.py:370-373: /images/ -> /labels/, extension -> .txt"""
    sa, sb = os.sep + 'images' + os.sep, os.sep + 'labels' + os.sep
    return [sb.join(x.rsplit(sa, 1)).rsplit('.', 1)[0] + '.txt' for x in img_paths]


def read_labels(lb_file):
    """verify_image_label's label checks (datasets.py:903-927) for box labels: [n, 5] float32 (cls, x, y, w, h),
    duplicate rows removed (np.unique), empty / missing -> [0, 5]"""
    if not os.path.isfile(lb_file):
        return np.zeros((0, 5), dtype=np.float32)
    with open(lb_file) as f:
        rows = [x.split() for x in f.read().strip().splitlines() if len(x)]
    if any(len(x) > 8 for x in rows):
        raise NotImplementedError(f'{lb_file}: polygon (segment) labels are outside the DMA-YOLO path')
    lab = np.array(rows, dtype=np.float32)
    if not len(lab):
        return np.zeros((0, 5), dtype=np.float32)
    assert lab.shape[1] == 5, f'labels require 5 columns, {lab.shape[1]} columns detected'
    assert (lab >= 0).all(), f'negative label values {lab[lab < 0]}'
    assert (lab[:, 1:] <= 1).all(), f'non-normalized or out of bounds coordinates {lab[:, 1:][lab[:, 1:] > 1]}'
    return np.unique(lab, axis=0)


def xywhn2xyxy(x, w=640, h=640, padw=0, padh=0):
    """utils/general.py: normalised xywh -> pixel xyxy"""
    y = np.copy(x)
    y[:, 0] = w * (x[:, 0] - x[:, 2] / 2) + padw
    y[:, 1] = h * (x[:, 1] - x[:, 3] / 2) + padh
    y[:, 2] = w * (x[:, 0] + x[:, 2] / 2) + padw
    y[:, 3] = h * (x[:, 1] + x[:, 3] / 2) + padh
    return y


def xyxy2xywhn(x, w=640, h=640, clip=False, eps=0.0):
    """utils/general.py: pixel xyxy -> normalised xywh (optionally clipped to the image, 1 - eps)"""
    if clip:
        x = x.copy()
        x[:, [0, 2]] = x[:, [0, 2]].clip(0, w - eps)
        x[:, [1, 3]] = x[:, [1, 3]].clip(0, h - eps)
    y = np.copy(x)
    y[:, 0] = ((x[:, 0] + x[:, 2]) / 2) / w
    y[:, 1] = ((x[:, 1] + x[:, 3]) / 2) / h
    y[:, 2] = (x[:, 2] - x[:, 0]) / w
    y[:, 3] = (x[:, 3] - x[:, 1]) / h
    return y


def _read_bgr(path, rgb=False):
    """cv2.imread(path) (BGR uint8 HWC) through PIL, EXIF orientation applied as cv2 does; rgb=True skips the channel
    flip (the GPU composition reads RGB and writes BGR)"""
    from PIL import Image, ImageOps
    with Image.open(path) as im:
        im = ImageOps.exif_transpose(im).convert('RGB')
        return np.array(im) if rgb else np.ascontiguousarray(np.asarray(im)[:, :, ::-1])


# ------------------------------------------------------------------ dataset / loader

class LoadImagesAndLabels(torch.utils.data.Dataset):
    """utils/datasets.py:376-656 (box labels): validation / rect batches (augment=False) and the training
    augmentation path (augment=True, hyp with the hsv_* / degrees / translate / scale / shear / perspective / flip* /
    mosaic / mixup keys of data/hyps/*.yaml)."""

    def __init__(self, path, img_size=640, batch_size=16, augment=False, hyp=None, rect=False, stride=32, pad=0.0,
                 single_cls=False):
        self.img_size, self.stride, self.rect, self.augment, self.hyp = img_size, stride, rect, augment, hyp
        self.gpu_augment = False  # GpuAugmentLoader sets it: pixel work deferred to one kernel per batch
        self.mosaic = augment and not rect  # load 4 images at a time into a mosaic (only during training)
        self.mosaic_border = [-img_size // 2, -img_size // 2]
        f = []
        for p in path if isinstance(path, list) else [path]:
            p = Path(p)
            if p.is_dir():
                f += glob.glob(str(p / '**' / '*.*'), recursive=True)
            elif p.is_file():
                with open(p) as t:
                    parent = str(p.parent) + os.sep
                    f += [x.replace('./', parent) if x.startswith('./') else x for x in t.read().strip().splitlines()]
            else:
                raise FileNotFoundError(f'{p} does not exist')
        self.img_files = sorted(x.replace('/', os.sep) for x in f if x.split('.')[-1].lower() in IMG_FORMATS)
        assert self.img_files, f'No images found in {path}'
        self.label_files = img2label_paths(self.img_files)
        from PIL import Image, ImageOps
        shapes = []
        for fn in self.img_files:
            with Image.open(fn) as im:
                shapes.append(ImageOps.exif_transpose(im).size)  # (w, h), exif-corrected (exif_size)
        self.labels = [read_labels(lf) for lf in self.label_files]
        if single_cls:
            for lab in self.labels:
                lab[:, 0] = 0
        self.shapes = np.array(shapes, dtype=np.float64)
        n = len(self.shapes)
        bi = np.floor(np.arange(n) / batch_size).astype(np.int64)
        nb = bi[-1] + 1
        self.batch, self.n = bi, n
        self.indices = range(n)
        if self.rect:  # datasets.py:461-483: sort by aspect ratio, one letterbox shape per batch
            s = self.shapes
            ar = s[:, 1] / s[:, 0]
            irect = ar.argsort()
            self.img_files = [self.img_files[i] for i in irect]
            self.label_files = [self.label_files[i] for i in irect]
            self.labels = [self.labels[i] for i in irect]
            self.shapes = s[irect]
            ar = ar[irect]
            shapes = [[1, 1]] * nb
            for i in range(nb):
                ari = ar[bi == i]
                mini, maxi = ari.min(), ari.max()
                if maxi < 1:
                    shapes[i] = [maxi, 1]
                elif mini > 1:
                    shapes[i] = [1, 1 / mini]
            self.batch_shapes = np.ceil(np.array(shapes) * img_size / stride + pad).astype(np.int64) * stride

    def __len__(self):
        return len(self.img_files)

    def load_image(self, i):
        """datasets.py:659-675: BGR image, long side resized to img_size (INTER_AREA down when not augmenting)"""
        im = _read_bgr(self.img_files[i])
        h0, w0 = im.shape[:2]
        r = self.img_size / max(h0, w0)
        if r != 1:
            w, h = int(w0 * r), int(h0 * r)
            im = resize_area(im, w, h) if (r < 1 and not self.augment) else resize_linear(im, w, h)
        return im, (h0, w0), im.shape[:2]

    def load_image_raw(self, i):
        """load_image without the pixel work: the decoded image as an RGB uint8 HWC tensor (DataLoader workers hand
        tensors over through shared memory, not the pipe), its size and the size load_image would resize it to
        (augment.mosaic_canvas in gpu_compose mode; resize and RGB -> BGR then run inside dmy_mosaic_compose)"""
        im = torch.from_numpy(_read_bgr(self.img_files[i], rgb=True))
        h0, w0 = im.shape[:2]
        r = self.img_size / max(h0, w0)
        if r != 1:
            assert r > 1 or self.augment, 'the GPU composition restates the INTER_LINEAR (augment) resize only'
            return im, (h0, w0), (int(h0 * r), int(w0 * r))
        return im, (h0, w0), (h0, w0)

    def record(self, index):
        """datasets.py:552-622 up to the pixel work: every random draw in the reference's order (mosaic?, the mosaic
        and its perspective draw, mixup? and its second mosaic and beta ratio, else letterbox + perspective draw,
        HSV gains, up-down / left-right flips) and the final normalised labels.  -> dict with the canvas `img`, the
        forward map `M`, output `size`, `persp`, `changed`, `mix`, `luts`, `flipud`, `fliplr`, `labels` [n, 5],
        `shapes`; render_cpu / render_batch_gpu (dmayolo.augment) turn it into pixels."""
        from .augment import mosaic_warp, perspective_matrix, warp_labels, hsv_luts
        index = self.indices[index]
        hyp = self.hyp
        mix = None
        if self.mosaic and random.random() < hyp['mosaic']:
            img, M, size, persp, changed, labels = mosaic_warp(self, index)
            shapes = None
            if random.random() < hyp['mixup']:  # augmentations.py:271-276 (ratio drawn after the second mosaic)
                img2, M2, _, persp2, changed2, labels2 = mosaic_warp(self, random.randint(0, self.n - 1))
                mix = (img2, M2, persp2, changed2, np.random.beta(32.0, 32.0))
                labels = np.concatenate((labels, labels2), 0)
        else:
            img, (h0, w0), (h, w) = self.load_image(index)
            shape = self.batch_shapes[self.batch[index]] if self.rect else self.img_size
            img, ratio, pad = letterbox(img, shape, auto=False, scaleup=self.augment)
            shapes = (h0, w0), ((h / h0, w / w0), pad)  # for COCO mAP rescaling
            labels = self.labels[index].copy()
            if labels.size:
                labels[:, 1:] = xywhn2xyxy(labels[:, 1:], ratio[0] * w, ratio[1] * h, padw=pad[0], padh=pad[1])
            M, size, persp, changed = np.eye(3), (img.shape[1], img.shape[0]), 0.0, False
            if self.augment:
                persp = hyp['perspective']
                M, sc, size, changed = perspective_matrix(img.shape, hyp['degrees'], hyp['translate'], hyp['scale'],
                                                          hyp['shear'], persp)
                labels = warp_labels(labels, M, sc, size, persp)
        nl = len(labels)
        if nl:
            labels[:, 1:5] = xyxy2xywhn(labels[:, 1:5], w=size[0], h=size[1], clip=True, eps=1E-3)
        luts, fud, flr = None, False, False
        if self.augment:
            luts = hsv_luts(hyp['hsv_h'], hyp['hsv_s'], hyp['hsv_v'])
            if random.random() < hyp['flipud']:
                fud = True
                if nl:
                    labels[:, 2] = 1 - labels[:, 2]
            if random.random() < hyp['fliplr']:
                flr = True
                if nl:
                    labels[:, 1] = 1 - labels[:, 1]
        return dict(img=img, M=M, size=size, persp=persp, changed=changed, mix=mix, luts=luts, flipud=fud,
                    fliplr=flr, labels=labels, shapes=shapes)

    def __getitem__(self, index):
        """datasets.py:552-622.  With gpu_augment the pixel work is deferred: the item's image is the record
        (collate_fn keeps it) and GpuAugmentLoader renders the batch on the GPU."""
        from .augment import render_cpu
        rec = self.record(index)
        nl = len(rec['labels'])
        labels_out = torch.zeros((nl, 6))
        if nl:
            labels_out[:, 1:] = torch.from_numpy(rec['labels'])
        if self.gpu_augment:
            return rec, labels_out, self.img_files[self.indices[index]], rec['shapes']
        img = render_cpu(rec)
        img = np.ascontiguousarray(img.transpose((2, 0, 1))[::-1])  # HWC to CHW, BGR to RGB
        return torch.from_numpy(img), labels_out, self.img_files[self.indices[index]], rec['shapes']

    @staticmethod
    def collate_fn(batch):
        """datasets.py:624-629: stack images, image index into column 0 of the concatenated labels (deferred
        records -- gpu_augment -- are passed through as a list)"""
        img, label, path, shapes = zip(*batch)
        for i, lab in enumerate(label):
            lab[:, 0] = i
        imgs = list(img) if isinstance(img[0], dict) else torch.stack(img, 0)
        return imgs, torch.cat(label, 0), path, shapes


class GpuAugmentLoader:
    """Iterates a DataLoader over deferred records (the workers decode, resize, compose mosaics and draw the random
    parameters) and renders every batch with one dmy_augment_batch launch on `device`: yields
    (uint8 [B, 3, H, W] on the GPU, targets [nt, 6], paths, shapes) like the host path, bit-identical to it."""

    def __init__(self, loader, device):
        self.loader, self.device = loader, device
        self.dataset, self.sampler = loader.dataset, loader.sampler

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        from .augment import render_batch_gpu
        for recs, targets, paths, shapes in self.loader:
            yield render_batch_gpu(recs, self.device), targets, paths, shapes


def create_dataloader(path, imgsz, batch_size, stride, single_cls=False, hyp=None, augment=False, pad=0.0, rect=False,
                      rank=-1, workers=8, shuffle=False, gpu_augment=None, gpu_compose=True):
    """utils/datasets.py:95-121 (torch DataLoader; DistributedSampler under DDP so ranks shard the images).
    gpu_augment=<device>: the augmentation tail runs on that GPU (GpuAugmentLoader); gpu_compose: the mosaic canvases
    (resize + placement) as well."""
    dataset = LoadImagesAndLabels(path, imgsz, batch_size, augment=augment, hyp=hyp, rect=rect, stride=int(stride),
                                  pad=pad, single_cls=single_cls)
    dataset.gpu_augment = gpu_augment is not None
    # mosaic canvases composed on the GPU too (dmy_mosaic_compose): the workers only decode and draw
    dataset.gpu_compose = gpu_augment is not None and gpu_compose
    batch_size = min(batch_size, len(dataset))
    nw = min([os.cpu_count() or 1, batch_size if batch_size > 1 else 0, workers])
    sampler = None if rank == -1 else torch.utils.data.distributed.DistributedSampler(dataset, shuffle=shuffle)
    # persistent workers: the reference's InfiniteDataLoader (datasets.py:124-141) reuses its workers across epochs
    loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle and sampler is None,
                                         num_workers=nw, sampler=sampler, pin_memory=True,
                                         collate_fn=LoadImagesAndLabels.collate_fn, persistent_workers=nw > 0)
    if gpu_augment is not None:
        loader = GpuAugmentLoader(loader, gpu_augment)
    return loader, dataset
