"""GPU: the augmentation tail kernel (csrc/augment.hip, dmy_augment_batch) against the host restatement
(dmayolo.augment.render_cpu) on the same records: bit-identical uint8 batches for mosaics with and without mixup,
HSV, both flips, a perspective warp, the non-mosaic letterbox + warp path and the no-augmentation copy path; and
the GpuAugmentLoader end to end against the host DataLoader under the same seeds."""
import os
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dataset(tmp_path, n=8, seed=0):
    from PIL import Image
    (tmp_path / 'images').mkdir()
    (tmp_path / 'labels').mkdir()
    rng = np.random.default_rng(seed)
    for i in range(n):
        w, h = int(rng.integers(120, 260)), int(rng.integers(100, 220))
        yy, xx = np.mgrid[0:h, 0:w]
        im = np.stack([(xx * (3 + c) + yy * (5 - c) + rng.integers(0, 40, (h, w))) % 256 for c in range(3)], -1)
        rows = []
        for _ in range(int(rng.integers(1, 5))):
            bw, bh = rng.uniform(0.05, 0.4), rng.uniform(0.05, 0.4)
            rows.append(f'{int(rng.integers(0, 3))} {rng.uniform(bw / 2, 1 - bw / 2):.6f} '
                        f'{rng.uniform(bh / 2, 1 - bh / 2):.6f} {bw:.6f} {bh:.6f}')
        Image.fromarray(im.astype(np.uint8)).save(tmp_path / 'images' / f'{i}.png')
        (tmp_path / 'labels' / f'{i}.txt').write_text('\n'.join(rows))
    return str(tmp_path / 'images')


def _hyp(**kw):
    from dmayolo.synthetic import HYP_VISDRONE
    h = dict(HYP_VISDRONE)
    h.update(kw)
    return h


CASES = {
    'mosaic_warp_only': dict(hsv_h=0, hsv_s=0, hsv_v=0, fliplr=0.0, mixup=0.0),
    'mosaic_hsv_flips': dict(fliplr=0.5, flipud=0.5, mixup=0.0),
    'mosaic_mixup': dict(mixup=1.0, degrees=5.0, shear=2.0),
    'mosaic_perspective': dict(perspective=0.0005, degrees=3.0, translate=0.1),
    'letterbox_warp': dict(mosaic=0.0, degrees=10.0, scale=0.3, fliplr=1.0),
}


@pytest.mark.parametrize('case', list(CASES))
def test_gpu_tail_equals_host_tail(tmp_path, case):
    from dmayolo.data import LoadImagesAndLabels
    from dmayolo.augment import render_cpu, render_batch_gpu
    ds = LoadImagesAndLabels(_dataset(tmp_path), img_size=160, batch_size=8, augment=True, hyp=_hyp(**CASES[case]))
    random.seed(7)
    np.random.seed(7)
    recs = [ds.record(i) for i in range(8)]
    host = np.stack([np.ascontiguousarray(render_cpu(r).transpose(2, 0, 1)[::-1]) for r in recs])
    dev = render_batch_gpu(recs, torch.device('cuda')).cpu().numpy()
    assert dev.shape == host.shape == (8, 3, 160, 160)
    diff = dev.astype(int) != host.astype(int)
    if diff.any():
        for b, c, y, x in list(zip(*np.nonzero(diff)))[:8]:
            print('diff at', (b, c, y, x), 'host', host[b, :, y, x], 'dev', dev[b, :, y, x])
    assert not diff.any(), f'{diff.sum()} of {diff.size} bytes differ'


def test_gpu_hsv_exhaustive_colours():
    """every 8-bit BGR colour through BGR2HSV -> LUTs -> HSV2BGR on the GPU (copy path, no warp) == the host"""
    from dmayolo.augment import render_batch_gpu, apply_hsv, hsv_luts
    c = np.arange(1 << 24, dtype=np.uint32)
    canvas = np.stack([c & 255, (c >> 8) & 255, c >> 16], -1).astype(np.uint8).reshape(4096, 4096, 3)
    np.random.seed(1)
    luts = hsv_luts(0.4, 0.7, 0.5)
    rec = dict(img=canvas, M=np.eye(3), size=(4096, 4096), persp=0.0, changed=False, mix=None, luts=luts,
               flipud=False, fliplr=False)
    dev = render_batch_gpu([rec], torch.device('cuda'))[0].cpu().numpy()
    host = canvas.copy()
    apply_hsv(host, luts)
    host = host.transpose(2, 0, 1)[::-1]
    bad = np.nonzero((dev != host).any(0).reshape(-1))[0]
    for i in bad[:8]:
        print('colour', canvas.reshape(-1, 3)[i], 'host', host.reshape(3, -1)[:, i], 'dev', dev.reshape(3, -1)[:, i])
    assert len(bad) == 0, f'{len(bad)} colours differ'


def test_gpu_tail_copy_path_without_augmentation(tmp_path):
    from dmayolo.data import LoadImagesAndLabels
    from dmayolo.augment import render_batch_gpu
    ds = LoadImagesAndLabels(_dataset(tmp_path), img_size=160, batch_size=4, augment=False, rect=True)
    recs = [ds.record(i) for i in range(4)]  # one rect batch: same letterbox shape
    out = render_batch_gpu(recs, torch.device('cuda')).cpu()
    for r, o in zip(recs, out):
        assert torch.equal(o, torch.from_numpy(np.ascontiguousarray(r['img'].transpose(2, 0, 1)[::-1])))


def test_gpu_augment_loader_matches_host_loader(tmp_path):
    from dmayolo.data import create_dataloader
    path = _dataset(tmp_path)
    hyp = _hyp(mixup=0.5, fliplr=0.5)
    outs = []
    for gpu in (None, torch.device('cuda')):
        random.seed(3)
        np.random.seed(3)
        loader, _ = create_dataloader(path, 160, 4, 32, hyp=hyp, augment=True, workers=0, gpu_augment=gpu)
        outs.append([(im.cpu(), t) for im, t, _, _ in loader])
    for (ih, th), (ig, tg) in zip(*outs):
        assert torch.equal(ih, ig) and torch.equal(th, tg)


def test_gpu_tail_throughput_at_1536():
    """one batch of 32 mosaics at 1536 (3072^2 canvases): kernel time vs the bytes it must move"""
    from dmayolo.augment import render_batch_gpu
    rng = np.random.default_rng(0)
    canvas = rng.integers(0, 256, (3072, 3072, 3), dtype=np.uint8)
    M = np.array([[0.9, 0.02, -700.0], [-0.02, 0.9, -650.0], [0.0, 0.0, 1.0]])
    luts = np.stack([np.arange(256) % 180, np.arange(256), np.arange(256)]).astype(np.uint8)
    recs = [dict(img=canvas, M=M, size=(1536, 1536), persp=0.0, changed=True, mix=None, luts=luts, flipud=False,
                 fliplr=bool(i % 2), labels=None, shapes=None) for i in range(32)]
    out = render_batch_gpu(recs, torch.device('cuda'))
    torch.cuda.synchronize()
    from dmayolo.functional import KernelTimer  # noqa: F401  (import check only)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = render_batch_gpu(recs, torch.device('cuda'))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print(f'render 32 x 1536^2 (incl. 32 canvas uploads of 28 MB): {ms:.1f} ms')
    assert out.shape == (32, 3, 1536, 1536)


@pytest.mark.parametrize('case', ['mosaic_warp_only', 'mosaic_mixup'])
def test_gpu_mosaic_compose_equals_host(tmp_path, case):
    """dmy_mosaic_compose (resize_linear + placement of the 4 decoded images on the GPU) == compose_cpu on the same
    MosaicSpecs, and the whole deferred batch (compose + tail) == render_cpu"""
    from dmayolo.data import LoadImagesAndLabels
    from dmayolo.augment import MosaicSpec, compose_cpu, compose_batch_gpu, render_cpu, render_batch_gpu
    ds = LoadImagesAndLabels(_dataset(tmp_path), img_size=160, batch_size=8, augment=True, hyp=_hyp(**CASES[case]))
    ds.gpu_compose = True
    random.seed(11)
    np.random.seed(11)
    recs = [ds.record(i) for i in range(8)]
    specs = [r['img'] for r in recs if isinstance(r['img'], MosaicSpec)]
    assert len(specs) == 8
    keep = []
    dev = [c.cpu().numpy() for c in compose_batch_gpu(specs, torch.device('cuda'), keep)]
    for sp, d in zip(specs, dev):
        h = compose_cpu(sp)
        assert d.shape == h.shape and np.array_equal(d, h), f'{int((d != h).sum())} canvas bytes differ'
    host = np.stack([np.ascontiguousarray(render_cpu(r).transpose(2, 0, 1)[::-1]) for r in recs])
    out = render_batch_gpu(recs, torch.device('cuda')).cpu().numpy()
    assert np.array_equal(out, host)
