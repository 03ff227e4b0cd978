"""Loader-fed throughput of the training data path at the north-star shape: a synthetic
VisDrone-like JPEG dataset (1360 x 765 images, 20-60 boxes each) through create_dataloader(augment=True, hyp VisDrone)
at img 1536, batch 32, on `workers` processes, rendered on the GPU (GpuAugmentLoader), with the mosaic canvases
composed on the host (numpy resize + placement in the workers) or on the GPU (dmy_mosaic_compose).
python tools/gpu/loader_bench.py [n_images] [workers] [batches]  -> one JSON line per mode"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dma-yolo_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def make_dataset(root, n, seed=0):
    from PIL import Image
    os.makedirs(os.path.join(root, 'images'), exist_ok=True)
    os.makedirs(os.path.join(root, 'labels'), exist_ok=True)
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:765, 0:1360]
    for i in range(n):
        base = np.stack([(xx * (1 + c) + yy * (2 + i % 3) + 40 * c) % 256 for c in range(3)], -1)
        im = (base + rng.integers(0, 48, base.shape)).clip(0, 255).astype(np.uint8)
        Image.fromarray(im).save(os.path.join(root, 'images', f'{i}.jpg'), quality=90)
        k = int(rng.integers(20, 60))
        wh = rng.uniform(0.01, 0.08, (k, 2))
        xy = rng.uniform(wh / 2, 1 - wh / 2)
        cls = rng.integers(0, 10, k)
        with open(os.path.join(root, 'labels', f'{i}.txt'), 'w') as f:
            f.write('\n'.join(f'{c} {x:.6f} {y:.6f} {w:.6f} {h:.6f}' for c, (x, y), (w, h) in zip(cls, xy, wh)))
    return os.path.join(root, 'images')


def main():
    from dmayolo.data import create_dataloader
    from dmayolo.synthetic import HYP_VISDRONE
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    batches = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    path = make_dataset(os.path.join(os.environ.get('TMPDIR', '/tmp'), 'dmy_loader_bench'), n)
    dev = torch.device('cuda', 0)
    for compose in (True, False):
        loader, _ = create_dataloader(path, 1536, 32, 32, hyp=dict(HYP_VISDRONE), augment=True, workers=workers,
                                      shuffle=True, gpu_augment=dev, gpu_compose=compose)
        seen, t0, done = 0, None, 0
        while done < batches + 2:
            for imgs, targets, _, _ in loader:
                torch.cuda.synchronize()
                done += 1
                print(f'{"gpu" if compose else "host"} compose batch {done}', file=sys.stderr, flush=True)
                if done == 2:  # the first two batches include the worker start-up
                    t0 = time.perf_counter()
                elif done > 2:
                    seen += imgs.shape[0]
                if done >= batches + 2:
                    break
        dt = time.perf_counter() - t0
        print(json.dumps({'mode': 'gpu_compose' if compose else 'host_compose', 'img': 1536, 'batch': 32,
                          'workers': workers, 'images': seen, 'seconds': round(dt, 3),
                          'img_per_s': round(seen / dt, 2)}), flush=True)


if __name__ == '__main__':
    main()
