"""utils/general.py counterparts on the hot path: make_divisible, box converters, and the
batched gfx950 non_max_suppression (utils/general.py:633-725)."""
import math
import os

import torch

from ..functional import call, ptr, stream


def make_divisible(x, divisor):
    """utils/general.py:450-452."""
    return math.ceil(x / divisor) * divisor


def xywh2xyxy(x):
    """utils/general.py:539-546."""
    y = x.clone()
    y[:, 0] = x[:, 0] - x[:, 2] / 2
    y[:, 1] = x[:, 1] - x[:, 3] / 2
    y[:, 2] = x[:, 0] + x[:, 2] / 2
    y[:, 3] = x[:, 1] + x[:, 3] / 2
    return y


def xyxy2xywh(x):
    """utils/general.py:529-536."""
    y = x.clone()
    y[:, 0] = (x[:, 0] + x[:, 2]) / 2
    y[:, 1] = (x[:, 1] + x[:, 3]) / 2
    y[:, 2] = x[:, 2] - x[:, 0]
    y[:, 3] = x[:, 3] - x[:, 1]
    return y


def clip_coords(boxes, shape):
    """utils/general.py:620-630 (tensor branch): clamp xyxy boxes to (height, width) in place."""
    boxes[:, 0].clamp_(0, shape[1])
    boxes[:, 1].clamp_(0, shape[0])
    boxes[:, 2].clamp_(0, shape[1])
    boxes[:, 3].clamp_(0, shape[0])


def scale_coords(img1_shape, coords, img0_shape, ratio_pad=None):
    """utils/general.py:605-617: xyxy coords from the letterboxed img1_shape back to img0_shape, in place."""
    if ratio_pad is None:
        gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
        pad = (img1_shape[1] - img0_shape[1] * gain) / 2, (img1_shape[0] - img0_shape[0] * gain) / 2
    else:
        gain = ratio_pad[0][0]
        pad = ratio_pad[1]
    coords[:, [0, 2]] -= pad[0]
    coords[:, [1, 3]] -= pad[1]
    coords[:, :4] /= gain
    clip_coords(coords, img0_shape)
    return coords


def _pow2(n, lo=2048):
    c = lo
    while c < n:
        c <<= 1
    return c


_CAP_HINT = {}  # (A, nc, multi) -> sort capacity that held every image's candidates last time
_MASK_CAP = []


def _mask_cap():
    """largest sort capacity the bitmask NMS path (dmy_nms_greedy_mask) takes; DMY_NMS_MASK=0 keeps the lazy kernel"""
    if not _MASK_CAP:
        _MASK_CAP.append(call('dmy_nms_mask_rows') if os.environ.get('DMY_NMS_MASK', '1') != '0' else 0)
    return _MASK_CAP[0]


def nms_prepare(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False, multi_label=False,
                labels=(), max_det=300):
    """argument checks and the launch plan of non_max_suppression: (fp32 contiguous prediction, plan dict) -- the
    plan's `cap` is the sort capacity the launch will use (the hint from earlier calls of this shape)"""
    assert 0 <= conf_thres <= 1 and 0 <= iou_thres <= 1
    if labels is not None and len(labels) and any(len(l) for l in labels):
        raise NotImplementedError('autolabel (labels=...) is outside the DMA-YOLO hot path')
    pred = prediction.detach()
    if pred.dtype != torch.float32:
        pred = pred.float()
    pred = pred.contiguous()
    nimg, A, no = pred.shape
    nc = no - 5
    multi = bool(multi_label and nc > 1)
    cls_ok = None
    if classes is not None:
        cls_ok = torch.zeros(nc, dtype=torch.uint8, device=pred.device)
        cls_ok[torch.tensor([c for c in classes if 0 <= c < nc], dtype=torch.long, device=pred.device)] = 1
    key = (A, nc, multi)
    plan = dict(conf=float(conf_thres), iou=float(iou_thres), multi=multi, cls_ok=cls_ok, agnostic=bool(agnostic),
                max_det=int(max_det), key=key, cap=min(_CAP_HINT.get(key, 2048), _pow2(A * (nc if multi else 1))))
    return pred, plan


def nms_buffers(dev, nimg):
    """a private (candidate counter, pinned host counts) pair for a caller that owns them, e.g. a recorded graph
    (infer.GraphedDetector): the counter starts zeroed and every call re-zeroes it, so no other stream can share it"""
    return (torch.zeros(max(nimg, 64), dtype=torch.int32, device=dev),
            torch.zeros(max(2 * nimg, 64), dtype=torch.int32, pin_memory=True))


def nms_launch(pred, plan, cap=None, bufs=None):
    """the NMS kernels of one call at sort capacity `cap`, no host synchronisation (so it can be recorded into a HIP
    graph, infer.GraphedDetector.detect): returns (cnt, out) -- cnt = [candidate counts | keep counts] (int32, in the
    stream's pinned host buffer, or the caller's own `bufs` = nms_buffers(); a device tensor inside a capture that has
    neither), out = (nimg, max_det, 6) rows; nms_finish reads them"""
    nimg, A, no = pred.shape
    dev = pred.device
    cap = plan['cap'] if cap is None else cap
    max_nms = 30000
    if bufs is not None:
        ctr, cnt = bufs[0], bufs[1][:2 * nimg]
    else:
        ctr = _nms_counter(dev, nimg)  # zero on entry; the greedy launch hands the counts to cnt and re-zeroes it
        cnt = _nms_host_counts(dev, nimg)  # pinned host memory the scan writes directly: no read-back copy
    if cnt is None:
        cnt = torch.empty(2 * nimg, dtype=torch.int32, device=dev)
    keys = torch.empty((nimg, cap), dtype=torch.int64, device=dev)
    call('dmy_nms_candidates', ptr(pred), nimg, A, no, plan['conf'], int(plan['multi']), ptr(plan['cls_ok']), ptr(keys),
         cap, ptr(ctr), stream())
    call('dmy_nms_sort', ptr(keys), cap, ptr(ctr), nimg, stream())
    out = torch.empty((nimg, plan['max_det'], 6), dtype=torch.float32, device=dev)
    if cap <= _mask_cap():  # IoU bitmask + one-wave scan (same keep set and order as the lazy greedy kernel)
        mask = torch.empty(nimg * cap * (cap // 64), dtype=torch.int64, device=dev)
        call('dmy_nms_greedy_mask', ptr(pred), nimg, A, no, plan['iou'], int(plan['agnostic']), plan['max_det'],
             max_nms, ptr(keys), cap, ptr(ctr), None, ptr(mask), ptr(out), ptr(cnt[nimg:]), ptr(cnt), stream())
    else:
        boxes = torch.empty((nimg, max_nms, 5), dtype=torch.float32, device=dev)
        call('dmy_nms_greedy', ptr(pred), nimg, A, no, plan['iou'], int(plan['agnostic']), plan['max_det'], max_nms,
             ptr(keys), cap, ptr(ctr), ptr(boxes), ptr(out), ptr(cnt[nimg:]), ptr(cnt), stream())
    return cnt, out


_NMS_CTR = {}
_NMS_HOST = {}


def _nms_host_counts(dev, nimg):
    """[candidate counts | keep counts] of the current stream's calls in pinned host memory (int32, 2 * nimg): the
    greedy / scan kernels store them there, so nms_finish reads them after a stream synchronize instead of a device ->
    host copy.  None during a graph capture that has no buffer yet (the device tensor is used then)"""
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    t = _NMS_HOST.get(key)
    if t is None or t.numel() < 2 * nimg:
        if torch.cuda.is_current_stream_capturing():
            return None
        t = _NMS_HOST[key] = torch.zeros(max(2 * nimg, 64), dtype=torch.int32, pin_memory=True)
    return t[:2 * nimg]


def _nms_counter(dev, nimg):
    """the candidate counter of the current stream: int32 [>= nimg], zero between calls (the greedy launch of each call
    copies the counts out and re-zeroes it), so a call needs no fill launch.  One per (device, stream handle) for eager
    calls, which run in issue order on that stream; a recorded graph owns its own pair (nms_buffers).  Created (zeroed) outside graph capture when possible; one created during a capture is
    zeroed by a fill recorded in that graph"""
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    t = _NMS_CTR.get(key)
    if t is None or t.numel() < nimg:
        t = torch.zeros(max(nimg, 64), dtype=torch.int32, device=dev)
        if not torch.cuda.is_current_stream_capturing():
            _NMS_CTR[key] = t
    return t


def nms_finish(plan, cap, cnt, out):
    """the one host read of a launch: the per-image detections, or None when some image had more candidates than the
    sort capacity held (the caller reruns at the capacity this records as the new hint)"""
    nimg = out.shape[0]
    if not cnt.is_cuda:  # pinned host counts written by the kernels: wait for them, read them in place
        torch.cuda.current_stream(out.device).synchronize()
    h = cnt.tolist()  # the one host synchronisation
    need = max(h[:nimg])
    if need > cap:
        _CAP_HINT[plan['key']] = _pow2(need)  # overflow: every candidate must enter the sort
        return None
    nk = h[nimg:]
    return [out[b, :nk[b]] for b in range(nimg)]


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                        multi_label=False, labels=(), max_det=300):
    """Drop-in for utils/general.py:633-725 (merge=False).  Returns a list of (k, 6) tensors
    [xyxy, conf, cls] on the input device, rows in NMS keep order.

    All per-image work runs in three HIP kernels (candidates, bitonic sort, greedy lazy-IoU scan) and the host
    synchronises ONCE per call, reading the candidate counts and keep counts together (one int32 vector).  The
    sort capacity is the power of two that held the previous call's candidates for this prediction shape; when a
    batch overflows it (its true count comes back in the same read) the call reruns once at the exact capacity, so
    the top-`max_nms` cut always sees every candidate (utils/general.py:702-703).
    """
    pred, plan = nms_prepare(prediction, conf_thres, iou_thres, classes, agnostic, multi_label, labels, max_det)
    if pred.shape[0] == 0:
        return []
    cap = plan['cap']
    while True:
        cnt, out = nms_launch(pred, plan, cap)
        res = nms_finish(plan, cap, cnt, out)
        if res is not None:
            return res
        cap = _CAP_HINT[plan['key']]
