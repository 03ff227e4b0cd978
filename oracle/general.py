"""CPU restatement of utils/general.non_max_suppression (+ torchvision.ops.nms) (TEST INFRASTRUCTURE ONLY)."""
import torch


def xywh2xyxy(x):
    """utils/general.py:539-546."""
    y = x.clone()
    y[:, 0] = x[:, 0] - x[:, 2] / 2
    y[:, 1] = x[:, 1] - x[:, 3] / 2
    y[:, 2] = x[:, 0] + x[:, 2] / 2
    y[:, 3] = x[:, 1] + x[:, 3] / 2
    return y


def greedy_nms(boxes, scores, iou_thres, max_keep=None):
    """torchvision.ops.nms CPU algorithm (third-party, torchvision>=0.8.1 unpinned, requirements.txt:12):
    stable descending score order; suppress j iff IoU(i, j) > thr; areas without +1.
    `keep` grows in score order, so stopping at max_keep returns exactly nms(...)[:max_keep]."""
    order = torch.sort(scores, stable=True, descending=True)[1]
    x1, y1, x2, y2 = boxes.unbind(1)
    area = (x2 - x1) * (y2 - y1)
    dead = torch.zeros(len(scores), dtype=torch.bool)
    keep = []
    for k in range(len(order)):
        i = order[k]
        if dead[i]:
            continue
        keep.append(int(i))
        if max_keep is not None and len(keep) >= max_keep:
            break
        rest = order[k + 1:]
        w = (torch.minimum(x2[i], x2[rest]) - torch.maximum(x1[i], x1[rest])).clamp(min=0)
        h = (torch.minimum(y2[i], y2[rest]) - torch.maximum(y1[i], y1[rest])).clamp(min=0)
        inter = w * h
        dead[rest[inter / (area[i] + area[rest] - inter) > iou_thres]] = True
    return torch.tensor(keep, dtype=torch.int64)


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                        multi_label=False, labels=(), max_det=300):
    """utils/general.py:633-725 (merge=False; the 10 s wall-clock guard is not part of the contract)."""
    nc = prediction.shape[2] - 5
    max_wh, max_nms = 4096, 30000
    multi_label &= nc > 1
    out = [torch.zeros((0, 6))] * prediction.shape[0]
    for b in range(prediction.shape[0]):
        x = prediction[b][prediction[b, :, 4] > conf_thres].clone()
        if not x.shape[0]:
            continue
        x[:, 5:] *= x[:, 4:5]
        box = xywh2xyxy(x[:, :4])
        if multi_label:
            i, j = (x[:, 5:] > conf_thres).nonzero(as_tuple=False).T
            x = torch.cat((box[i], x[i, j + 5, None], j[:, None].float()), 1)
        else:
            conf, j = x[:, 5:].max(1, keepdim=True)
            x = torch.cat((box, conf, j.float()), 1)[conf.view(-1) > conf_thres]
        if classes is not None:
            x = x[(x[:, 5:6] == torch.tensor(classes)).any(1)]
        n = x.shape[0]
        if not n:
            continue
        if n > max_nms:
            x = x[torch.sort(x[:, 4], stable=True, descending=True)[1][:max_nms]]
        c = x[:, 5:6] * (0 if agnostic else max_wh)
        keep = greedy_nms(x[:, :4] + c, x[:, 4], iou_thres, max_det)[:max_det]
        out[b] = x[keep]
    return out
