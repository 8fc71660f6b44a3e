"""1-D segment ops (reference: misc/detr_utils/box_ops.py:7-47): (centre, length) <-> (start, end),
IoU and generalised IoU."""
import torch


def box_cl_to_xy(x):
    c, l = x.unbind(-1)
    return torch.stack([c - 0.5 * l, c + 0.5 * l], dim=-1)


def box_xy_to_cl(x):
    x0, x1 = x.unbind(-1)
    return torch.stack([(x0 + x1) / 2, (x1 - x0)], dim=-1)


def box_iou(boxes1, boxes2):
    area1 = boxes1[..., 1] - boxes1[..., 0]
    area2 = boxes2[..., 1] - boxes2[..., 0]
    lt = torch.max(boxes1[..., :, None, 0], boxes2[..., None, :, 0])
    rb = torch.min(boxes1[..., :, None, 1], boxes2[..., None, :, 1])
    inter = (rb - lt).clamp(min=0)
    union = area1[..., :, None] + area2[..., None, :] - inter
    return inter / (union + 1e-5), union


def generalized_box_iou(boxes1, boxes2):
    iou, union = box_iou(boxes1, boxes2)
    lt = torch.min(boxes1[..., :, None, 0], boxes2[..., None, :, 0])
    rb = torch.max(boxes1[..., :, None, 1], boxes2[..., None, :, 1])
    area = (rb - lt).clamp(min=0)
    return iou - (area - union) / (area + 1e-5)


def inverse_sigmoid(x, eps=1e-5):
    """misc/detr_utils/misc.py:540-544."""
    x = x.clamp(min=0, max=1)
    x1 = x.clamp(min=eps)
    x2 = (1 - x).clamp(min=eps)
    return torch.log(x1 / x2)
