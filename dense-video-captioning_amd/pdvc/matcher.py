"""Hungarian matcher (reference: pdvc/matcher.py:22-152).

Cost = cost_bbox * L1 + cost_class * focal-style class cost + cost_giou * (-GIoU), computed for every video
of the batch on the GPU in one pass; ONE device->host copy brings all cost blocks over; the assignment is
scipy's linear_sum_assignment per video (the reference's solver, so matched indices are bit-exact).
The reference also solves a 4x-replicated "many-to-one" problem whose result no loss uses; it is skipped.
"""
import numpy as np
import torch
from scipy.optimize import linear_sum_assignment
from torch import nn

from .box_ops import box_cl_to_xy, generalized_box_iou


class HungarianMatcher(nn.Module):
    def __init__(self, cost_class=1, cost_bbox=1, cost_giou=1, cost_alpha=0.25, cost_gamma=2):
        super().__init__()
        self.cost_class = cost_class
        self.cost_bbox = cost_bbox
        self.cost_giou = cost_giou
        self.cost_alpha = cost_alpha
        self.cost_gamma = cost_gamma
        assert cost_class != 0 or cost_bbox != 0 or cost_giou != 0, "all costs cant be 0"

    @torch.no_grad()
    def cost_blocks(self, pred_logits, pred_boxes, targets):
        """Per-video cost matrices (Q, E_v) as a list of device tensors (matcher.py:87-121)."""
        out_prob = pred_logits.sigmoid()  # (N, Q, C)
        alpha, gamma = self.cost_alpha, self.cost_gamma
        neg = (1 - alpha) * (out_prob ** gamma) * (-(1 - out_prob + 1e-8).log())
        pos = alpha * ((1 - out_prob) ** gamma) * (-(out_prob + 1e-8).log())
        blocks = []
        for v, t in enumerate(targets):
            ids, tb = t["labels"], t["boxes"]
            c_class = pos[v][:, ids] - neg[v][:, ids]
            c_bbox = torch.cdist(pred_boxes[v], tb, p=1)
            c_giou = -generalized_box_iou(box_cl_to_xy(pred_boxes[v]), box_cl_to_xy(tb))
            blocks.append(self.cost_bbox * c_bbox + self.cost_class * c_class + self.cost_giou * c_giou)
        return blocks

    @torch.no_grad()
    def forward(self, outputs, targets):
        return self.solve(self.cost_blocks(outputs["pred_logits"], outputs["pred_boxes"], targets))

    @staticmethod
    def solve(blocks):
        sizes = [b.shape[1] for b in blocks]
        flat = torch.cat([b.reshape(-1) for b in blocks]).cpu().numpy() if blocks else np.zeros(0)
        out, off = [], 0
        for b, e in zip(blocks, sizes):
            q = b.shape[0]
            c = flat[off:off + q * e].reshape(q, e)
            off += q * e
            i, j = linear_sum_assignment(c)
            out.append((torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64)))
        return out, None


def build_matcher(args):
    return HungarianMatcher(cost_class=args.set_cost_class, cost_bbox=args.set_cost_bbox,
                            cost_giou=args.set_cost_giou, cost_alpha=args.cost_alpha, cost_gamma=args.cost_gamma)
