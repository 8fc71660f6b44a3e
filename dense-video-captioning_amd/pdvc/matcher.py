"""Hungarian matcher (reference: pdvc/matcher.py:22-152).

Cost = cost_bbox * L1 + cost_class * focal-style class cost + cost_giou * (-GIoU), computed for every video
of the batch on the GPU in one pass.  The assignment is solved on the GPU (pdvc_lsap_f32, csrc/lsap.hip: the
algorithm and tie rule of scipy's linear_sum_assignment, so matched indices are scipy's bit for bit) with no
host round trip; `solve_padded` keeps the host/scipy route (ONE device->host copy for every block).
The reference also solves a 4x-replicated "many-to-one" problem whose result no loss uses; it is skipped.
"""
import os

import numpy as np
import torch
from scipy.optimize import linear_sum_assignment
from torch import nn

from . import _native as _n
from . import hostio
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
        C = self.cost_padded(pred_logits, pred_boxes, padded_targets(targets, pred_boxes.device))
        return [C[v, :, :len(t["labels"])] for v, t in enumerate(targets)]

    @torch.no_grad()
    def cost_padded(self, pred_logits, pred_boxes, pt):
        """All videos at once: (N, Q, Emax) cost with targets padded to Emax (padding columns are junk and
        are sliced away by the caller).  Elementwise the same operations as the reference's flat cost."""
        if (pred_logits.is_cuda and pred_logits.dtype == torch.float32
                and os.environ.get("PDVC_FUSED_CRITERION", "1") != "0"):
            # one launch: the same fp32 operations in the same order as below (csrc/setcrit.hip; a few ulp apart)
            from .ops.functions.setcrit import match_cost
            return match_cost(pred_logits, pred_boxes, pt["labels"], pt["boxes"], self.cost_alpha, self.cost_gamma,
                              self.cost_bbox, self.cost_class, self.cost_giou)
        out_prob = pred_logits.sigmoid()  # (N, Q, C)
        alpha, gamma = self.cost_alpha, self.cost_gamma
        neg = (1 - alpha) * (out_prob ** gamma) * (-(1 - out_prob + 1e-8).log())
        pos = alpha * ((1 - out_prob) ** gamma) * (-(out_prob + 1e-8).log())
        N, Q, _ = out_prob.shape
        ids = pt["labels"][:, None, :].expand(N, Q, pt["labels"].shape[1])
        c_class = pos.gather(2, ids) - neg.gather(2, ids)
        # torch.cdist(p=1) of the reference (matcher.py:105) as |dc| + |dl| in its summation order: the same bits,
        # and two small elementwise kernels instead of cdist's generic kernel (0.48 ms per step at 1024 videos)
        c_bbox = (pred_boxes[:, :, None, :] - pt["boxes"][:, None, :, :]).abs().sum(-1)
        c_giou = -generalized_box_iou(box_cl_to_xy(pred_boxes), box_cl_to_xy(pt["boxes"]))
        return self.cost_bbox * c_bbox + self.cost_class * c_class + self.cost_giou * c_giou

    @torch.no_grad()
    def forward(self, outputs, targets):
        return self.solve(self.cost_blocks(outputs["pred_logits"], outputs["pred_boxes"], targets))

    @staticmethod
    @torch.no_grad()
    def solve_device(costs, sizes, sizes_dev):
        """costs (P, Q, Emax) device float32, sizes host list (P,), sizes_dev the same as a device int32 tensor
        -> DeviceMatching: per problem the matched queries ascending and their targets, on the device."""
        P, Q, E = costs.shape
        qo = torch.zeros((P, max(E, 1)), dtype=torch.int64, device=costs.device)
        to = torch.zeros_like(qo)
        _n.call("pdvc_lsap_f32", _n.ptr(costs.contiguous()), P, Q, E, _n.int_array(tuple(sizes)),
                _n.ptr(sizes_dev), _n.ptr(qo), _n.ptr(to), _n.stream())
        return DeviceMatching(qo, to, list(sizes), sizes_dev)

    @staticmethod
    def solve_padded(costs, sizes):
        """costs: list of (N, Q, Emax) device tensors (one per decoder layer) -> per layer, per video
        (query ids, target ids); ONE device->host copy for everything."""
        flat = torch.stack(costs).cpu().numpy()  # (Ld, N, Q, Emax)
        out = []
        for layer in flat:
            res = []
            for v, e in enumerate(sizes):
                i, j = linear_sum_assignment(layer[v, :, :e])
                res.append((torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64)))
            out.append(res)
        return out

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


class DeviceMatching:
    """Matchings of P problems held on the device: queries (P, Emax) ascending, targets (P, Emax)."""

    def __init__(self, queries, targets, sizes, sizes_dev=None):
        self.queries, self.targets, self.sizes = queries, targets, sizes
        self.sizes_dev = sizes_dev  # the true per-problem counts (sizes may be a capacity bound)
        self._host = None

    def host(self):
        if self._host is None:  # device->host copies, only when a caller asks for Python lists
            q, t = self.queries.cpu(), self.targets.cpu()
            sizes = self.sizes_dev.cpu().tolist() if self.sizes_dev is not None else self.sizes
            self._host = [(q[p, :e].clone(), t[p, :e].clone()) for p, e in enumerate(sizes)]
        return self._host


class LazyIndices:
    """The reference's per-video list of (query ids, target ids) for one block of N problems of a
    DeviceMatching; materialised on the host on first access (the training step never needs it)."""

    def __init__(self, matching, block, n):
        self.matching, self.block, self.n = matching, block, n

    def __len__(self):
        return self.n

    def _list(self):
        return self.matching.host()[self.block * self.n:(self.block + 1) * self.n]

    def __getitem__(self, i):
        return self._list()[i]

    def __iter__(self):
        return iter(self._list())


def padded_targets(targets, device, capacity=None):
    """Targets of a batch padded to the largest event count: labels (N, Emax) long, boxes (N, Emax, 2)
    (padding boxes are a harmless (0.5, 0.5) segment), valid (N, Emax) bool, sizes [E_v].  capacity: pad to
    that many events per video instead (a shape-stable batch, pdvc/batch_layout.py), recorded as
    "capacity": the host-side code then sizes everything by it and reads the true counts on the device."""
    sizes = [len(t["labels"]) for t in targets]
    emax = max(max(sizes), 1)
    if capacity is not None:
        if emax > capacity:
            raise ValueError(f"padded_targets: a video has {emax} events, capacity {capacity}")
        emax = capacity
    N = len(targets)
    labels = torch.zeros(N, emax, dtype=torch.long)
    boxes = torch.full((N, emax, 2), 0.5)
    valid = torch.zeros(N, emax, dtype=torch.bool)
    for v, t in enumerate(targets):
        e = sizes[v]
        if e:
            labels[v, :e] = t["labels"].detach().cpu()
            boxes[v, :e] = t["boxes"].detach().cpu()
            valid[v, :e] = True
    sizes_t = torch.tensor(sizes, dtype=torch.long)
    return {"labels": hostio.to_device(labels, device), "boxes": hostio.to_device(boxes, device),
            "valid": hostio.to_device(valid, device), "sizes": sizes,
            "sizes_long": hostio.to_device(sizes_t, device), "sizes_i32": hostio.to_device(sizes_t.int(), device),
            "num_boxes": hostio.to_device(sizes_t.float().clamp(min=1.0), device), "capacity": capacity}


def build_matcher(args):
    return HungarianMatcher(cost_class=args.set_cost_class, cost_bbox=args.set_cost_bbox,
                            cost_giou=args.set_cost_giou, cost_alpha=args.cost_alpha, cost_gamma=args.cost_gamma)
