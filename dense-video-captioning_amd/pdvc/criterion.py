"""Set criterion (reference: pdvc/criterion.py:14-256) with per-video semantics for batches.

For one video every number equals the reference's.  A batch of N videos returns, for every loss key, the
mean over videos of the per-video values (each video normalised by its own event count, exactly as the
reference's batch-size-1 training does); gradients are therefore the average of N batch-1 gradients.
The decoder layers are stacked and matched together: one cost pass, and the assignments are solved on the GPU
(pdvc_lsap_f32, scipy's algorithm and tie rule) with no host round trip -- the reference copies the costs to the
host and runs scipy once per layer.  solve_padded keeps the host route (one copy for every layer).
"""
import os

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import box_ops, hostio
from .matcher import LazyIndices, padded_targets
from .ops.functions import setcrit

COUNTER_CLASS_RATE = [0.00000000e+00, 0.00000000e+00, 1.93425917e-01, 4.12129084e-01, 1.88929963e-01,
                      7.81296833e-02, 5.09541413e-02, 3.12718553e-02, 1.84833650e-02, 8.39244680e-03,
                      6.59406534e-03, 4.49595364e-03, 2.19802178e-03, 1.79838146e-03, 5.99460486e-04,
                      4.99550405e-04, 4.99550405e-04, 1.99820162e-04, 2.99730243e-04, 3.99640324e-04,
                      2.99730243e-04, 0.00000000e+00, 1.99820162e-04, 0.00000000e+00, 0.00000000e+00,
                      0.00000000e+00, 9.99100809e-05, 9.99100809e-05]


def fused_enabled(t):
    """The native set criterion (ops/functions/setcrit.py) for float32 GPU tensors; PDVC_FUSED_CRITERION=0 keeps
    the torch form (A/B and tests)."""
    return t.is_cuda and t.dtype == torch.float32 and os.environ.get("PDVC_FUSED_CRITERION", "1") != "0"


def sigmoid_focal_terms(inputs, targets, alpha=0.25, gamma=2):
    """Elementwise focal loss (criterion.py:222-248 before its reductions)."""
    prob = inputs.sigmoid()
    ce = F.binary_cross_entropy_with_logits(inputs, targets, reduction="none")
    p_t = prob * targets + (1 - prob) * (1 - targets)
    loss = ce * ((1 - p_t) ** gamma)
    if alpha >= 0:
        loss = (alpha * targets + (1 - alpha) * (1 - targets)) * loss
    return loss


def counter_loss_terms(inputs, targets, gau_mask, beta, weight):
    """cross_entropy_with_gaussian_mask (criterion.py:200-220) up to its batch mean: (N,) per video."""
    n = targets.shape[1]
    mu = torch.arange(n, device=inputs.device).unsqueeze(0).expand(n, n).float()
    x = mu.transpose(0, 1)
    mask_dict = torch.exp(-(x - mu) ** 2 / (2 * 2 ** 2))
    _, ind = targets.max(dim=1)
    mask = mask_dict[ind]
    loss = F.binary_cross_entropy_with_logits(inputs, targets, reduction="none", weight=1 - weight)
    coef = targets + ((1 - mask) ** beta) * (1 - targets) if gau_mask else targets + (1 - targets)
    return (loss * coef).mean(1)


class SetCriterion(nn.Module):
    def __init__(self, num_classes, matcher, weight_dict, losses, focal_alpha=0.25, focal_gamma=2, opt={}):
        super().__init__()
        self.num_classes = num_classes
        self.matcher = matcher
        self.weight_dict = weight_dict
        self.losses = losses
        self.focal_alpha = focal_alpha
        self.focal_gamma = focal_gamma
        self.opt = opt
        self.counter_class_rate = torch.tensor(COUNTER_CLASS_RATE)
        self.device_matching = None  # None: match on the GPU whenever the costs live there

    # -------------------------------------------------------------------------------------------------
    def layer_losses(self, outputs, pt, indices):
        """Per-video losses of one decoder layer, averaged over the batch (see video_losses)."""
        v = self.video_losses(outputs["pred_logits"], outputs["pred_boxes"], outputs["pred_count"], pt, indices)
        return {k: t.mean() for k, t in v.items()}

    def video_losses(self, logits, boxes, count, pt, indices, pairs=None, query_mask=None):
        """Per-video loss vectors (N,) for a batch of N videos -- or of N = layers x videos when the decoder
        layers are stacked -- computed for all at once.  logits (N,Q,C), boxes (N,Q,2), count (N,K+1); pt:
        padded targets; indices: list of (query ids, target ids) per video, or None with `pairs` = device
        tensors (video, query, target, rank, per-video match count) and the largest count."""
        N, Q, C = logits.shape
        dev = logits.device
        sizes = pt["sizes"]
        nb = pt["num_boxes"]  # (N,) float, clamp(min=1)
        # matched pairs of every video, flattened: (video, query, target slot, rank) and the per-video match
        # counts -- one asynchronous host->device copy
        pvalid = None  # capacity-padded batch: the pairs of phantom targets are masked out (pdvc/batch_layout.py)
        if pairs is None:
            vid = np.concatenate([np.full(len(i), v, np.int64) for v, (i, _) in enumerate(indices)])
            qid = np.concatenate([i.numpy() for i, _ in indices])
            tid = np.concatenate([j.numpy() for _, j in indices])
            rank = np.concatenate([np.arange(len(i)) for i, _ in indices])
            nmatch = np.asarray([len(i) for i, _ in indices], np.int64)
            pv, pq, pt_, pr, n_dev = hostio.pack_to_device([vid, qid, tid, rank, nmatch], dev)
            emax = max(len(i) for i, _ in indices) if indices else 0
        elif len(pairs) == 7:
            pv, pq, pt_, pr, n_dev, emax, pvalid = pairs
        else:
            pv, pq, pt_, pr, n_dev, emax = pairs
        # labels: focal loss over every query and class (criterion.py:46-65)
        if pvalid is None:
            tclass = torch.full((N, Q), self.num_classes, dtype=torch.int64, device=dev)
            tclass[pv, pq] = pt["labels"][pv, pt_]
        else:  # a phantom pair writes into a spare column
            tclass = torch.full((N, Q + 1), self.num_classes, dtype=torch.int64, device=dev)
            tclass[pv, torch.where(pvalid, pq, Q)] = pt["labels"][pv, pt_]
            tclass = tclass[:, :Q]
        onehot = torch.zeros((N, Q, C + 1), dtype=logits.dtype, device=dev)
        onehot.scatter_(2, tclass.unsqueeze(-1), 1)
        onehot = onehot[:, :, :-1]
        focal = sigmoid_focal_terms(logits, onehot, self.focal_alpha, self.focal_gamma)  # (N,Q,C)
        if query_mask is None:
            loss_ce = focal.mean(1).sum(1) / nb * Q
        else:  # 'gt_proposals' batch: the sum over each video's real proposals (= its batch-1 mean x its Q)
            loss_ce = (focal * query_mask[:, :, None].to(focal.dtype)).sum((1, 2)) / nb
        # counter (criterion.py:67-76)
        max_length = count.shape[1] - 1
        ctgt = pt["sizes_long"].clamp(max=max_length)
        ctgt_onehot = torch.zeros_like(count)
        ctgt_onehot.scatter_(1, ctgt.unsqueeze(-1), 1)
        weight = hostio.const(("counter_class_rate", max_length), lambda: self.counter_class_rate[:max_length + 1],
                              dev)
        loss_counter = counter_loss_terms(count, ctgt_onehot, self.opt.lloss_gau_mask, self.opt.lloss_beta, weight)
        # cardinality (logging only, criterion.py:80-92)
        card_hit = logits.argmax(-1) != C - 1
        if query_mask is not None:
            card_hit = card_hit & query_mask
        card_pred = card_hit.sum(1).float()
        card_err = (card_pred - pt["sizes_long"].float()).abs()
        # boxes (criterion.py:94-123): L1 and GIoU of matched pairs, per-video sums via index_add
        src = boxes[pv, pq]
        tgt = pt["boxes"][pv, pt_]
        l1 = F.l1_loss(src, tgt, reduction="none").sum(1)
        sxy, txy = box_ops.box_cl_to_xy(src), box_ops.box_cl_to_xy(tgt)
        giou = box_ops.generalized_box_iou(sxy[:, None], txy[:, None])[:, 0, 0]
        gterm = 1 - giou
        if pvalid is not None:
            w = pvalid.to(l1.dtype)
            l1, gterm = l1 * w, gterm * w
        loss_bbox = torch.zeros(N, device=dev, dtype=l1.dtype).index_add_(0, pv, l1) / nb
        loss_giou = torch.zeros(N, device=dev, dtype=l1.dtype).index_add_(0, pv, gterm) / nb
        # self-IoU among each video's matched predictions, upper triangle, / (n(n-1)/2)
        padded = torch.zeros(N, max(emax, 1), 2, device=dev, dtype=sxy.dtype)
        padded[pv, pr] = sxy
        valid = torch.zeros(N, max(emax, 1), dtype=torch.bool, device=dev)
        valid.index_put_((pv, pr), torch.ones(pv.shape, dtype=torch.bool, device=dev) if pvalid is None
                         else pvalid)  # no host scalar
        iou = box_ops.box_iou(padded, padded)[0]
        iou = torch.triu(iou, diagonal=1) * (valid[:, :, None] & valid[:, None, :])
        n = n_dev.to(l1.dtype)
        loss_self_iou = iou.sum((1, 2)) / (0.5 * n * (n - 1))
        return {"loss_ce": loss_ce, "loss_counter": loss_counter, "loss_bbox": loss_bbox, "loss_giou": loss_giou,
                "loss_self_iou": loss_self_iou, "cardinality_error": card_err}

    def forward(self, outputs, targets, padded=None):
        """Reference contract: returns (losses, last_indices[, aux_indices]); indices are
        (list of per-video (query ids, target ids), None).  `padded` may carry padded_targets(targets)."""
        pt = padded if padded is not None else padded_targets(targets, outputs["pred_logits"].device)
        layers = [outputs] + list(outputs.get("aux_outputs", []))
        Ld = len(layers)
        N = outputs["pred_logits"].shape[0]
        # every decoder layer at once: the layers are stacked as Ld*N "videos" against repeated targets --
        # one cost pass, one device->host copy for all matchings, one pass per loss term
        ptL = repeat_targets(pt, Ld)
        logits = torch.cat([o["pred_logits"] for o in layers], 0)
        boxes = torch.cat([o["pred_boxes"] for o in layers], 0)
        count = torch.cat([o["pred_count"] for o in layers], 0)
        costs = self.matcher.cost_padded(logits, boxes, ptL)  # (Ld*N, Q, Emax)
        qm = outputs.get("query_mask")  # 'gt_proposals': padded proposal slots never match, nor enter a loss
        if qm is not None:
            qm = qm.repeat(Ld, 1)
            costs = costs.masked_fill(~qm[:, :, None], 1.0e6)
        on_device = self.device_matching if self.device_matching is not None else costs.is_cuda
        cap = pt.get("capacity")
        if cap is not None and not (on_device and costs.dtype == torch.float32 and cap <= costs.shape[1]):
            raise ValueError("a capacity-padded batch needs the device matching with capacity <= queries")
        if on_device and costs.dtype == torch.float32 and max(pt["sizes"], default=0) <= costs.shape[1]:
            # matching on the GPU (scipy's algorithm): no host round trip anywhere in the training step; a
            # capacity-padded batch passes the capacity as every problem's host bound, the counts on the device
            m = self.matcher.solve_device(costs, ptL["sizes"] if cap is None else [cap] * costs.shape[0],
                                          ptL["sizes_i32"])
            idx = [(LazyIndices(m, b, N), None) for b in range(Ld)]
            if fused_enabled(logits) and costs.shape[2] <= setcrit.MAX_TARGETS:
                # every loss term of every (layer, video) problem in one launch, its backward in one more
                max_length = count.shape[1] - 1
                rate = hostio.const(("counter_class_rate", max_length),
                                    lambda: self.counter_class_rate[:max_length + 1], logits.device)
                lv = setcrit.set_losses(logits, boxes, count, ptL, m, qm, rate, self.opt, self.focal_alpha,
                                        self.focal_gamma)  # (Ld * N, 6)
                per_layer = lv.view(Ld, N, 6).mean(1).reshape(-1).unbind(0)
                per_layer = [dict(zip(setcrit.LOSS_KEYS, per_layer[6 * i:6 * i + 6])) for i in range(Ld)]
                return self._layer_dicts(outputs, idx, per_layer)
            pp, pk, nm, emax = static_pairs(ptL)
            pairs = (pp, m.queries[pp, pk], m.targets[pp, pk], pk, nm, emax)
            if cap is not None:
                pairs = pairs + (pk < nm[pp],)
            per = self.video_losses(logits, boxes, count, ptL, None, pairs, qm)
        else:
            solved = self.matcher.solve_padded(list(costs.view(Ld, N, *costs.shape[1:])), pt["sizes"])
            idx = [(s_, None) for s_ in solved]
            per = self.video_losses(logits, boxes, count, ptL, [m_ for s_ in solved for m_ in s_], query_mask=qm)
        per = {k: v.view(Ld, N).mean(1) for k, v in per.items()}
        return self._layer_dicts(outputs, idx, [{k: v[i] for k, v in per.items()} for i in range(Ld)])

    @staticmethod
    def _layer_dicts(outputs, idx, per_layer):
        """The reference's return value: the last layer's losses, then each aux layer's under key + f"_{i}"."""
        last_indices = idx[0]
        outputs["matched_indices"] = last_indices
        losses = dict(per_layer[0])
        if "aux_outputs" in outputs:
            aux_indices = idx[1:]
            for i in range(len(per_layer) - 1):
                losses.update({k + f"_{i}": v for k, v in per_layer[i + 1].items()})
            return losses, last_indices, aux_indices
        return losses, last_indices


def static_pairs(pt):
    """(problem, rank) of every matched pair -- known from the target counts alone, since every target is
    matched -- plus the per-problem match counts and the largest; device tensors, cached on the dict."""
    key = ("pairs",)
    if key not in pt:
        # a capacity-padded batch: every (problem, rank < capacity) pair, the phantom ones masked by the caller
        sizes = pt["sizes"] if pt.get("capacity") is None else [pt["capacity"]] * len(pt["sizes"])
        pp = np.concatenate([np.full(e, p, np.int64) for p, e in enumerate(sizes)] or [np.zeros(0, np.int64)])
        pk = np.concatenate([np.arange(e) for e in sizes] or [np.zeros(0, np.int64)])
        dev = pt["sizes_long"].device
        pp_d, pk_d = hostio.pack_to_device([pp, pk], dev)
        pt[key] = (pp_d, pk_d, pt["sizes_long"], max(sizes, default=0))
    return pt[key]


def repeat_targets(pt, times):
    """Padded targets repeated for `times` stacked decoder layers (cached on the dict)."""
    if times == 1:
        return pt
    key = ("repeat", times)
    if key not in pt:
        rep = {k: (v.repeat(times, *([1] * (v.dim() - 1))) if isinstance(v, torch.Tensor) else v)
               for k, v in pt.items() if not isinstance(k, tuple)}
        rep["sizes"] = list(pt["sizes"]) * times
        pt[key] = rep
    return pt[key]
