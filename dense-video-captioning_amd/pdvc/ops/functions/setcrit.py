"""The set criterion's matching cost and loss terms as native launches (csrc/setcrit.hip).

Reference: HungarianMatcher.forward's cost (pdvc/matcher.py:87-117) and SetCriterion.loss_labels / loss_boxes /
cross_entropy_with_gaussian_mask / sigmoid_focal_loss (pdvc/criterion.py:46-123, 200-248).  Over the stacked
(decoder layer, video) problems the torch form is ~60 small launches forward and as many backward; here it is one
cost launch before the assignment, one loss launch after it (every term of every problem with its local
gradients) and one elementwise launch in the backward.
"""
import torch
from torch.autograd import Function

from pdvc import _native as _n

LOSS_KEYS = ("loss_ce", "loss_counter", "loss_bbox", "loss_giou", "loss_self_iou", "cardinality_error")
MAX_TARGETS = 64  # csrc/setcrit.hip kSetMaxE


def match_cost(logits, boxes, labels, tboxes, alpha, gamma, w_bbox, w_class, w_giou):
    """cost (P, Q, E) of HungarianMatcher.cost_padded: the same fp32 operations in the same order (a few ulp)."""
    P, Q, C = logits.shape
    E = labels.shape[1]
    cost = logits.new_empty(P, Q, E)
    _n.call("pdvc_match_cost_f32", _n.ptr(logits.contiguous()), _n.ptr(boxes.contiguous()), _n.ptr(labels),
            _n.ptr(tboxes.contiguous()), P, Q, C, E, float(alpha), float(1 - alpha), float(gamma), float(w_bbox),
            float(w_class), float(w_giou), _n.ptr(cost), _n.stream())
    return cost


class SetLossFunction(Function):
    """losses (P, 6) in LOSS_KEYS order for P problems; differentiable in logits, boxes and count (the
    cardinality column is a logged count, as in the reference: no gradient)."""

    @staticmethod
    def forward(ctx, logits, boxes, count, labels, tboxes, nmatch, num_boxes, match_query, match_target, query_mask,
                rate, focal_alpha, focal_gamma, gau_mask, beta):
        P, Q, C = logits.shape
        E, K1 = labels.shape[1], count.shape[1]
        if E > MAX_TARGETS:
            raise RuntimeError(f"set losses: at most {MAX_TARGETS} targets per problem, got {E}")
        logits, boxes, count = logits.contiguous(), boxes.contiguous(), count.contiguous()
        losses = logits.new_empty(P, 6)
        dlogit = torch.empty_like(logits)
        dcount = torch.empty_like(count)
        dbox = logits.new_empty(3, P, Q, 2)
        qm = None if query_mask is None else query_mask.to(torch.uint8).contiguous()
        _n.call("pdvc_set_losses_f32", _n.ptr(logits), _n.ptr(boxes), _n.ptr(count), _n.ptr(labels),
                _n.ptr(tboxes.contiguous()), _n.ptr(nmatch), _n.ptr(num_boxes), _n.ptr(match_query.contiguous()),
                _n.ptr(match_target.contiguous()), _n.ptr(qm) if qm is not None else None, _n.ptr(rate), P, Q, C, E,
                K1, float(focal_alpha), float(focal_gamma), int(gau_mask), float(beta), _n.ptr(losses),
                _n.ptr(dlogit), _n.ptr(dcount), _n.ptr(dbox), _n.stream())
        ctx.save_for_backward(dlogit, dcount, dbox)
        return losses

    @staticmethod
    def backward(ctx, g):
        dlogit, dcount, dbox = ctx.saved_tensors
        P, Q, C = dlogit.shape
        K1 = dcount.shape[1]
        gl, gc, gb = torch.empty_like(dlogit), torch.empty_like(dcount), dlogit.new_empty(P, Q, 2)
        _n.call("pdvc_set_losses_backward_f32", _n.ptr(g.contiguous()), _n.ptr(dlogit), _n.ptr(dcount), _n.ptr(dbox),
                P, Q, C, K1, _n.ptr(gl), _n.ptr(gc), _n.ptr(gb), _n.stream())
        return (gl, gb, gc) + (None,) * 12


def set_losses(logits, boxes, count, pt, matching, query_mask, rate, opt, focal_alpha, focal_gamma):
    """(P, 6) per-problem losses; pt: padded targets of the stacked problems, matching: DeviceMatching."""
    return SetLossFunction.apply(logits, boxes, count, pt["labels"], pt["boxes"], pt["sizes_long"], pt["num_boxes"],
                                 matching.queries, matching.targets, query_mask, rate, focal_alpha, focal_gamma,
                                 opt.lloss_gau_mask, opt.lloss_beta)
