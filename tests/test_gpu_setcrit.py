"""GPU parity of the native set criterion (csrc/setcrit.hip, pdvc/ops/functions/setcrit.py) against the torch form
of the same module (PDVC_FUSED_CRITERION=0: pdvc/criterion.py video_losses and matcher.py cost_padded, which the
CPU tests and the reference fixtures pin to the reference's pdvc/criterion.py:46-123,200-248 and matcher.py:87-117).

- the matching costs agree to a few ulp (the kernel repeats torch's fp32 operations in torch's order; exp / log /
  division may round differently from torch's kernels), and the device assignment -- the matched indices -- is the
  same;
- every loss of every decoder layer and the gradients of logits, boxes and counts of a weighted loss sum agree
  within the per-tensor parity bound (tests/parity.py: 1e-4 * max|ref| + 1e-7), with ragged event counts, a video
  with one event (its self-IoU is 0/0 in the reference too), capacity-padded targets and proposal masks.
The whole-model fixtures (test_gpu_batch.py, test_gpu_model.py) run the native form against the reference."""
import os
import sys
import types

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from parity import assert_close  # noqa: E402

DEV = "cuda"


def make_case(N=6, Q=100, Ld=2, K1=11, seed=0, capacity=None):
    g = torch.Generator().manual_seed(seed)
    targets = []
    for v in range(N):
        e = 1 + (v * 3) % 7
        c = torch.rand(e, generator=g) * 0.8 + 0.1
        targets.append({"labels": torch.zeros(e, dtype=torch.long),
                        "boxes": torch.stack([c, torch.rand(e, generator=g) * 0.3 + 0.02], -1)})
    layers = [{"pred_logits": torch.randn(N, Q, 1, generator=g) * 2,
               "pred_boxes": torch.rand(N, Q, 2, generator=g) * 0.9 + 0.05,
               "pred_count": torch.randn(N, K1, generator=g)} for _ in range(Ld)]
    return targets, layers


def run(targets, layers, fused, monkeypatch, capacity=None, query_mask=None, weigh_self_iou=False):
    from pdvc.criterion import SetCriterion, repeat_targets
    from pdvc.matcher import HungarianMatcher, padded_targets
    monkeypatch.setenv("PDVC_FUSED_CRITERION", "1" if fused else "0")
    opt = types.SimpleNamespace(lloss_gau_mask=1, lloss_beta=1)
    weight = {"loss_ce": 2, "loss_bbox": 5, "loss_giou": 2, "loss_counter": 0.5, "loss_self_iou": 0.3}
    crit = SetCriterion(1, HungarianMatcher(2, 5, 2), weight, ["labels", "boxes"], opt=opt)
    leaves = [{k: v.to(DEV).clone().requires_grad_() for k, v in lay.items()} for lay in layers]
    out = dict(leaves[0])
    out["aux_outputs"] = [dict(l) for l in leaves[1:]]
    if query_mask is not None:
        out["query_mask"] = query_mask.to(DEV)
    pt = padded_targets(targets, DEV, capacity)
    costs = crit.matcher.cost_padded(torch.cat([l["pred_logits"] for l in leaves]).detach(),
                                     torch.cat([l["pred_boxes"] for l in leaves]).detach(),
                                     repeat_targets(pt, len(leaves)))
    losses, last, aux = crit(out, targets, pt)
    wsum = sum(v * (i + 1) * 0.37 for i, (k, v) in enumerate(sorted(losses.items()))
               if "cardinality" not in k and "self_iou" not in k)
    # self-IoU is logged, never weighted by the reference (pdvc.py:583-588); it is 0/0 for one-event videos there
    # too.  Its gradient is checked where every video has two events.
    if weigh_self_iou:
        wsum = wsum + sum(v * 0.1 for k, v in losses.items() if "self_iou" in k)
    wsum.backward()
    grads = {f"{k}{i}": l[k].grad for i, l in enumerate(leaves) for k in l}
    idx = [[(i.tolist(), j.tolist()) for i, j in last[0]]] + [[(i.tolist(), j.tolist()) for i, j in a[0]] for a in aux]
    return {k: v.detach() for k, v in losses.items()}, grads, idx, costs


@pytest.mark.parametrize("capacity", [None, 12])
def test_fused_criterion_matches_torch_form(capacity, monkeypatch):
    targets, layers = make_case(seed=3)
    lt, gt, it, ct = run(targets, layers, False, monkeypatch, capacity)
    lf, gf, itf, cf = run(targets, layers, True, monkeypatch, capacity)
    assert_close(cf, ct, "matching cost", 1e-6)
    assert it == itf, "matched indices differ"
    assert set(lt) == set(lf)
    for k in lt:
        if "self_iou" in k:
            assert torch.equal(torch.isnan(lt[k]), torch.isnan(lf[k])), k
            if torch.isnan(lt[k]):
                continue
        assert_close(lf[k], lt[k], k, 1e-5)
    for k in gt:
        assert_close(gf[k], gt[k], "grad " + k, 1e-4)


def test_fused_criterion_self_iou_finite_when_every_video_has_two_events(monkeypatch):
    targets, layers = make_case(N=4, seed=5)
    for t in targets:  # at least two events each: the self-IoU term is finite and weighted
        if len(t["labels"]) < 2:
            t["labels"] = torch.zeros(2, dtype=torch.long)
            t["boxes"] = torch.tensor([[0.3, 0.2], [0.6, 0.25]])
    lt, gt, _, _ = run(targets, layers, False, monkeypatch, weigh_self_iou=True)
    lf, gf, _, _ = run(targets, layers, True, monkeypatch, weigh_self_iou=True)
    for k in lt:
        assert torch.isfinite(lf[k]).all(), k
        assert_close(lf[k], lt[k], k, 1e-5)
    for k in gt:
        assert_close(gf[k], gt[k], "grad " + k, 1e-4)


def test_fused_criterion_with_proposal_mask(monkeypatch):
    """'gt_proposals' batches: padded proposal slots never match and enter no loss (criterion.py query_mask)."""
    targets, layers = make_case(N=3, Q=30, seed=7)
    qm = torch.ones(3, 30, dtype=torch.bool)
    qm[1, 20:] = False
    qm[2, 25:] = False
    lt, gt, it, _ = run(targets, layers, False, monkeypatch, query_mask=qm)
    lf, gf, itf, _ = run(targets, layers, True, monkeypatch, query_mask=qm)
    assert it == itf
    for k in lt:
        if "self_iou" in k and torch.isnan(lt[k]):
            continue
        assert_close(lf[k], lt[k], k, 1e-5)
    for k in gt:
        assert_close(gf[k], gt[k], "grad " + k, 1e-4)
