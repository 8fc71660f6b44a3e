"""GPU parity of the two-stage 'gt_proposals' input (cfgs/*_gt.yml; reference pdvc/pdvc.py:138-143,
misc/utils.py:31-49, deformable_transformer.py:65-78 get_proposal_pos_embed and :136-142
prepare_decoder_input_proposal, :301 disable_iterative_refine) against the reference run one video at a time
(tests/golden/make_golden.py::whole_model_batch_gt).

The ground-truth segments are the decoder's queries (their sine embedding through pos_trans / pos_trans_norm), the
boxes are the proposals, the length / class / box / GIoU losses weigh 0 and the caption cost leaves the matcher
(decide_two_stage mutates the criterion, as the reference does).  The reference runs batch 1, where every proposal
is real; the batch here pads the shorter videos' proposal lists (gt_boxes_mask): padded slots are masked as keys
of the decoder self-attention, never matched, and left out of every loss and of the count head's max.
Tolerances as tests/test_gpu_batch.py (tests/parity.py); matched indices and greedy tokens bit-exact."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import test_gpu_model as TM  # noqa: E402
import test_gpu_batch as TB  # noqa: E402
from parity import assert_scalar  # noqa: E402

DEV = "cuda"
NAME = "pdvc_batch3_anet_gt"


@pytest.fixture(scope="module")
def fixture():
    return TM.load(NAME)


def test_gt_proposals_batched_step_equals_reference(fixture):
    d = fixture
    nv = int(d["n_videos"])
    model, criterion = TM.build_filled(d)
    model.train()
    dt = TB.batch_dt(d)
    counts = [len(t["labels"]) for t in dt["video_target"]]
    assert len(set(counts)) > 1 and bool((~dt["gt_boxes_mask"]).any()), "the batch must pad proposal lists"
    cap = TB.Capture(criterion)
    out, loss = model(dt, criterion, "gt_proposals")
    # decide_two_stage's weights, as the reference left them
    assert [criterion.weight_dict[str(k)] for k in d["weight_dict_keys"]] == d["weight_dict_vals"].tolist()
    for k in [f[len("v0.loss."):] for f in d.files if f.startswith("v0.loss.")]:
        assert_scalar(loss[k], np.mean([float(d[f"v{v}.loss.{k}"]) for v in range(nv)]), f"loss {k}")
    for v in range(nv):
        e = counts[v]
        TB.close(out["pred_logits"][v:v + 1, :e], d[f"v{v}.pred_logits"], f"video {v} pred_logits")
        TB.close(out["pred_boxes"][v:v + 1, :e], d[f"v{v}.pred_boxes"], f"video {v} pred_boxes (the proposals)")
        TB.close(out["pred_count"][v:v + 1], d[f"v{v}.pred_count"], f"video {v} pred_count")
    for l_id, per_video in enumerate(cap.layer_indices()):
        for v, (i, j) in enumerate(per_video):
            assert i.tolist() == d[f"v{v}.matched.{l_id}.q"].tolist(), f"layer {l_id} video {v} matched queries"
            assert j.tolist() == d[f"v{v}.matched.{l_id}.g"].tolist(), f"layer {l_id} video {v} matched targets"
    probs = out["caption_probs"]["cap_prob_train"]
    row = 0
    for v in range(nv):
        ref = d[f"v{v}.cap_prob_train"]
        TB.close(probs[row:row + ref.shape[0], :ref.shape[1]], ref, f"video {v} cap_prob_train")
        row += ref.shape[0]
    wd = criterion.weight_dict
    total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    assert_scalar(total, np.mean([float(d[f"v{v}.total_loss"]) for v in range(nv)]), "total loss")
    total.backward()
    TB._check_grads(d, model.named_parameters(), "gt_proposals batch")


def test_gt_proposals_step_graph(fixture):
    """The same batch through StepGraph ('gt_proposals' is captured whole, trunk included)."""
    from pdvc.step_graph import StepGraph
    d = fixture
    nv = int(d["n_videos"])
    model, criterion = TM.build_filled(d)
    model.train()
    sg = StepGraph(model, criterion, TB.batch_dt(d), transformer_input_type="gt_proposals")
    for _ in range(2):
        assert_scalar(sg.replay(), np.mean([float(d[f"v{v}.total_loss"]) for v in range(nv)]), "total loss (graph)")
        TB._check_grads(d, model.named_parameters(), "gt_proposals step graph")


def test_gt_proposals_eval_matches_reference(fixture):
    """Eval forward with greedy captions of every proposal: each video's real proposals against its reference
    batch-1 eval (pred_logits, boxes, tokens bit-exact, caption log-probabilities)."""
    d = fixture
    nv = int(d["n_videos"])
    model, criterion = TM.build_filled(d)
    model.eval()
    dt = TB.batch_dt(d)
    counts = [len(t["labels"]) for t in dt["video_target"]]
    with torch.no_grad():
        out, _ = model(dt, criterion, "gt_proposals", eval_mode=True)
    for v in range(nv):
        e = counts[v]
        TB.close(out["pred_logits"][v:v + 1, :e], d[f"v{v}.eval.pred_logits"], f"video {v} eval pred_logits")
        TB.close(out["pred_boxes"][v:v + 1, :e], d[f"v{v}.eval.pred_boxes"], f"video {v} eval pred_boxes")
        ref_seq = d[f"v{v}.eval.seq"]
        steps = ref_seq.shape[-1]
        got = out["seq"][v:v + 1, :e].cpu().numpy()
        assert got[..., :steps].tolist() == ref_seq.tolist(), f"video {v} greedy tokens"
        TB.close(out["caption_probs"]["cap_prob_eval"][v:v + 1, :e, :steps], d[f"v{v}.eval.cap_prob_eval"],
                 f"video {v} cap_prob_eval")
