"""GPU parity of the BATCHED training step -- the path bench.py times at 1024 videos per GPU -- against the
reference run one video at a time (tests/golden/make_golden.py::whole_model_batch).

The reference cannot batch (pdvc/CaptioningHead/LSTM_DSA.py:59,121 assert one video) and normalises every
loss by that video's event count (pdvc/criterion.py:167-171).  The MI355X path's batch semantics: every loss
key is the mean over videos of the reference's batch-1 value, so the gradient of one N-video step is the mean
of the N batch-1 gradients.  The fixture has 3 videos with 2, 3 and 5 events, ragged caption lengths,
different durations and one padded (masked) video; it holds each video's losses, matched indices of every
decoder layer, heads, captioning log-probabilities, eval outputs and PostProcess results, and the mean
gradient of every parameter as a full tensor.  Tolerance (tests/parity.py): max|got - ref| <= 1e-4 * max|ref|
+ 1e-7 per tensor (fp32), plus the fixture's stored SVD packing error for packed gradients; matched indices,
ranked query ids, labels, counts and greedy tokens bit-exact."""
import os
import sys
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import test_gpu_model as TM  # noqa: E402
from parity import assert_close, assert_scalar, bound  # noqa: E402

DEV = "cuda"
TOL = 1e-4
NAME = "pdvc_batch3_anet"


def close(got, ref, what, tol=TOL, extra=0.0):
    assert_close(got, ref, what, tol, extra=extra)


def batch_dt(d):
    """The 3 fixture videos as ONE batch through our collate (the reference collate_fn's padding)."""
    import weights as W
    from pdvc.data import collate, to_device
    return to_device(collate(W.batch_items(vocab=29)), DEV)


class Capture:
    """Wraps a criterion's forward to keep its (losses, last_indices, aux_indices) return value."""

    def __init__(self, criterion):
        self.result = None
        orig = criterion.forward

        def fwd(*a, **k):
            self.result = orig(*a, **k)
            return self.result
        criterion.forward = fwd

    def layer_indices(self):
        _, last, aux = self.result
        return [list(aux[l][0]) for l in range(len(aux))] + [list(last[0])]


@pytest.fixture(scope="module")
def fixture():
    return TM.load(NAME)


def _check_forward(d, out, loss, cap, nv):
    wd_keys = [f[len("v0.loss."):] for f in d.files if f.startswith("v0.loss.")]
    for k in wd_keys:
        ref = np.mean([float(d[f"v{v}.loss.{k}"]) for v in range(nv)])
        got = loss[k].item() if isinstance(loss[k], torch.Tensor) else float(loss[k])
        assert_scalar(got, ref, f"loss {k} vs the mean of the batch-1 values")
    for v in range(nv):
        close(out["pred_logits"][v:v + 1], d[f"v{v}.pred_logits"], f"video {v} pred_logits")
        close(out["pred_boxes"][v:v + 1], d[f"v{v}.pred_boxes"], f"video {v} pred_boxes")
        close(out["pred_count"][v:v + 1], d[f"v{v}.pred_count"], f"video {v} pred_count")
    for l_id, per_video in enumerate(cap.layer_indices()):
        for v, (i, j) in enumerate(per_video):
            assert i.tolist() == d[f"v{v}.matched.{l_id}.q"].tolist(), f"layer {l_id} video {v} matched queries"
            assert j.tolist() == d[f"v{v}.matched.{l_id}.g"].tolist(), f"layer {l_id} video {v} matched targets"
    # captioning log-probabilities of the last layer: rows grouped by video, each video's own step count
    probs = out["caption_probs"]["cap_prob_train"]
    row = 0
    for v in range(nv):
        ref = d[f"v{v}.cap_prob_train"]
        e, steps = ref.shape[0], ref.shape[1]
        close(probs[row:row + e, :steps], ref, f"video {v} cap_prob_train")
        row += e
    assert row == probs.shape[0]


def _check_grads(d, named_params, what):
    n_checked = 0
    for n, p in named_params:
        if "gradnone." + n in d.files:
            assert p.grad is None, f"{what}: {n} must receive no gradient (as in the reference)"
            continue
        assert p.grad is not None, f"{what}: {n} has no gradient"
        close(p.grad, TM.full_grad(d, n), f"{what}: grad {n}", extra=TM.grad_err(d, n))
        n_checked += 1
    assert n_checked > 100


# the smallest reference gradients of the batch fixture sit in the caption head (LSTM_DSA.py:218-220, 245-258)
MUTANTS = ("caption_head.0.core.h2att.weight", "caption_head.0.core.h2att.bias", "caption_head.0.core.ctx2att.bias",
           "caption_head.0.core.alpha_net.weight")


def _check_mutants(d, named_params):
    """The bound must reject a zeroed or sign-flipped gradient of every checked tensor, the smallest included:
    a bound that lets those through does not constrain the tensor."""
    params = dict(named_params)
    for n, p in params.items():
        if p.grad is None:
            continue
        ref = TM.full_grad(d, n)
        peak = float(np.abs(ref).max())
        if peak > 1e-6:
            assert bound(ref, extra=TM.grad_err(d, n)) < 0.5 * peak, f"{n}: the bound does not constrain the tensor"
    for n in MUTANTS:
        g = params[n].grad
        ref = TM.full_grad(d, n)
        for bad in (torch.zeros_like(g), -g, g * 1.01):
            with pytest.raises(AssertionError):
                close(bad, ref, f"mutant {n}", extra=TM.grad_err(d, n))


def test_batched_step_equals_mean_of_reference_batch1_steps(fixture):
    d = fixture
    nv = int(d["n_videos"])
    model, criterion = TM.build_filled(d)
    model.train()
    dt = batch_dt(d)
    assert dt["video_tensor"].shape[0] == nv and not bool(dt["video_mask"].all()), "fixture must pad one video"
    cap = Capture(criterion)
    out, loss = model(dt, criterion, "queries")
    _check_forward(d, out, loss, cap, nv)
    wd = criterion.weight_dict
    total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    ref_total = np.mean([float(d[f"v{v}.total_loss"]) for v in range(nv)])
    assert_scalar(total, ref_total, "total loss")
    total.backward()
    _check_grads(d, model.named_parameters(), "eager batch")
    _check_mutants(d, model.named_parameters())


def test_batched_step_graph_equals_reference(fixture):
    """The same batch through StepGraph (forward + losses + backward as one hipGraph replay, the bench path)."""
    from pdvc.step_graph import StepGraph
    d = fixture
    nv = int(d["n_videos"])
    model, criterion = TM.build_filled(d)
    model.train()
    dt = batch_dt(d)
    sg = StepGraph(model, criterion, dt)
    for _ in range(2):
        total = sg.replay().item()
        ref_total = np.mean([float(d[f"v{v}.total_loss"]) for v in range(nv)])
        assert_scalar(total, ref_total, "total loss (graph replay)")
        _check_grads(d, model.named_parameters(), "step graph")


@pytest.mark.parametrize("on_gemm3", [False, True])
def test_batched_eval_and_postprocess_match_reference(fixture, on_gemm3, monkeypatch):
    """Eval forward (greedy captions) of the 3-video batch and our PostProcess on it against each video's
    reference eval forward and reference PostProcess (pdvc/pdvc.py:493-546).  on_gemm3: every eligible product on
    the in-tree fp32 GEMM at these small row counts (MIN_ROWS = 0) -- the greedy step's word, h and attention-gate
    products among them, as at the bench's row counts."""
    from data.video_dataset import Translator
    if on_gemm3:
        import pdvc.ops.functions.gemm3 as G
        monkeypatch.setattr(G, "MIN_ROWS", 0)
        monkeypatch.setattr(G, "ENABLED", True)
    d = fixture
    nv = int(d["n_videos"])
    model, criterion = TM.build_filled(d)
    model.eval()
    dt = batch_dt(d)
    with torch.no_grad():
        out, _ = model(dt, criterion, "queries", eval_mode=True)
    tr = Translator.from_vocab({str(i): f"w{i}" for i in range(1, 30)})
    loader = types.SimpleNamespace(dataset=types.SimpleNamespace(translator=tr))
    post = TM.build_post(d)
    res = post(out, dt["video_length"][:, 1], loader)
    assert len(res) == nv
    for v in range(nv):
        close(out["pred_logits"][v:v + 1], d[f"v{v}.eval.pred_logits"], f"video {v} eval pred_logits")
        close(out["pred_boxes"][v:v + 1], d[f"v{v}.eval.pred_boxes"], f"video {v} eval pred_boxes")
        ref_seq = d[f"v{v}.eval.seq"]
        steps = ref_seq.shape[-1]
        got_seq = out["seq"][v:v + 1].cpu().numpy()
        assert got_seq[..., :steps].tolist() == ref_seq.tolist(), f"video {v} greedy tokens"
        assert not got_seq[..., steps:].any(), f"video {v}: tokens after the video's last step"
        close(out["caption_probs"]["cap_prob_eval"][v:v + 1, :, :steps], d[f"v{v}.eval.cap_prob_eval"],
              f"video {v} cap_prob_eval")
        r = res[v]
        close(r["scores"], d[f"v{v}.post.scores"], f"video {v} scores")
        assert r["query_id"].tolist() == d[f"v{v}.post.query_id"].tolist(), f"video {v} ranked query ids"
        assert r["labels"].tolist() == d[f"v{v}.post.labels"].tolist()
        close(r["boxes"], d[f"v{v}.post.boxes"], f"video {v} boxes")
        close(r["raw_boxes"], d[f"v{v}.post.boxes"], f"video {v} raw_boxes (the reference returns boxes)")
        close(r["vid_duration"], d[f"v{v}.post.vid_duration"], f"video {v} duration")
        assert int(r["pred_seq_len"]) == int(d[f"v{v}.post.pred_seq_len"])
        close(np.asarray(r["caption_scores"]), d[f"v{v}.post.caption_scores"], f"video {v} caption scores")
        assert list(r["captions"]) == [str(s) for s in d[f"v{v}.post.captions"]], f"video {v} captions"


# ------------------------------------------------------------------------------------------------
# capacity-padded batches (pdvc/batch_layout.py): one captured step for a stream of ragged batches
# ------------------------------------------------------------------------------------------------
CAPS = dict(events=7, rows=16, words=12)


def padded_dt(items, packed=False):
    """packed: a token capacity 8 above the batch's caption-token count, so the logit projection runs over the
    packed valid tokens (pdvc/caption_tokens.py), and live-row capacities per step, so the recurrence runs each step
    over the rows still in their video's loop; else every (row, step) position."""
    import weights as W  # noqa: F401
    from pdvc.batch_layout import pad_to_capacity
    from pdvc.data import collate, to_device
    c = collate(items)
    tokens = alive = None
    if packed:  # and the recurrence over the live rows of each step (with 2 rows of slack)
        from pdvc.batch_layout import live_rows
        from pdvc.pdvc import video_steps
        tokens = int(c["cap_mask"][:, 1:CAPS["words"]].sum()) + 8
        counts = [len(t["labels"]) for t in c["video_target"]]
        alive = [min(a + 2, CAPS["rows"]) for a in live_rows(counts, video_steps(c["cap_tensor"], counts),
                                                             CAPS["words"] - 1)]
    return to_device(pad_to_capacity(c, tokens=tokens, alive=alive, **CAPS), DEV)


def _check_padded_forward(d, out, loss, nv, cap):
    wd_keys = [f[len("v0.loss."):] for f in d.files if f.startswith("v0.loss.")]
    for k in wd_keys:
        ref = np.mean([float(d[f"v{v}.loss.{k}"]) for v in range(nv)])
        assert_scalar(loss[k], ref, f"loss {k} (capacity-padded) vs the mean of the batch-1 values")
    for v in range(nv):
        close(out["pred_logits"][v:v + 1], d[f"v{v}.pred_logits"], f"video {v} pred_logits")
        close(out["pred_boxes"][v:v + 1], d[f"v{v}.pred_boxes"], f"video {v} pred_boxes")
    probs = out["caption_probs"]["cap_prob_train"]
    assert probs.shape[0] == cap["rows"] and probs.shape[1] == cap["words"] - 1
    row = 0
    for v in range(nv):
        ref = d[f"v{v}.cap_prob_train"]
        e, steps = ref.shape[0], ref.shape[1]
        close(probs[row:row + e, :steps], ref, f"video {v} cap_prob_train (capacity-padded)")
        row += e


@pytest.mark.parametrize("packed", [False, True], ids=["all_positions", "packed_tokens"])
def test_capacity_padded_batch_equals_reference(fixture, packed):
    """The fixture's 3 videos padded to fixed capacities (7 events per video, 16 caption rows per layer, 12-token
    captions): phantom targets and caption rows change no loss and no gradient -- the same bound against the
    reference's batch-1 steps as the unpadded batch.  packed: the logits over the packed caption tokens only."""
    d = fixture
    nv = int(d["n_videos"])
    model, criterion = TM.build_filled(d)
    model.train()
    import weights as W
    dt = padded_dt(W.batch_items(vocab=29), packed)
    out, loss = model(dt, criterion, "queries")
    _check_padded_forward(d, out, loss, nv, dt["capacity"])
    wd = criterion.weight_dict
    total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    assert_scalar(total, np.mean([float(d[f"v{v}.total_loss"]) for v in range(nv)]), "total loss (capacity-padded)")
    total.backward()
    _check_grads(d, model.named_parameters(), "capacity-padded batch")


@pytest.mark.parametrize("packed", [False, True], ids=["all_positions", "packed_tokens"])
def test_capacity_step_graph_follows_a_ragged_stream(fixture, packed):
    """ONE StepGraph captured on a capacity-padded batch serves batches of other event counts and caption lengths:
    load() a batch of the same videos in another order (per-position counts 5, 2, 3 instead of 2, 3, 5) and the
    replay equals the eager unpadded step on it; load the first batch back and the replay equals the reference."""
    from pdvc.data import collate, to_device
    from pdvc.step_graph import StepGraph
    import weights as W
    d = fixture
    nv = int(d["n_videos"])
    model, criterion = TM.build_filled(d)
    model.train()
    items = W.batch_items(vocab=29)
    perm = [items[2], items[0], items[1]]
    # eager reference on the permuted batch, unpadded
    wd = criterion.weight_dict
    model.zero_grad(set_to_none=True)
    out_b, loss_b = model(to_device(collate(perm), DEV), criterion, "queries")
    total_b = sum(loss_b[k] * wd[k] for k in loss_b.keys() if k in wd)
    total_b.backward()
    grads_b = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    total_b = total_b.item()
    del out_b, loss_b  # the eager step's autograd graph (its default-stream AccumulateGrad nodes) must not outlive it
    model.zero_grad(set_to_none=True)
    sg = StepGraph(model, criterion, padded_dt(items, packed))
    assert_scalar(sg.replay(), np.mean([float(d[f"v{v}.total_loss"]) for v in range(nv)]), "replay, batch A")
    _check_grads(d, model.named_parameters(), "capacity step graph, batch A")
    sg.load(padded_dt(perm, packed))
    assert_scalar(sg.replay(), total_b, "replay after load(batch B)")
    for n, p in model.named_parameters():
        if n in grads_b:
            close(p.grad, grads_b[n], f"capacity step graph, batch B: grad {n}")
    sg.load(padded_dt(items, packed))
    sg.replay()
    _check_grads(d, model.named_parameters(), "capacity step graph, batch A again")
