"""GPU: the captured training step at the bench's scale against the eager step it replaces.

The headline model (cfgs/anet_tsp_pdvc.yml, T=512, C=768, Q=100, 2+2 layers) on 256 synthetic videos -- enough for
torch's multi-block reductions, whose semaphores are zeroed by tiny captured memset nodes (csrc/graphfix.hip
rewrites them) -- with every dropout off, including the decoder self-attention kernel's own
(its probability comes from the cfg chain, so it is overridden by keyword, not by a command-line flag).  Then:

  * two eager steps on the same batch and weights agree (the step is reproducible at this scale), and
  * three replays of the StepGraph captured on that batch, with unrelated eager work between them, give every loss
    and every parameter gradient of the eager step within tests/parity.py's bound (1e-4 of each tensor's max|ref|).
"""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
for p in (ROOT, PKG, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

from parity import assert_close, assert_scalar  # noqa: E402

VIDEOS = 256


def _model():
    import opts
    from pdvc import gemm_tuning
    from pdvc.pdvc import build
    gemm_tuning.enable()
    torch.manual_seed(0)
    args = opts.parse_opts(["--cfg_path", "cfgs/anet_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG,
                           feature_dim=768, num_queries=100, frame_embedding_num=512, transformer_dropout_prob=0.0,
                           hidden_dropout_prob=0.0, drop_prob=0.0)
    model, criterion, _ = build(args)
    model = model.cuda().train()
    for mod in model.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0  # (the captioner's att_drop: built by the reference with p = 0.5, never applied)
        elif isinstance(getattr(mod, "dropout", None), float):
            assert mod.dropout == 0.0, "the self-attention kernel's dropout survived the overrides"
    return args, model, criterion


def _eager(model, criterion, dt):
    wd = criterion.weight_dict
    model.zero_grad(set_to_none=True)
    _, loss = model(dt, criterion, "queries")
    total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    total.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    return float(total), {k: float(v) for k, v in loss.items()}, grads


@pytest.mark.gpu
def test_step_graph_replays_equal_eager_step_at_scale():
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.step_graph import StepGraph
    args, model, criterion = _model()
    dt = to_device(collate(synthetic_videos(VIDEOS, 512, 768, 4, 13, args.vocab_size + 1, seed=1000)), "cuda")
    total, losses, grads = _eager(model, criterion, dt)
    assert len(grads) > 120
    total2, losses2, grads2 = _eager(model, criterion, dt)
    assert_scalar(total2, total, "second eager step: total loss")
    for n, g in grads.items():
        assert_close(grads2[n], g, f"second eager step: grad {n}")
    model.zero_grad(set_to_none=True)
    sg = StepGraph(model, criterion, dt)
    assert sg.memsets_replaced >= 0 and sg.node_counts.get("memset", 0) == 0
    for r in range(3):
        t = sg.replay()
        torch.cuda.synchronize()
        assert_scalar(t, total, f"replay {r}: total loss")
        for k, v in sg.losses.items():
            assert_scalar(v, losses[k], f"replay {r}: {k}")
        for n, p in model.named_parameters():
            if n in grads:
                assert_close(p.grad, grads[n], f"replay {r}: grad {n}")
            else:
                assert p.grad is None, f"replay {r}: {n} must receive no gradient"
        junk = [torch.randn(4096 + 17 * i, device="cuda").sum() for i in range(64)]  # eager work between replays
        del junk
