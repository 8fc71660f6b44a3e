"""GPU: no garbage collection runs inside the StepGraph capture, whatever garbage is pending.

Round 4's pass AC aborted inside a step-graph capture; StepGraph now disables the collector for the capture
(pdvc/step_graph.py).  This test makes the worst case for that guard: the collector's threshold at 1 (a collection
on almost every container allocation), pending cyclic garbage holding CUDA tensors, an eager autograd graph whose
backward never ran, and an instantiated CUDAGraph, and a gc.callbacks hook recording every collection that starts
while the current stream is capturing.  The StepGraph must capture with no such collection, and its replay must
equal the eager step within tests/parity.py's bound.  tools/gc_capture_probe.py shows, case by case, what a
collection inside a capture does to it.
"""
import gc
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
from test_gpu_step_graph_scale import _eager, _model  # noqa: E402


class _Cycle:
    def __init__(self, payload):
        self.payload = payload
        self.me = self


def _pending_garbage(model, criterion, dt):
    """Cyclic garbage only the collector can free: CUDA tensors, a live eager autograd graph of the model itself
    (its AccumulateGrad nodes and saved activations), and an instantiated graph with its pool's output."""
    _Cycle([torch.randn(1 << 18, device="cuda") for _ in range(4)])
    _, loss = model(dt, criterion, "queries")
    _Cycle(loss)  # backward never runs: the graph stays alive inside the cycle
    a = torch.randn(4096, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        a * 2
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b = a * 2 + 1
    g.replay()
    _Cycle((g, b))


@pytest.mark.gpu
def test_no_collection_inside_step_graph_capture():
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.step_graph import StepGraph
    args, model, criterion = _model()
    dt = to_device(collate(synthetic_videos(8, 512, 768, 4, 13, args.vocab_size + 1, seed=77)), "cuda")
    total, losses, grads = _eager(model, criterion, dt)
    model.zero_grad(set_to_none=True)

    inside = []

    def hook(phase, info):
        if phase == "start" and torch.cuda.is_current_stream_capturing():
            inside.append(info.get("generation"))

    thresholds = gc.get_threshold()
    gc.callbacks.append(hook)
    try:
        gc.collect()
        _pending_garbage(model, criterion, dt)
        gc.set_threshold(1)  # a young-generation collection on every container allocation
        sg = StepGraph(model, criterion, dt, warmup=1)
        assert gc.isenabled(), "StepGraph must re-enable the collector after the capture"
    finally:
        gc.set_threshold(*thresholds)
        gc.callbacks.remove(hook)
    assert inside == [], f"{len(inside)} garbage collection(s) started inside the capture (generations {inside})"
    for r in range(2):
        t = sg.replay()
        torch.cuda.synchronize()
        assert_scalar(t, total, f"replay {r}: total loss")
        for k, v in sg.losses.items():
            assert_scalar(v, losses[k], f"replay {r}: {k}")
        for n, p in model.named_parameters():
            if n in grads:
                assert_close(p.grad, grads[n], f"replay {r}: grad {n}")
