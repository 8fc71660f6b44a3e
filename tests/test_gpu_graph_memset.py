"""Captured memset nodes and their rewrite as kernel nodes (csrc/graphfix.hip, pdvc/step_graph.py replace_memsets).

On this ROCm stack a small hipMemsetAsync captured by torch.cuda.graph did not re-apply on replays after the first
when eager work ran between replays (tools/memset_torch_probe.py: a 160-B zero-fill left 3073 where 1 was due); torch's
multi-block reductions zero their semaphores with such 4-32 B memsets, and the 1024-video training step graph's
replays produced garbage gradients through them (tools/check_graph_replays.py).  StepGraph rewrites every memset node
as a kernel node before instantiation; these tests check the rewrite on the two shapes of the problem."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _node_types(graph):
    hip = ctypes.CDLL("libamdhip64.so")
    raw = ctypes.c_void_p(graph.raw_cuda_graph())
    k = ctypes.c_size_t(0)
    hip.hipGraphGetNodes(raw, None, ctypes.byref(k))
    nodes = (ctypes.c_void_p * k.value)()
    hip.hipGraphGetNodes(raw, nodes, ctypes.byref(k))
    out = []
    for nd in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        out.append(t.value)
    return out


@pytest.mark.parametrize("n", [1, 8, 40, 400])
def test_small_captured_memset_reapplies_after_rewrite(n):
    from pdvc.step_graph import replace_memsets
    hip = ctypes.CDLL("libamdhip64.so")
    buf = torch.empty(n, device=DEV)
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=side):
        buf.fill_(5.0)
        s = torch.cuda.current_stream().cuda_stream
        assert hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, ctypes.c_size_t(n * 4), ctypes.c_void_p(s)) == 0
        buf.add_(1.0)
    assert 2 in _node_types(g)  # the memset was captured as a memset node
    assert replace_memsets(g) == 1
    assert 2 not in _node_types(g)
    g.instantiate()
    for _ in range(4):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(buf, torch.ones_like(buf)), buf[:4].tolist()
        junk = [torch.full((n + 13 * i,), 7.0, device=DEV) * 2 for i in range(32)]  # eager work between replays
        del junk


def test_multiblock_reduction_in_graph_follows_new_inputs():
    """A column sum torch runs as a multi-block reduction (semaphores zeroed by captured memsets), replayed on new
    inputs with eager work between replays, equals the eager sum every time."""
    from pdvc.step_graph import replace_memsets
    x = torch.randn(1 << 21, 3, device=DEV)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        out = x.sum(0)  # warm-up
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=side):
        out = x.sum(0)
    replace_memsets(g)
    assert 2 not in _node_types(g)
    g.instantiate()
    for r in range(4):
        x.copy_(torch.randn_like(x) * (r + 1))
        g.replay()
        torch.cuda.synchronize()
        ref = x.double().sum(0)
        assert (out.double() - ref).abs().max().item() <= 1e-3 * ref.abs().max().item() + 1e-2, (r, out, ref)
        junk = [torch.randn(4096 + 17 * i, device=DEV).sum() for i in range(64)]
        del junk
