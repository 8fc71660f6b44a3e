"""CPU: the process-wide CUDAGraph patch of pdvc/step_graph.py rewriting_graphs is re-entrant -- a nested use keeps
the rewriting class and only the outermost exit restores torch's -- and restores it when the body raises."""
import pytest
import torch
import torch.cuda.graphs as tg

from pdvc.step_graph import _RewritingGraph, rewriting_graphs


def test_rewriting_graphs_nests_and_restores():
    orig = (torch.cuda.CUDAGraph, tg.CUDAGraph)
    with rewriting_graphs():
        assert torch.cuda.CUDAGraph is _RewritingGraph and tg.CUDAGraph is _RewritingGraph
        with rewriting_graphs():
            assert torch.cuda.CUDAGraph is _RewritingGraph
        assert torch.cuda.CUDAGraph is _RewritingGraph, "an inner exit must not restore torch's class"
    assert (torch.cuda.CUDAGraph, tg.CUDAGraph) == orig
    with pytest.raises(RuntimeError):
        with rewriting_graphs():
            raise RuntimeError("body failed")
    assert (torch.cuda.CUDAGraph, tg.CUDAGraph) == orig
