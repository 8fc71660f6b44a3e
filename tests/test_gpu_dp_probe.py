"""GPU: the data-parallel overlap probe (pdvc/step_graph.py dp_overlap_supported) tells a gating event from one that
does not gate, deterministically: with the side stream's wait made a no-op, the waiting copy runs while
the probe's replay is held at its host flag, and the probe must answer False every time; with the real wait, True."""
import pytest

pytestmark = pytest.mark.gpu


def test_probe_rejects_a_wait_that_does_not_hold(monkeypatch):
    from pdvc import distributed as D
    from pdvc import step_graph as SG
    monkeypatch.delenv("PDVC_DP_OVERLAP", raising=False)
    saved = list(SG._DP_OVERLAP)
    try:
        for _ in range(3):
            SG._DP_OVERLAP.clear()
            with monkeypatch.context() as m:
                m.setattr(D.GraphEvent, "wait", lambda self, stream: None)
                assert SG.dp_overlap_supported() is False
        SG._DP_OVERLAP.clear()
        assert SG.dp_overlap_supported() is True
    finally:
        SG._DP_OVERLAP[:] = saved
