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
            SG._DP_TRIALS.clear()
            with monkeypatch.context() as m:
                m.setattr(D.GraphEvent, "wait", lambda self, stream: None)
                assert SG.dp_overlap_supported() is False
            if SG._DP_TRIALS and all(c for c, *_ in SG._DP_TRIALS):
                # the side stream ran beside the held replay: the unheld copy read the replay's zero marker
                assert all(vc == 0.0 and v == 0.0 for _, _, vc, v in SG._DP_TRIALS), SG._DP_TRIALS
        SG._DP_OVERLAP.clear()
        SG._DP_TRIALS.clear()
        ok = SG.dp_overlap_supported()
        if SG._DP_TRIALS and not all(c for c, *_ in SG._DP_TRIALS):
            # torch handed the probe a side stream on the replay's hardware queue: it cannot run beside the replay,
            # so the probe must (and did) keep the serial reduction -- nothing to overlap with on that stream
            assert ok is False
            pytest.skip("the side stream shares the replay's hardware queue in this process")
        assert ok is True, SG._DP_TRIALS
        assert all(h and v in (7.0, 3.0) for _, h, _, v in SG._DP_TRIALS)
    finally:
        SG._DP_OVERLAP[:] = saved
