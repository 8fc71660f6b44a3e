"""Probe: can an event recorded inside a stream capture gate work outside the graph (the DP overlap's mechanism)?
torch's ROCm build refuses torch.cuda.Event(external=True) ("External events are disallowed in rocm"), so the step
graph records its own (pdvc.distributed.GraphEvent, hipEventRecordExternal); this runs the step graph's probe."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dense-video-captioning_amd")]
import torch  # noqa: E402

if __name__ == "__main__":
    print(torch.__version__, torch.version.hip, flush=True)
    try:
        torch.cuda.Event(external=True).record()
        print("torch external event: ok")
    except RuntimeError as e:
        print("torch external event:", e)
    os.environ["PDVC_DP_OVERLAP"] = "1"
    os.environ["PDVC_DP_OVERLAP_DEBUG"] = "1"
    from pdvc.step_graph import dp_overlap_supported
    print("GraphEvent gates a stream outside the graph:", dp_overlap_supported(), flush=True)
    # control: the same replay with the side stream NOT waiting -- its copy runs at once and reads the zero
    import torch as T
    from pdvc.distributed import GraphEvent
    big = T.ones(1 << 22, device="cuda")
    mark = T.zeros(1, device="cuda")
    ev = GraphEvent()
    g = T.cuda.CUDAGraph()
    with T.cuda.graph(g):
        for _ in range(64):
            big.mul_(1.0001).add_(1e-4)
        mark.copy_(big[:1] * 0.0 + 7.0)
        ev.record()
        for _ in range(64):
            big.mul_(1.0001).add_(1e-4)
        mark.fill_(3.0)
    side = T.cuda.Stream()
    for wait in (False, True, False, True):
        mark.zero_()
        g.replay()
        if wait:
            ev.wait(side)
        with T.cuda.stream(side):
            v = mark.clone()
        T.cuda.synchronize()
        print(f"side stream {'waits on' if wait else 'ignores'} the event: reads {float(v)}", flush=True)
