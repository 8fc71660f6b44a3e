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
    from pdvc.step_graph import dp_overlap_supported
    print("GraphEvent gates a stream outside the graph:", dp_overlap_supported(), flush=True)
