"""Device time of pdvc_colsum_f32 (the bias-gradient column sums) at the step's large shapes (diagnostic)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dense-video-captioning_amd")]
import torch  # noqa: E402
from pdvc.ops.functions.linear import colsum  # noqa: E402

for rows, cols in ((983040, 256), (983040, 512), (524288, 512), (262144, 512), (102400, 512)):
    x = torch.randn(rows, cols, device="cuda")
    ref = x.double().sum(0)
    for _ in range(3):
        y = colsum(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        y = colsum(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    err = (y.double() - ref).abs().max().item()
    print(f"{rows}x{cols}: {ms * 1e3:7.1f} us  {rows * cols * 4 / ms / 1e6:6.0f} GB/s  err {err:.2e}", flush=True)
    del x
