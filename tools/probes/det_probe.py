"""Run-to-run determinism of pdvc_msda1d_backward_ex_f32 outputs at the encoder-like test shape (diagnostic)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dense-video-captioning_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pdvc.ops.functions.ms_deform_attn_func import msda1d_backward, msda1d_forward  # noqa: E402

rng = np.random.RandomState(1)
T_l, Lq, M, D, N = (128, 64, 32, 16), 240, 8, 64, 2
S = sum(T_l)
c = lambda a: torch.tensor(a, dtype=torch.float32, device="cuda")
value = c(rng.randn(N, S, M, D))
proj = c(np.concatenate([rng.randn(N, Lq, M * 16) * 3.0, rng.randn(N, Lq, M * 16)], -1))
ref = c(rng.uniform(-0.05, 1.05, size=(N, Lq, 4, 1)))
gout = c(rng.randn(N, Lq, M * D))
out, sa, sl = msda1d_forward(value, None, proj, ref, T_l, 0, M * 16)
runs = [msda1d_backward(value, None, proj, ref, sa, sl, out, gout, T_l, 0, M * 16, level_sums=ls)
        for ls in (False, False, True, True)]
for i in range(1, 4):
    print(i, "gv equal", torch.equal(runs[0][0], runs[i][0]), (runs[0][0] - runs[i][0]).abs().max().item(),
          "gp equal", torch.equal(runs[0][1], runs[i][1]), (runs[0][1] - runs[i][1]).abs().max().item())
d = (runs[0][0] - runs[2][0]).abs().view(N, S, M, D).amax((2, 3))
print("rows differing:", torch.nonzero(d).tolist()[:20])
