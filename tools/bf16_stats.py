"""Which GEMMs of a training step take the bf16 path (pdvc/precision.py) and which stay on torch's fp32 GEMM
because hipBLASLt offers no bf16-compute algorithm.  python tools/bf16_stats.py [videos] [T]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path[:0] = [PKG, ROOT]

import torch  # noqa: E402
import opts  # noqa: E402
from pdvc.pdvc import build  # noqa: E402
from pdvc.data import collate, synthetic_videos, to_device  # noqa: E402
from pdvc import precision  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
T = int(sys.argv[2]) if len(sys.argv) > 2 else 256
args = opts.parse_opts(["--cfg_path", "cfgs/yc2_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG, feature_dim=768,
                       num_queries=100, frame_embedding_num=T)
model, criterion, _ = build(args)
model = model.cuda().train()
dt = to_device(collate(synthetic_videos(B, T, 768, 8, 9, args.vocab_size + 1, seed=3)), "cuda")
wd = criterion.weight_dict
with precision.bf16_matmul():
    _, loss = model(dt, criterion, "queries")
    sum(loss[k] * wd[k] for k in loss.keys() if k in wd).backward()
torch.cuda.synchronize()
tot = [0, 0]
for k, (ok, fb) in sorted(precision.STATS.items(), key=lambda kv: -kv[1][1]):
    tot[0] += ok
    tot[1] += fb
    print(f"{str(k):50s} bf16 {ok:4d}  fp32-fallback {fb:4d}")
print("total", tot)
