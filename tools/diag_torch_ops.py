"""Diagnosis: which torch (non-HIP-extension) element-wise / reduction ops one eager training step of bench.py's
headline workload issues, with their shapes, device time and the innermost caller in this repo.

    python tools/diag_torch_ops.py [--videos 128] [--workload anet_tsp]

One eager step at a reduced batch (per-video shapes are the bench's), after one warm-up step; device times scaled
to 1024 videos.  Grouped by (op, input shapes, caller)."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
videos, workload = 128, None
if "--videos" in sys.argv:
    videos = int(sys.argv[sys.argv.index("--videos") + 1])
if "--workload" in sys.argv:
    workload = sys.argv[sys.argv.index("--workload") + 1]
sys.argv = [sys.argv[0], "--videos-per-gpu", str(videos)] + (["--workload", workload] if workload else [])

import torch  # noqa: E402
import bench  # noqa: E402

OPS = ("aten::add", "aten::add_", "aten::copy_", "aten::sum", "aten::fill_", "aten::index_add_", "aten::mul",
       "aten::threshold_backward", "aten::zero_", "aten::clone", "aten::cat", "aten::mul_", "aten::div", "aten::sub",
       "aten::masked_fill", "aten::where", "aten::index_put_", "aten::scatter_add_", "aten::gather", "aten::max")


def main():
    from pdvc.data import collate, synthetic_videos, to_device
    a = bench.parse()
    dev = torch.device("cuda:0")
    args, model, criterion = bench.build_model(a, dev)
    model.train()
    vocab = args.vocab_size + 1
    dt = to_device(collate(synthetic_videos(videos, a.T, a.C, a.events, a.words, vocab, seed=1000)), dev)
    wd = criterion.weight_dict

    def step():
        _, loss = model(dt, criterion, "queries")
        total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
        model.zero_grad(set_to_none=True)
        total.backward()

    step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    scale = 1024 / videos
    groups = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        t = ev.self_device_time_total if hasattr(ev, "self_device_time_total") else ev.self_cuda_time_total
        if t <= 0:
            continue
        where = "autograd/engine"
        for fr in (ev.stack or []):
            if ROOT in fr and "/tools/" not in fr:
                where = fr.replace(ROOT + "/", "")
                break
        key = (ev.name, str(ev.input_shapes)[:90], where[:110])
        groups[key][0] += 1
        groups[key][1] += t
    tot = sum(v[1] for v in groups.values())
    print(f"{tot * scale / 1e3:.2f} ms per 1024-video step in these ops ({videos} videos measured)")
    for (name, shapes, where), (n, t) in sorted(groups.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{t * scale / 1e3:7.3f} ms {n:3d}  {name:24s} {shapes}  <- {where}")


if __name__ == "__main__":
    main()
