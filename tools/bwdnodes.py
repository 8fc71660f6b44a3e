"""Which autograd nodes run in the backward of one eager PDVC training step, and how many GPU kernels each
issues (diagnostic):  python tools/bwdnodes.py [--videos 16]"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=16)
    a = ap.parse_args()
    import opts
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.pdvc import build
    torch.manual_seed(0)
    args = opts.parse_opts(["--cfg_path", "cfgs/anet_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG,
                           feature_dim=768, num_queries=100, frame_embedding_num=512)
    model, criterion, _ = build(args)
    model = model.cuda().train()
    dt = to_device(collate(synthetic_videos(a.videos, 512, 768, 4, 13, args.vocab_size + 1, seed=1000)), "cuda")
    wd = criterion.weight_dict

    def fwd():
        out, loss = model(dt, criterion, "queries")
        return sum(loss[k] * wd[k] for k in loss.keys() if k in wd)

    fwd().backward()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    total = fwd()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        total.backward()
        torch.cuda.synchronize()
    nodes = collections.Counter()
    kern = collections.Counter()
    for e in prof.events():
        if e.name.startswith("autograd::engine::evaluate_function: "):
            n = e.name.split(": ", 1)[1]
            nodes[n] += 1
            kern[n] += sum(1 for k in e.kernels) if hasattr(e, "kernels") else 0
    print(f"{sum(nodes.values())} backward nodes")
    for n, c in nodes.most_common(60):
        print(f"{c:5d}  {n}")


if __name__ == "__main__":
    main()
