"""Which autograd node / forward op owns each small torch kernel of one eager PDVC training step (diagnostic):
    python tools/opparents.py [--videos 256] [--top 50]
torch.profiler over 1 eager step; every aten op that launched device work is attributed to its nearest
ancestor that names an autograd node ("autograd::engine::evaluate_function: XBackward") or, in the forward,
to its outermost aten / user-level parent.  Backward ops run on the autograd engine's C++ thread, so Python
stacks cannot name them; the event tree can."""
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
    ap.add_argument("--videos", type=int, default=256)
    ap.add_argument("--top", type=int, default=50)
    ap.add_argument("--bf16", action="store_true", help="the yc2_tsp_bf16 workload: cfgs/yc2_tsp_pdvc.yml, T=256, "
                    "8 events x 9 words, every GEMM on bf16 operands (pdvc/precision.py)")
    a = ap.parse_args()
    import opts
    from pdvc import gemm_tuning
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.pdvc import build
    gemm_tuning.enable()
    torch.manual_seed(0)
    cfg, T, E, W = ("cfgs/yc2_tsp_pdvc.yml", 256, 8, 9) if a.bf16 else ("cfgs/anet_tsp_pdvc.yml", 512, 4, 13)
    args = opts.parse_opts(["--cfg_path", cfg, "--device", "cuda"], cfg_root=PKG,
                           feature_dim=768, num_queries=100, frame_embedding_num=512)
    model, criterion, _ = build(args)
    model = model.cuda().train()
    dt = to_device(collate(synthetic_videos(a.videos, T, 768, E, W, args.vocab_size + 1, seed=1000)), "cuda")
    from pdvc.precision import bf16_matmul
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=args.lr, weight_decay=args.weight_decay, fused=True)
    wd = criterion.weight_dict

    def step():
        with bf16_matmul(a.bf16):
            out, loss = model(dt, criterion, "queries")
            total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
            opt.zero_grad(set_to_none=True)
            total.backward()
        torch.nn.utils.clip_grad_norm_(params, args.grad_clip)
        opt.step()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    skip = ("aten::mm", "aten::addmm", "aten::addmm_", "aten::bmm", "aten::baddbmm")
    rows = collections.defaultdict(lambda: [0.0, 0])
    for e in prof.events():
        if not e.name.startswith("aten::") or e.name in skip:
            continue
        dev = e.self_device_time_total
        if dev <= 0:
            continue
        owner, p = None, e.cpu_parent
        outer = e.name
        while p is not None:
            if p.name.startswith("autograd::engine::evaluate_function"):
                owner = p.name.split(":", 4)[-1].strip()
                break
            if not p.name.startswith("aten::"):
                owner = owner or p.name
            else:
                outer = p.name
            p = p.cpu_parent
        key = (e.name, str(e.input_shapes)[:70], owner or ("fwd " + outer))
        rows[key][0] += dev / 1e3
        rows[key][1] += 1
    tot = sum(v[0] for v in rows.values())
    print(f"non-GEMM aten device time {tot:.2f} ms/step over {sum(v[1] for v in rows.values())} ops")
    for (name, shp, owner), (ms, n) in sorted(rows.items(), key=lambda x: -x[1][0])[:a.top]:
        print(f"{ms:7.3f} ms n={n:4d} {name:22s} {shp:70s} <- {owner[:70]}")
    # launches per owner (autograd node or forward op): where the op count comes from
    by_owner = collections.defaultdict(lambda: [0.0, 0, collections.Counter()])
    for (name, shp, owner), (ms, n) in rows.items():
        r = by_owner[owner]
        r[0] += ms
        r[1] += n
        r[2][name] += n
    print("\nops per owner (count-sorted)")
    for owner, (ms, n, names) in sorted(by_owner.items(), key=lambda x: -x[1][1])[:a.top]:
        top = ", ".join(f"{k.replace('aten::', '')}x{c}" for k, c in names.most_common(6))
        print(f"n={n:4d} {ms:7.3f} ms  {owner[:60]:60s} {top}")


if __name__ == "__main__":
    main()
