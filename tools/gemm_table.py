"""Every GEMM of one eager PDVC training step at the bench shape with its achieved TF/s (diagnostic):
    python tools/gemm_table.py [--videos 256] [--no-table]
torch.profiler over 2 eager steps (the tuned GEMM table loaded as bench.py does); aten::mm / addmm / addmm_ /
bmm / baddbmm grouped by input shapes, sorted by device time."""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402

GEMMS = ("aten::mm", "aten::addmm", "aten::addmm_", "aten::bmm", "aten::baddbmm")


def flops(name, shapes):
    try:
        if name in ("aten::mm",):
            (m, k), (_, n) = shapes[0], shapes[1]
            return 2 * m * n * k
        if name in ("aten::addmm", "aten::addmm_"):
            (m, k), (_, n) = shapes[1], shapes[2]
            return 2 * m * n * k
        if name == "aten::bmm":
            (b, m, k), (_, _, n) = shapes[0], shapes[1]
            return 2 * b * m * n * k
        if name == "aten::baddbmm":
            (b, m, k), (_, _, n) = shapes[1], shapes[2]
            return 2 * b * m * n * k
    except (ValueError, IndexError, TypeError):
        return 0
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=256)
    ap.add_argument("--no-table", action="store_true")
    a = ap.parse_args()
    import opts
    from pdvc import gemm_tuning
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.pdvc import build
    if not a.no_table:
        print("tuned table:", gemm_tuning.enable())
    torch.manual_seed(0)
    args = opts.parse_opts(["--cfg_path", "cfgs/anet_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG,
                           feature_dim=768, num_queries=100, frame_embedding_num=512)
    model, criterion, _ = build(args)
    model = model.cuda().train()
    dt = to_device(collate(synthetic_videos(a.videos, 512, 768, 4, 13, args.vocab_size + 1, seed=1000)), "cuda")
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=args.lr, weight_decay=args.weight_decay, fused=True)
    wd = criterion.weight_dict

    def step():
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
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    rows = collections.defaultdict(lambda: [0.0, 0, 0])
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key in GEMMS:
            shapes = [tuple(s) for s in e.input_shapes if isinstance(s, (list, tuple))]
            k = (e.key, str(e.input_shapes)[:110])
            rows[k][0] += e.device_time_total / 2e3  # ms per step
            rows[k][1] += e.count // 2
            rows[k][2] = flops(e.key, [s for s in e.input_shapes])
    tot = sum(v[0] for v in rows.values())
    print(f"GEMM device time {tot:.2f} ms/step")
    for (name, shp), (ms, n, fl) in sorted(rows.items(), key=lambda x: -x[1][0])[:50]:
        tf = (fl * n) / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        print(f"{ms:7.3f} ms  n={n:3d}  {tf:6.1f} TF/s  {name:14s} {shp}")


if __name__ == "__main__":
    main()
