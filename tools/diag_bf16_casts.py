"""Diagnosis: which bf16 rounding passes the bf16 mode still makes (pdvc/precision.py CAST_LOG), per source.

One eager training step of bench.py's yc2_tsp_bf16 workload at a reduced batch (the per-video shapes are the
bench's), with PDVC_CAST_LOG=1: prints every rounding pass grouped by (where it was asked for, shape), with its
count and the bytes it moves (4 read + 2 written per element), scaled to the bench's 1024 videos, plus how many
operands the producing kernels wrote themselves (attach_bf16).

    PDVC_CAST_LOG=1 python tools/diag_bf16_casts.py [--videos 128]
"""
import os
import sys

os.environ.setdefault("PDVC_CAST_LOG", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

videos = 128
if "--videos" in sys.argv:
    videos = int(sys.argv[sys.argv.index("--videos") + 1])
sys.argv = [sys.argv[0], "--workload", "yc2_tsp_bf16", "--videos-per-gpu", str(videos)]

import torch  # noqa: E402
import bench  # noqa: E402


def main():
    from pdvc import precision as P
    from pdvc.data import collate, synthetic_videos, to_device
    a = bench.parse()
    dev = torch.device("cuda:0")
    args, model, criterion = bench.build_model(a, dev)
    model.train()
    vocab = args.vocab_size + 1
    dt = to_device(collate(synthetic_videos(videos, a.T, a.C, a.events, a.words, vocab, seed=1000)), dev)
    wd = criterion.weight_dict
    # the column-sum passes (bias gradients) the step makes, by call site: in the bf16 mode gemm3w's fused bias sums
    # are off, so every bias gradient not summed by a producing kernel is a pass of its own
    from pdvc import _native as _n
    colsums = []
    real_call = _n.call

    def call(name, *a, **kw):
        if name == "pdvc_colsum_f32" and P.CAST_LOG is not None:
            f, where = sys._getframe(1), []
            while f is not None and len(where) < 3:
                fn = f.f_code.co_filename
                if "/torch/" not in fn and fn != __file__:
                    where.append(f"{os.path.basename(fn)}:{f.f_lineno} {f.f_code.co_name}")
                f = f.f_back
            colsums.append(((a[1], a[2]), " < ".join(where) or "autograd"))
        return real_call(name, *a, **kw)
    _n.call = call

    def origin3():  # the three innermost frames outside precision.py, gemm3.py and torch: who asked for the rounding
        f, where = sys._getframe(2), []
        while f is not None and len(where) < 3:
            fn = f.f_code.co_filename
            if "/torch/" not in fn and not fn.endswith(("precision.py", "gemm3.py")) and fn != __file__:
                where.append(f"{os.path.basename(fn)}:{f.f_lineno} {f.f_code.co_name}")
            f = f.f_back
        return " < ".join(where) or "autograd"
    P._origin = origin3
    for step in range(2):  # the first step warms lazy state; the second is logged
        P.CAST_LOG.clear()
        colsums.clear()
        P.STATS_CAST[:] = [0, 0, 0]
        with P.bf16_matmul():
            _, loss = model(dt, criterion, "queries")
            total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
            model.zero_grad(set_to_none=True)
            total.backward()
        torch.cuda.synchronize()
    scale = 1024 / videos
    groups = {}
    for shape, where in P.CAST_LOG:
        n = 1
        for s in shape:
            n *= s
        g = groups.setdefault((where, shape), [0, 0])
        g[0] += 1
        g[1] += n * 6
    rows = sorted(groups.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for v in groups.values())
    print(f"rounding passes: {P.STATS_CAST[0]} made, {P.STATS_CAST[1]} reused, {P.STATS_CAST[2]} written by the "
          f"producing kernels; {tot * scale / 1e9:.2f} GB moved per 1024-video step "
          f"(~{tot * scale / 8e12 * 1e3:.2f} ms at 8 TB/s)")
    print(f"{'MB@1024':>9} {'n':>3}  shape  <- where")
    for (where, shape), (cnt, b) in rows:
        print(f"{b * scale / 1e6:9.1f} {cnt:3d}  {shape}  <- {where}")
    cs = {}
    for shape, where in colsums:
        g = cs.setdefault((where, shape), [0, 0])
        g[0] += 1
        g[1] += shape[0] * shape[1] * 4
    print(f"column-sum passes: {len(colsums)}")
    for (where, shape), (cnt, b) in sorted(cs.items(), key=lambda kv: -kv[1][1]):
        print(f"{b * scale / 1e6:9.1f} {cnt:3d}  {shape}  <- {where}")


if __name__ == "__main__":
    main()

