"""The GEMMs of one eager training step that stay on torch (hipBLASLt / rocBLAS): everything the in-tree gemm3 path
takes goes through the C ABI and is invisible to aten, so aten's GEMM calls are exactly the library ones.
    python tools/torch_gemms.py [--videos 1024]
Prints per (op, shapes, strides) group: calls, GFLOP, and the device time the profiler attributes to it."""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path[:0] = [ROOT, PKG, os.path.join(ROOT, "tools")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=1024)
    a = ap.parse_args()
    import opts
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.pdvc import build
    from torch.utils._python_dispatch import TorchDispatchMode
    torch.manual_seed(0)
    args = opts.parse_opts(["--cfg_path", "cfgs/anet_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG,
                           feature_dim=768, num_queries=100, frame_embedding_num=512)
    model, criterion, _ = build(args)
    model = model.cuda().train()
    dt = to_device(collate(synthetic_videos(a.videos, 512, 768, 4, 13, args.vocab_size + 1, seed=1000)), "cuda")
    wd = criterion.weight_dict

    def step():
        out, loss = model(dt, criterion, "queries")
        total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
        model.zero_grad(set_to_none=True)
        total.backward()

    step()
    torch.cuda.synchronize()
    aten = torch.ops.aten
    packets = {aten.mm, aten.addmm, aten.addmm_, aten._addmm_activation, aten.bmm, aten.baddbmm}
    seen = collections.defaultdict(lambda: [0, 0.0, 0.0])

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            if func.overloadpacket in packets:
                ts = [t for t in args if isinstance(t, torch.Tensor)]
                x, y = ts[-2], ts[-1]
                b = x.shape[0] if x.dim() == 3 else 1
                key = (str(func.overloadpacket).split(".")[-1], tuple(x.shape), x.stride(), tuple(y.shape), y.stride())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r = func(*args, **(kwargs or {}))
                e1.record()
                seen[key][0] += 1
                seen[key][1] += 2 * b * x.shape[-2] * x.shape[-1] * y.shape[-1]
                seen[key].append((e0, e1))
                return r
            return func(*args, **(kwargs or {}))

    with Mode():
        step()
    torch.cuda.synchronize()
    rows = []
    for k, v in seen.items():
        ms = sum(e0.elapsed_time(e1) for e0, e1 in v[3:])
        rows.append((ms, v[0], v[1], k))
    rows.sort(key=lambda r: -r[0])
    print(f"torch GEMMs: {sum(r[1] for r in rows)} calls, {sum(r[2] for r in rows) / 1e9:.1f} GFLOP, "
          f"{sum(r[0] for r in rows):.2f} ms")
    for ms, n, fl, k in rows[:40]:
        print(f"{ms:8.3f} ms {n:4d} x {fl / 1e9:8.2f} GF {fl / max(ms, 1e-9) / 1e9:7.1f} TF/s  {k}")


if __name__ == "__main__":
    main()
