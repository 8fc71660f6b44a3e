"""Host-side profile of the bench training step (cProfile over K steps after warmup) -- diagnostic.
    python tools/hostprof.py [--steps 5]"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dense-video-captioning_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    graph = "--graph" in sys.argv
    argv = [x for x in sys.argv[1:] if x != "--graph"]
    sys.argv = [sys.argv[0], "--cpu-seconds", "0"] + argv
    a = bench.parse()
    from pdvc.data import synthetic_videos, collate, to_device
    device = torch.device("cuda:0")
    torch.manual_seed(0)
    args, model, criterion = bench.build_model(a, device)
    model.train()
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=args.lr, weight_decay=args.weight_decay)
    dt = to_device(collate(synthetic_videos(a.videos_per_gpu, a.T, a.C, a.events, a.words, args.vocab_size + 1,
                                            seed=1000)), device)
    wd = criterion.weight_dict

    def step():
        out, loss = model(dt, criterion, "queries")
        total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
        opt.zero_grad(set_to_none=True)
        total.backward()
        torch.nn.utils.clip_grad_norm_(params, args.grad_clip)
        opt.step()

    if graph:
        model.enable_graph(dt)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    # phase timing with syncs
    for name, fn in (("forward+loss", lambda: model(dt, criterion, "queries")),):
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        print(f"{name}: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms", flush=True)
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    print(f"step wall {(time.perf_counter() - t0) / a.steps * 1e3:.2f} ms (under cProfile)")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
    print(s.getvalue()[:12000])
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(60)
    print(s.getvalue()[:14000])


if __name__ == "__main__":
    main()
