"""Stage-by-stage check of the whole-step hipGraph at the bench shape (diagnostic):
    python tools/stepgraph_diag.py [--videos 2] [--dropout 1] [--stage replay|clip|adam]
Each stage synchronises and reports, so a failure names the stage that raised it."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path.insert(0, PKG)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=2)
    ap.add_argument("--dropout", type=int, default=1)
    ap.add_argument("--stage", default="adam")
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--opt-first", type=int, default=0)
    ap.add_argument("--tight", type=int, default=0, help="bench-like loop: no synchronisation between steps")
    a = ap.parse_args()
    import opts
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.pdvc import build
    from pdvc.step_graph import StepGraph
    torch.manual_seed(0)
    args = opts.parse_opts(["--cfg_path", "cfgs/anet_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG, feature_dim=768,
                           num_queries=100, frame_embedding_num=512)
    if not a.dropout:
        args.transformer_dropout_prob = 0.0
        args.drop_prob = 0.0
    model, criterion, _ = build(args)
    model = model.cuda().train()
    dt = to_device(collate(synthetic_videos(a.videos, 512, 768, 4, 13, args.vocab_size + 1, seed=a.seed)),
                   "cuda")
    params = [p for p in model.parameters() if p.requires_grad]
    if a.opt_first:
        opt = torch.optim.AdamW(params, lr=args.lr, weight_decay=args.weight_decay)
    sg = StepGraph(model, criterion, dt)
    if a.tight:
        for i in range(a.tight):
            sg.replay()
            torch.nn.utils.clip_grad_norm_(params, args.grad_clip)
            opt.step()
        torch.cuda.synchronize()
        print(f"tight loop ok: total {sg.total.item():.5f}", flush=True)
        return
    torch.cuda.synchronize()
    print("capture ok", flush=True)
    for i in range(2):
        t = sg.replay()
        torch.cuda.synchronize()
        bad = [n for n, p in model.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        print(f"replay {i} ok: total {t.item():.5f}, non-finite grads {bad[:3]}", flush=True)
    if a.stage == "replay":
        return
    torch.nn.utils.clip_grad_norm_(params, args.grad_clip)
    torch.cuda.synchronize()
    print("clip ok", flush=True)
    if a.stage == "clip":
        return
    if not a.opt_first:
        opt = torch.optim.AdamW(params, lr=args.lr, weight_decay=args.weight_decay)
    for i in range(3):
        sg.replay()
        torch.nn.utils.clip_grad_norm_(params, args.grad_clip)
        opt.step()
        torch.cuda.synchronize()
        print(f"step {i} ok: total {sg.total.item():.5f}", flush=True)


if __name__ == "__main__":
    main()
