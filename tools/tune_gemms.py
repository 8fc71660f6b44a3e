"""Search the fastest hipBLASLt / rocBLAS solution for every GEMM shape of the bench training step and write
the table pdvc/gemm_tuning.py loads (GPU box):
    python tools/tune_gemms.py [--videos 256] [--out gpurun_out/gemm_gfx950.csv]
One eager training step at the bench shapes with TunableOp tuning on (PYTORCH_TUNABLEOP_VERBOSE prints one line
per tuned op, so a long search shows progress).  Copy the result to dense-video-captioning_amd/tuning/."""
import argparse
import os
import sys
import time

os.environ.setdefault("PYTORCH_TUNABLEOP_VERBOSE", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=256)
    ap.add_argument("--out", default="gpurun_out/gemm_gfx950.csv")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ms", type=int, default=30)
    ap.add_argument("--seed-table", default=None, help="start from an existing table (shapes in it are kept)")
    a = ap.parse_args()
    import opts
    import torch.cuda.tunable as tun
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.pdvc import build
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    if a.seed_table and os.path.exists(a.seed_table):
        import shutil
        shutil.copyfile(a.seed_table, a.out)
    tun.set_filename(a.out)
    tun.set_max_tuning_iterations(a.iters)
    tun.set_max_tuning_duration(a.ms)
    torch.manual_seed(0)
    args = opts.parse_opts(["--cfg_path", "cfgs/anet_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG,
                           feature_dim=768, num_queries=100, frame_embedding_num=512)
    model, criterion, _ = build(args)
    model = model.cuda().train()
    dt = to_device(collate(synthetic_videos(a.videos, 512, 768, 4, 13, args.vocab_size + 1, seed=1000)), "cuda")
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=args.lr, weight_decay=args.weight_decay, fused=True)
    wd = criterion.weight_dict
    tun.enable(True)
    tun.tuning_enable(True)
    t0 = time.time()
    out, loss = model(dt, criterion, "queries")
    total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    opt.zero_grad(set_to_none=True)
    total.backward()
    torch.nn.utils.clip_grad_norm_(params, args.grad_clip)
    opt.step()
    torch.cuda.synchronize()
    tun.tuning_enable(False)
    n = len(tun.get_results())
    print(f"tuned {n} GEMM shapes in {time.time() - t0:.0f} s -> {a.out}", flush=True)
    # TunableOp writes the table at exit


if __name__ == "__main__":
    main()
