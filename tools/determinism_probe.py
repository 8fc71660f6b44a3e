"""Where is the headline step non-deterministic?  Two eager steps of the headline model on the same batch and weights,
every dropout off: forward hooks on every module keep each module output of step 1 and compare step 2's bitwise, in
call order; then the parameter gradients of the two steps.  Prints the first modules whose outputs differ and the
gradients that differ (bitwise, and the largest relative difference).

    python tools/determinism_probe.py [--videos 256] [--no-table] [--backward]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402


def flat(x, out):
    if isinstance(x, torch.Tensor):
        if x.is_floating_point() or x.dtype in (torch.int64, torch.int32, torch.bool):
            out.append(x)
    elif isinstance(x, dict):
        for v in x.values():
            flat(v, out)
    elif isinstance(x, (list, tuple)):
        for v in x:
            flat(v, out)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=256)
    ap.add_argument("--no-table", action="store_true")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import opts
    from pdvc import gemm_tuning
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.pdvc import build
    if not a.no_table:
        gemm_tuning.enable()
    torch.manual_seed(0)
    # every dropout off: as keyword overrides -- the cfg chain (anet_c3d_pdvcl.yml: transformer_dropout_prob 0.1)
    # overrides command-line flags, and that probability also drives the decoder self-attention kernel's dropout
    args = opts.parse_opts(["--cfg_path", "cfgs/anet_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG,
                           feature_dim=768, num_queries=100, frame_embedding_num=512, transformer_dropout_prob=0.0,
                           hidden_dropout_prob=0.0, drop_prob=0.0)
    model, criterion, _ = build(args)
    model = model.cuda().train()
    for mod in model.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        elif isinstance(getattr(mod, "dropout", None), float):  # QuerySelfAttention: the MHA kernel's own dropout
            mod.dropout = 0.0
    wd = criterion.weight_dict
    dt = to_device(collate(synthetic_videos(a.videos, 512, 768, 4, 13, args.vocab_size + 1, seed=1000)), "cuda")
    names = {m: n for n, m in list(model.named_modules()) + [("criterion." + n, m) for n, m in criterion.named_modules()]}
    rec = []  # (name, [tensors]) in call order, this step

    def hook(mod, inp, out):
        rec.append((names.get(mod, type(mod).__name__), [t.detach().clone() for t in flat(out, [])]))

    hs = [m.register_forward_hook(hook) for m in names]
    runs = []
    for s in range(a.steps):
        rec.clear()
        model.zero_grad(set_to_none=True)
        out, loss = model(dt, criterion, "queries")
        total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
        total.backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
        losses = {k: float(v) for k, v in loss.items()}
        runs.append((list(rec), grads, losses, float(total)))
        print(f"step {s}: total {float(total):.9f}", flush=True)
        del out, loss, total
    for h in hs:
        h.remove()
    r0 = runs[0]
    for s in range(1, a.steps):
        r = runs[s]
        print(f"--- step {s} vs step 0", flush=True)
        nd = 0
        if len(r[0]) != len(r0[0]):
            print(f"module call counts differ: {len(r[0])} vs {len(r0[0])}")
        for (n0, t0), (n1, t1) in zip(r0[0], r[0]):
            diffs = []
            for x, y in zip(t0, t1):
                if x.shape != y.shape:
                    diffs.append(f"shape {tuple(x.shape)} vs {tuple(y.shape)}")
                elif not torch.equal(x, y):
                    if x.is_floating_point():
                        m = x.abs().max().item()
                        diffs.append(f"max|d| {(x - y).abs().max().item():.3e} of max {m:.3e}")
                    else:
                        diffs.append(f"{int((x != y).sum())} entries")
            if diffs:
                nd += 1
                if nd <= 12:
                    print(f"  module {n0}: {'; '.join(diffs[:3])}", flush=True)
        print(f"  {nd} of {len(r0[0])} module calls differ", flush=True)
        gd = []
        for n, g in r0[1].items():
            g1 = r[1].get(n)
            if g1 is None or not torch.equal(g, g1):
                m = g.abs().max().item()
                gd.append(((g - g1).abs().max().item() / max(m, 1e-30) if g1 is not None else float("inf"), n))
        gd.sort(reverse=True)
        print(f"  {len(gd)} of {len(r0[1])} gradients differ bitwise; worst: " +
              ", ".join(f"{e:.2e} {n}" for e, n in gd[:6]), flush=True)
        ld = {k: r[2][k] - r0[2][k] for k in r0[2] if r[2][k] != r0[2][k]}
        print(f"  losses that differ: {ld}", flush=True)


if __name__ == "__main__":
    main()
