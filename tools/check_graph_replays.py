"""Correctness of the replayed step graph at the bench's scale: the headline model with every dropout off, one eager
step's losses and gradients against those of three replays of the captured step (same batch).  At 1024 videos the
graph holds torch's multi-block reductions, whose semaphores are zeroed by tiny captured memset nodes (4-32 B;
tools/diag_graph_nodes.py) -- a small captured memset was found not to re-apply on replays after eager work
(tools/memset_torch_probe.py), so the replays are checked here, not only at the fixtures' batch sizes.

    python tools/check_graph_replays.py [--videos 1024]
Prints, per replay, the largest per-tensor relative gradient difference max|g - g_eager| / max|g_eager|."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=1024)
    a = ap.parse_args()
    import opts
    from pdvc import gemm_tuning
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.pdvc import build
    from pdvc.step_graph import StepGraph
    gemm_tuning.enable()
    torch.manual_seed(0)
    # every dropout off: as keyword overrides -- the cfg chain (anet_c3d_pdvcl.yml: transformer_dropout_prob 0.1)
    # overrides command-line flags, and that probability also drives the decoder self-attention kernel's dropout
    args = opts.parse_opts(["--cfg_path", "cfgs/anet_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG,
                           feature_dim=768, num_queries=100, frame_embedding_num=512, transformer_dropout_prob=0.0,
                           hidden_dropout_prob=0.0, drop_prob=0.0)
    model, criterion, _ = build(args)
    model = model.cuda().train()
    for mod in model.modules():  # any remaining dropout off
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        elif isinstance(getattr(mod, "dropout", None), float):  # QuerySelfAttention: the MHA kernel's own dropout
            mod.dropout = 0.0
    wd = criterion.weight_dict
    dt = to_device(collate(synthetic_videos(a.videos, 512, 768, 4, 13, args.vocab_size + 1, seed=1000)), "cuda")
    out, loss = model(dt, criterion, "queries")
    total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    total.backward()
    torch.cuda.synchronize()
    ref = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    ref_total = total.item()
    ref_losses = {k: float(v) for k, v in loss.items()}
    del out, loss, total
    # a second eager step: how far two eager steps on the same batch differ (atomics in the backward, split-K GEMMs,
    # and through them near-tied set matchings of a random-init model) -- the scale the replays are judged on
    model.zero_grad(set_to_none=True)
    out, loss = model(dt, criterion, "queries")
    total2 = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    total2.backward()
    torch.cuda.synchronize()
    gmax0 = max(v.abs().max().item() for v in ref.values())
    e2 = sorted((((p.grad - ref[n]).abs().max().item() / ref[n].abs().max().item(), n)
                 for n, p in model.named_parameters() if n in ref and ref[n].abs().max().item() >= 1e-4 * gmax0),
                reverse=True)
    print(f"second eager step: total loss {total2.item():.6f}; worst relative gradient differences "
          + ", ".join(f"{e:.2e} {n}" for e, n in e2[:4]), flush=True)
    del out, loss, total2
    model.zero_grad(set_to_none=True)
    sg = StepGraph(model, criterion, dt)
    print(f"videos {a.videos}: eager total loss {ref_total:.6f}, {len(ref)} gradients", flush=True)
    gmax = max(v.abs().max().item() for v in ref.values())
    for r in range(3):
        t = sg.replay().item()
        torch.cuda.synchronize()
        errs = []
        for n, p in model.named_parameters():
            if n not in ref:
                continue
            m = ref[n].abs().max().item()
            if m < 1e-4 * gmax:  # near-zero in exact arithmetic (e.g. a softmax logit bias): no relative scale
                continue
            errs.append(((p.grad - ref[n]).abs().max().item() / m, n))
        errs.sort(reverse=True)
        dl = {k: float(v) - ref_losses[k] for k, v in sg.losses.items() if abs(float(v) - ref_losses[k]) >
              1e-4 * max(abs(ref_losses[k]), 1e-3)}
        print(f"replay {r}: total loss {t:.6f} (eager {ref_total:.6f}); worst relative gradient differences "
              + ", ".join(f"{e:.2e} {n}" for e, n in errs[:4]) + f"; losses off by > 1e-4: {dl}", flush=True)
        junk = [torch.randn(4096 + 17 * i, device="cuda").sum() for i in range(64)]  # eager work between replays
        del junk


if __name__ == "__main__":
    main()
