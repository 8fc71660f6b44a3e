"""Which source lines issue the aten ops (~ GPU kernels) of one eager PDVC training step (diagnostic):
    python tools/opcount.py [--videos 16] [--top 60]
A TorchDispatchMode records every aten op with the innermost pdvc/ frame that called it; prints the lines
issuing the most ops.  Custom HIP launches (ctypes) are not aten ops and do not appear."""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

SKIP_OPS = {"aten::detach", "aten::view", "aten::_unsafe_view", "aten::t", "aten::transpose", "aten::reshape",
            "aten::expand", "aten::as_strided", "aten::permute", "aten::select", "aten::slice", "aten::unsqueeze",
            "aten::squeeze", "aten::alias", "aten::split", "aten::chunk", "aten::unbind", "aten::narrow",
            "aten::empty", "aten::empty_like", "aten::empty_strided", "aten::new_empty", "aten::new_empty_strided",
            "aten::lift_fresh", "aten::_to_copy.default"}


class Count(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.by_line = collections.Counter()
        self.by_op = collections.Counter()
        self.total = 0

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = "aten::" + func.__name__.split(".")[0]
        if name not in SKIP_OPS:
            where = "?"
            for fr in reversed(traceback.extract_stack(limit=40)):
                if "dense-video-captioning_amd" in fr.filename and "_python_dispatch" not in fr.filename:
                    where = f"{os.path.relpath(fr.filename, PKG)}:{fr.lineno} {fr.name}"
                    break
            self.by_line[where] += 1
            self.by_op[name] += 1
            self.total += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=16)
    ap.add_argument("--top", type=int, default=60)
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

    step()
    torch.cuda.synchronize()
    c = Count()
    with c:
        step()
    torch.cuda.synchronize()
    print(f"{c.total} aten ops in one step (views/allocs excluded)")
    for where, n in c.by_line.most_common(a.top):
        print(f"{n:6d}  {where}")
    print("--- by op")
    for op, n in c.by_op.most_common(30):
        print(f"{n:6d}  {op}")


if __name__ == "__main__":
    main()
