"""Diagnostic: gradient w.r.t. the decoder's initial reference points, split by consumer (decoder layer-0
cross-attention, layer-0 box head, caption rows), eager vs StepGraph replays."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dense-video-captioning_amd"), ROOT, os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import test_gpu_model as TM  # noqa: E402
import weights as W  # noqa: E402
import pdvc.pdvc as PP  # noqa: E402
import pdvc.deformable_transformer as DT  # noqa: E402
from pdvc.data import collate, to_device  # noqa: E402
from pdvc.step_graph import StepGraph  # noqa: E402

BUFS = {}


def tap(name, t):
    if isinstance(t, torch.Tensor) and t.requires_grad:
        def h(g):
            if name not in BUFS or BUFS[name].shape != g.shape:
                BUFS[name] = torch.empty_like(g)
            BUFS[name].copy_(g)
        t.register_hook(h)
    return t


orig_prep = DT.DeformableTransformer.prepare_decoder_input_query


def prep(self, memory, query_embed):
    r, tgt, r2, qe = orig_prep(self, memory, query_embed)
    return tap("ref_total", r), tgt, r, qe


DT.DeformableTransformer.prepare_decoder_input_query = prep
orig_layer_fwd = DT.DeformableTransformerDecoderLayer.forward


def layer_fwd(self, tgt, query_pos, reference_points, *a, **k):
    if getattr(self, "_lid", None) == 0:
        reference_points = tap("dec0_ref_in", reference_points * 1.0)
    return orig_layer_fwd(self, tgt, query_pos, reference_points, *a, **k)


DT.DeformableTransformerDecoderLayer.forward = layer_fwd
orig_inv = PP.inverse_sigmoid
calls = {"n": 0}


def inv(x, *a, **k):
    if x.dim() == 3 and x.shape[-1] == 1:
        x = tap("head0_ref", x * 1.0)
    return orig_inv(x, *a, **k)


PP.inverse_sigmoid = inv
orig_rows = PP.PDVC._caption_rows


def rows(self, *a, **k):
    R = orig_rows(self, *a, **k)
    R["ref_rows"] = tap("cap_ref_rows", R["ref_rows"] * 1.0)
    return R


PP.PDVC._caption_rows = rows


def main():
    d = TM.load("pdvc_batch3_anet")
    model, criterion = TM.build_filled(d)
    for i, layer in enumerate(model.transformer.decoder.layers):
        layer._lid = i
    model.train()
    wd = criterion.weight_dict
    mk = lambda: to_device(collate(W.batch_items(vocab=29)[1:2]), "cuda")
    dt = mk()
    _, loss = model(dt, criterion, "queries")
    sum(loss[k] * wd[k] for k in loss.keys() if k in wd).backward()
    torch.cuda.synchronize()
    eager = {k: v.clone() for k, v in BUFS.items()}
    print("eager taps:", {k: tuple(v.shape) for k, v in eager.items()}, flush=True)
    del loss, _
    model.zero_grad(set_to_none=True)
    BUFS.clear()
    sg = StepGraph(model, criterion, mk())
    for r in range(3):
        sg.replay()
        torch.cuda.synchronize()
        for k, v in eager.items():
            if k not in BUFS:
                print(f"replay {r}: {k} missing", flush=True)
                continue
            err = (BUFS[k] - v).abs().max().item()
            print(f"replay {r}: {k:14s} max|diff| {err:.3e}  (|g| {v.abs().max().item():.3e})", flush=True)


if __name__ == "__main__":
    main()
