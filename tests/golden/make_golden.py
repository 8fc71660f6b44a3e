#!/usr/bin/env python
"""Generate the golden fixtures in tests/golden/*.npz from the *reference* implementation.

Run in the build container only (it imports /root/reference, which does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
The fixtures are data (inputs + expected outputs); no reference source travels with them.

How the reference is driven:
  * three absent third-party modules are stubbed before import: torchvision (only
    torchvision.ops.boxes.box_area is imported, misc/detr_utils/box_ops.py:6), colorlog
    (misc/utils.py:12) and the CUDA extension MultiScaleDeformableAttention (only reached when
    query.device.type == 'cuda', pdvc/ops/modules/ms_deform_attn.py:119-124 -- never on CPU);
  * CUDA-op semantics (zeros padding, the reference's GPU MSDeformAttn path) are obtained by running
    the reference's own ms_deform_attn_core_pytorch with grid_sample's padding forced to 'zeros'
    (the upstream Deformable-DETR core that the CUDA kernel equals);
    border semantics (the reference CPU core, and MSDeformAttnCap on every device) are the
    unmodified reference core.
"""
import os
import sys
import types
import contextlib

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("PDVC_REFERENCE", "/root/reference")
sys.path.insert(0, HERE)
import weights as W  # noqa: E402


def install_stubs():
    tv = types.ModuleType("torchvision")
    tv.__version__ = "0.14.1"
    ops = types.ModuleType("torchvision.ops")
    boxes = types.ModuleType("torchvision.ops.boxes")
    boxes.box_area = lambda b: (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    ops.boxes = boxes
    tv.ops = ops
    sys.modules.update({"torchvision": tv, "torchvision.ops": ops, "torchvision.ops.boxes": boxes})
    cl = types.ModuleType("colorlog")

    class ColoredFormatter:  # noqa: D401 - stub
        def __init__(self, *a, **k):
            pass
    cl.ColoredFormatter = ColoredFormatter
    sys.modules["colorlog"] = cl
    msda = types.ModuleType("MultiScaleDeformableAttention")

    def _no_cuda(*a, **k):
        raise RuntimeError("reference CUDA extension is not available in the fixture generator")
    msda.ms_deform_attn_forward = _no_cuda
    msda.ms_deform_attn_backward = _no_cuda
    sys.modules["MultiScaleDeformableAttention"] = msda


install_stubs()
sys.path.insert(0, REF)
os.chdir(REF)  # cfg paths inside the reference are relative

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

_orig_grid_sample = F.grid_sample
_force = {"zeros": False}


def _grid_sample(input, grid, mode="bilinear", padding_mode="zeros", align_corners=None):
    if _force["zeros"]:
        padding_mode = "zeros"
    return _orig_grid_sample(input, grid, mode=mode, padding_mode=padding_mode, align_corners=align_corners)


F.grid_sample = _grid_sample
torch.nn.functional.grid_sample = _grid_sample


@contextlib.contextmanager
def zeros_padding():
    _force["zeros"] = True
    try:
        yield
    finally:
        _force["zeros"] = False


from pdvc.ops.functions.ms_deform_attn_func import ms_deform_attn_core_pytorch as ref_core  # noqa: E402
import pdvc.ops.modules.ms_deform_attn as ref_msda_mod  # noqa: E402


def zeros_core(value, shapes, loc, attn, return_value=False):
    with zeros_padding():
        return ref_core(value, shapes, loc, attn, return_value=return_value)


# The reference GPU path of MSDeformAttn = zeros semantics: route the module through zeros_core.
ref_msda_mod.ms_deform_attn_core_pytorch = zeros_core

OUT = {}


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    clean = {}
    for k, v in arrays.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        clean[k] = np.asarray(v)
    np.savez_compressed(path, **clean)
    OUT[name] = sum(a.nbytes for a in clean.values())


def t(x, dtype=torch.float64, grad=False):
    x = torch.as_tensor(np.asarray(x), dtype=dtype)
    return x.requires_grad_(grad)


# ---------------------------------------------------------------------------------------------
# 1. The reference op test's own inputs (pdvc/ops/test.py:21-44): 2-D shapes, seed 3, fp64.
# ---------------------------------------------------------------------------------------------
def op_reftest():
    N, M, D, Lq, L, P = 1, 2, 2, 2, 2, 2
    shapes = torch.as_tensor([(6, 4), (3, 2)], dtype=torch.long)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    S = int(sum((H * Wd).item() for H, Wd in shapes))
    torch.manual_seed(3)
    value = torch.rand(N, S, M, D) * 0.01
    loc = torch.rand(N, Lq, M, L, P, 2)
    attn = torch.rand(N, Lq, M, L, P) + 1e-5
    attn /= attn.sum(-1, keepdim=True).sum(-2, keepdim=True)
    g = torch.Generator().manual_seed(33)
    gout = torch.rand(N, Lq, M * D, generator=g, dtype=torch.float64) - 0.5
    res = dict(value=value.double(), loc=loc.double(), attn=attn.double(), shapes=shapes, lsi=lsi, grad_out=gout)
    for pad, core in (("zeros", zeros_core), ("border", ref_core)):
        v, lo, a = (x.double().clone().requires_grad_(True) for x in (value, loc, attn))
        out = core(v, shapes, lo, a)
        out.backward(gout)
        res[f"{pad}_out"] = out
        res[f"{pad}_grad_value"] = v.grad
        res[f"{pad}_grad_loc"] = lo.grad
        res[f"{pad}_grad_attn"] = a.grad
    save("op_reftest", **res)


# ---------------------------------------------------------------------------------------------
# 2. 1-D PDVC pyramids (the lifted form, ms_deform_attn.py:182-185), several D to cover the
#    reference's col2im dispatch branches (test.py:85), both padding semantics, fp64 and fp32.
# ---------------------------------------------------------------------------------------------
def op_1d():
    rng = np.random.RandomState(7)
    for D in (30, 32, 64, 71):
        T_l = [16, 8, 4, 2]
        N, M, Lq, L, P = 2, 4, 5, 4, 4
        S = sum(T_l)
        shapes = torch.as_tensor([[1, x] for x in T_l], dtype=torch.long)
        lsi = torch.as_tensor(np.concatenate([[0], np.cumsum(T_l)[:-1]]), dtype=torch.long)
        value = rng.randn(N, S, M, D)
        locx = rng.uniform(-0.2, 1.2, size=(N, Lq, M, L, P))
        loc = np.stack([locx, np.full_like(locx, 0.5)], -1)
        attn = rng.uniform(0.01, 1.0, size=(N, Lq, M, L, P))
        attn /= attn.sum(axis=(-1, -2), keepdims=True)
        gout = rng.randn(N, Lq, M * D)
        res = dict(value=value, loc=loc, attn=attn, shapes=shapes, lsi=lsi, grad_out=gout)
        for dt_name, dt in (("f64", torch.float64), ("f32", torch.float32)):
            for pad, core in (("zeros", zeros_core), ("border", ref_core)):
                v, lo, a = (t(x, dt, True) for x in (value, loc, attn))
                out = core(v, shapes, lo, a)
                out.backward(t(gout, dt))
                res[f"{pad}_{dt_name}_out"] = out
                res[f"{pad}_{dt_name}_grad_value"] = v.grad
                res[f"{pad}_{dt_name}_grad_loc"] = lo.grad
                res[f"{pad}_{dt_name}_grad_attn"] = a.grad
        save(f"op_1d_D{D}", **res)


# ---------------------------------------------------------------------------------------------
# 3. Raw-sample mode (return_value=True) = what MSDeformAttnCap returns (ms_deform_attn_func.py:64-65).
# ---------------------------------------------------------------------------------------------
def op_sample():
    rng = np.random.RandomState(11)
    T_l = [16, 8, 4, 2]
    N, M, D, Lq, L, P = 1, 1, 48, 6, 4, 4
    S = sum(T_l)
    shapes = torch.as_tensor([[1, x] for x in T_l], dtype=torch.long)
    lsi = torch.as_tensor(np.concatenate([[0], np.cumsum(T_l)[:-1]]), dtype=torch.long)
    value = rng.randn(N, S, M, D)
    locx = rng.uniform(-0.2, 1.2, size=(N, Lq, M, L, P))
    loc = np.stack([locx, np.full_like(locx, 0.5)], -1)
    attn = np.full((N, Lq, M, L, P), 1.0 / (L * P))
    gsamp = rng.randn(N * M, D, Lq, L, P)
    res = dict(value=value, loc=loc, shapes=shapes, lsi=lsi, grad_samples=gsamp)
    for dt_name, dt in (("f64", torch.float64), ("f32", torch.float32)):
        v, lo = t(value, dt, True), t(loc, dt, True)
        out = ref_core(v, shapes, lo, t(attn, dt), return_value=True)
        out.backward(t(gsamp, dt))
        res[f"{dt_name}_samples"] = out
        res[f"{dt_name}_grad_value"] = v.grad
        res[f"{dt_name}_grad_loc"] = lo.grad
    save("op_sample", **res)


def named_grads(module):
    return {"grad." + n: p.grad if p.grad is not None else torch.zeros(0) for n, p in module.named_parameters()}


# ---------------------------------------------------------------------------------------------
# 4. The MSDeformAttn module (ms_deform_attn.py:79-126) with GPU (zeros) semantics, 1-D refs.
# ---------------------------------------------------------------------------------------------
def module_msdeformattn():
    from pdvc.ops.modules import MSDeformAttn
    rng = np.random.RandomState(5)
    d, Mh, L, P = 64, 4, 4, 4
    T_l = [16, 8, 4, 2]
    S = sum(T_l)
    for ref_dim in (1, 2):
        m = MSDeformAttn(d, L, Mh, P)
        W.fill_module(m, overrides={"sampling_offsets": 0.5})
        N, Lq = 2, 7
        query = rng.randn(N, Lq, d).astype(np.float32)
        x = rng.randn(N, S, d).astype(np.float32)
        if ref_dim == 1:
            ref = rng.uniform(0.0, 1.0, size=(N, Lq, L, 1)).astype(np.float32)
        else:
            c = rng.uniform(0.1, 0.9, size=(N, Lq, L, 1))
            ln = rng.uniform(0.05, 0.6, size=(N, Lq, L, 1))
            ref = np.concatenate([c, ln], -1).astype(np.float32)
        pad = np.zeros((N, S), dtype=bool)
        pad[1, 14:16] = True
        pad[1, 22:24] = True
        gout = rng.randn(N, Lq, d).astype(np.float32)
        qt, rt, xt = t(query, torch.float32, True), t(ref, torch.float32, True), t(x, torch.float32, True)
        shapes = torch.as_tensor(T_l, dtype=torch.long)
        lsi = torch.as_tensor(np.concatenate([[0], np.cumsum(T_l)[:-1]]), dtype=torch.long)
        out = m(qt, rt, xt, shapes, lsi, torch.as_tensor(pad))
        out.backward(t(gout, torch.float32))
        save(f"module_msdeformattn_ref{ref_dim}", query=query, ref=ref, x=x, pad=pad, T_l=np.asarray(T_l),
             grad_out=gout, out=out, grad_query=qt.grad, grad_ref=rt.grad, grad_x=xt.grad, **named_grads(m))


# ---------------------------------------------------------------------------------------------
# 5. One deformable decoder layer (deformable_transformer.py:219-271) and one encoder layer
#    (:149-189), dropout 0, GPU semantics for MSDA.
# ---------------------------------------------------------------------------------------------
def module_layers():
    from pdvc.deformable_transformer import DeformableTransformerDecoderLayer, DeformableTransformerEncoderLayer
    rng = np.random.RandomState(9)
    d, ffn, Mh, L, P = 64, 48, 4, 4, 4
    T_l = [16, 8, 4, 2]
    S = sum(T_l)
    shapes = torch.as_tensor(T_l, dtype=torch.long)
    lsi = torch.as_tensor(np.concatenate([[0], np.cumsum(T_l)[:-1]]), dtype=torch.long)
    N, Q = 2, 9
    # decoder layer
    layer = DeformableTransformerDecoderLayer(d, ffn, 0.0, "relu", L, Mh, P)
    W.fill_module(layer, overrides={"sampling_offsets": 0.5})
    tgt = rng.randn(N, Q, d).astype(np.float32)
    qpos = rng.randn(N, Q, d).astype(np.float32)
    ref = rng.uniform(0, 1, size=(N, Q, L, 1)).astype(np.float32)
    src = rng.randn(N, S, d).astype(np.float32)
    pad = np.zeros((N, S), dtype=bool)
    qmask = np.ones((N, Q), dtype=bool)
    qmask[1, -2:] = False
    gout = rng.randn(N, Q, d).astype(np.float32)
    tt, pt, rt, st = (t(a, torch.float32, True) for a in (tgt, qpos, ref, src))
    out = layer(tt, pt, rt, st, shapes, lsi, torch.as_tensor(pad), torch.as_tensor(qmask))
    out.backward(t(gout, torch.float32))
    save("module_decoder_layer", tgt=tgt, query_pos=qpos, ref=ref, src=src, pad=pad, query_mask=qmask,
         T_l=np.asarray(T_l), grad_out=gout, out=out, grad_tgt=tt.grad, grad_query_pos=pt.grad,
         grad_ref=rt.grad, grad_src=st.grad, **named_grads(layer))
    # encoder layer
    layer = DeformableTransformerEncoderLayer(d, ffn, 0.0, "relu", L, Mh, P)
    W.fill_module(layer, overrides={"sampling_offsets": 0.5})
    src = rng.randn(N, S, d).astype(np.float32)
    pos = rng.randn(N, S, d).astype(np.float32)
    ref = rng.uniform(0, 1, size=(N, S, L, 1)).astype(np.float32)
    gout = rng.randn(N, S, d).astype(np.float32)
    st, pt = t(src, torch.float32, True), t(pos, torch.float32, True)
    out = layer(st, pt, t(ref, torch.float32), shapes, lsi, torch.as_tensor(pad))
    out.backward(t(gout, torch.float32))
    save("module_encoder_layer", src=src, pos=pos, ref=ref, pad=pad, T_l=np.asarray(T_l), grad_out=gout,
         out=out, grad_src=st.grad, grad_pos=pt.grad, **named_grads(layer))


def small_opt(**kw):
    opt = types.SimpleNamespace(
        vocab_size=23, input_encoding_size=32, rnn_size=64, num_layers=1, drop_prob=0.0,
        max_caption_len=6, clip_context_dim=64, cap_nheads=1, att_hid_size=48,
        wordRNN_input_feats_type="C", hidden_dim=64, cap_num_feature_levels=4, cap_dec_n_points=4,
        num_feature_levels=4, event_context_dim=None)
    for k, v in kw.items():
        setattr(opt, k, v)
    return opt


# ---------------------------------------------------------------------------------------------
# 6. The caption head (pdvc/CaptioningHead/LSTM_DSA.py): teacher-forced forward (captioning
#    logits = log_softmax outputs), build_loss, backward; greedy sample().
# ---------------------------------------------------------------------------------------------
def module_captioner():
    from pdvc.CaptioningHead.LSTM_DSA import LSTMDSACaptioner
    rng = np.random.RandomState(13)
    T_l = [16, 8, 4, 2]
    S = sum(T_l)
    for ref_dim in (1, 2):
        opt = small_opt()
        cap = LSTMDSACaptioner(opt)
        W.fill_module(cap, overrides={"sampling_offsets": 0.5})
        cap.train()
        E = 5
        hs = rng.randn(1, E, 64).astype(np.float32)
        if ref_dim == 1:
            ref = rng.uniform(0, 1, size=(1, E, 1)).astype(np.float32)
        else:
            ref = np.stack([rng.uniform(0.1, 0.9, size=(1, E)), rng.uniform(0.05, 0.7, size=(1, E))],
                           -1).astype(np.float32)
        memory = rng.randn(1, S, 64).astype(np.float32)
        mask = np.zeros((1, S), dtype=bool)
        K = 7
        cap_tensor = np.zeros((E, K), dtype=np.int64)
        lens = [5, 3, 6, 2, 4]
        for e in range(E):
            cap_tensor[e, 1:1 + lens[e]] = rng.randint(1, opt.vocab_size, size=lens[e])
        cap_mask = cap_tensor != 0
        cap_mask[:, 0] = True
        ht, rt, mt = t(hs, torch.float32, True), t(ref, torch.float32, True), t(memory, torch.float32, True)
        others = {"memory": mt, "spatial_shapes": torch.as_tensor(T_l, dtype=torch.long),
                  "level_start_index": torch.as_tensor(np.concatenate([[0], np.cumsum(T_l)[:-1]]), dtype=torch.long),
                  "mask_flatten": torch.as_tensor(mask), "valid_ratios": torch.ones(1, 4)}
        logprobs = cap(ht, rt, others, torch.as_tensor(cap_tensor))
        loss = cap.build_loss(logprobs, torch.as_tensor(cap_tensor[:, 1:]), torch.as_tensor(cap_mask[:, 1:])).mean()
        loss.backward()
        cap.eval()
        with torch.no_grad():
            seq, seqlp = cap.sample(ht.detach(), rt.detach(), {k: (v.detach() if isinstance(v, torch.Tensor) else v)
                                                               for k, v in others.items()})
        save(f"module_captioner_ref{ref_dim}", hs=hs, ref=ref, memory=memory, mask=mask, T_l=np.asarray(T_l),
             cap_tensor=cap_tensor, cap_mask=cap_mask, logprobs=logprobs, loss=loss, grad_hs=ht.grad,
             grad_ref=rt.grad, grad_memory=mt.grad, sample_seq=seq, sample_logprobs=seqlp, **named_grads(cap))


# ---------------------------------------------------------------------------------------------
# 7. Whole PDVC training fwd+bwd and eval fwd at a reduced size (hidden_dim must stay 512,
#    position_encoding.py:35,54).  cfg anet_tsp_pdvc.yml + overrides; dropout 0.
# ---------------------------------------------------------------------------------------------
def ref_args(cfg, **over):
    import opts as ref_opts
    argv = sys.argv
    sys.argv = ["x", "--cfg_path", cfg, "--device", "cpu"]
    try:
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            args = ref_opts.parse_opts()
    finally:
        sys.argv = argv
    for k, v in over.items():
        setattr(args, k, v)
    return args


def pack_grad(res, name, g):
    """Store one full gradient tensor under `name`.  A 2-D gradient of low numerical rank (a Linear weight
    gradient is a sum of one outer product per GEMM row: rank <= rows, e.g. S = 30 rows per video at T = 16)
    is stored as float32 factors `name.A` (m, r) @ `name.B` (r, n) of its float64 SVD, with the smallest r
    whose float32-factor reconstruction is within 1e-6 * max(1, max|g|) of every element; the achieved
    error is stored as `name.err`.  The tests rebuild the full tensor and compare every element."""
    g = g.detach().double().cpu().numpy()
    shape = g.shape
    if g.ndim > 2:  # conv weights (out, in, k): factored as (out, in*k)
        g = g.reshape(shape[0], -1)
    if g.ndim == 2 and min(g.shape) >= 32:
        m, n = g.shape
        U, s, Vt = np.linalg.svd(g, full_matrices=False)
        bound = 1e-6 * max(1.0, float(np.abs(g).max()))
        # candidate ranks: singular values above a relative noise floor, grown until the bound holds
        r = int((s > s[0] * 1e-7).sum()) if s[0] > 0 else 1
        while r <= min(m, n) and (m + n) * r < m * n // 2:
            A = (U[:, :r] * s[:r]).astype(np.float32)
            B = Vt[:r].astype(np.float32)
            err = float(np.abs(A.astype(np.float64) @ B.astype(np.float64) - g).max())
            if err <= bound:
                res[name + ".A"], res[name + ".B"], res[name + ".err"] = A, B, np.float64(err)
                res[name + ".shape"] = np.asarray(shape, np.int64)
                return
            r = max(r + 1, int(r * 1.25))
    res[name] = g.reshape(shape).astype(np.float32)


def pack_model_grads(res, model, scale=1.0):
    for n, p in model.named_parameters():
        if p.grad is None:
            res["gradnone." + n] = np.zeros(0)
        else:
            pack_grad(res, "grad." + n, p.grad * scale)


def whole_model():
    import io
    from pdvc.pdvc import build
    from data.video_dataset import collate_fn
    cases = [
        ("pdvc_small_anet", "cfgs/anet_tsp_pdvc.yml",
         dict(feature_dim=32, num_queries=10, enc_layers=2, dec_layers=2, transformer_ff_dim=64,
              vocab_size=29, transformer_dropout_prob=0.0, drop_prob=0.0, max_caption_len=8), 16, 3, 5, 120.0),
        ("pdvc_small_yc2_3l", "cfgs/yc2_tsp_pdvc.yml",
         dict(feature_dim=24, num_queries=12, enc_layers=3, dec_layers=3, transformer_ff_dim=32,
              vocab_size=31, transformer_dropout_prob=0.0, drop_prob=0.0, max_caption_len=8,
              max_eseq_length=20), 20, 4, 4, 200.0),
    ]
    for name, cfg, over, T, E, words, duration in cases:
        args = ref_args(cfg, **over)
        torch.manual_seed(0)
        with contextlib.redirect_stdout(io.StringIO()):
            model, criterion, _ = build(args)
        W.fill_module(model, overrides={"sampling_offsets": 0.5})
        model.train()
        batch = W.synthetic_video_batch(1, T, args.feature_dim, E, words, args.vocab_size, duration=duration, seed=1)
        dt = collate_fn(batch)
        dt = {k: v for k, v in dt.items()}
        dt["video_target"] = [{k: v for k, v in tg.items()} for tg in dt["video_target"]]
        out, loss = model(dt, criterion, "queries")
        wd = criterion.weight_dict
        total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
        total.backward()
        res = {"total_loss": total.detach()}
        for k, v in loss.items():
            res["loss." + k] = v.detach() if isinstance(v, torch.Tensor) else np.asarray(v)
        res["pred_logits"] = out["pred_logits"]
        res["pred_boxes"] = out["pred_boxes"]
        res["pred_count"] = out["pred_count"]
        res["cap_prob_train"] = out["caption_probs"]["cap_prob_train"]
        for li, (i, j) in enumerate(out["matched_indices"][0]):
            res[f"matched.last.{li}.q"] = i
            res[f"matched.last.{li}.g"] = j
        pack_model_grads(res, model)
        res["param_names"] = np.asarray([n for n, _ in model.named_parameters()])
        res["state_keys"] = np.asarray(list(model.state_dict().keys()))
        res["state_shapes"] = np.asarray([",".join(str(s) for s in v.shape) for v in model.state_dict().values()])
        # eval forward: greedy captions + PostProcess's top-k query ordering (pdvc/pdvc.py:511-514)
        model.eval()
        with torch.no_grad():
            out_e, loss_e = model(dt, criterion, "queries", eval_mode=True)
        prob = out_e["pred_logits"].sigmoid()
        topv, topi = torch.topk(prob.view(prob.shape[0], -1), prob.shape[1], dim=1)
        res["eval.pred_logits"] = out_e["pred_logits"]
        res["eval.pred_boxes"] = out_e["pred_boxes"]
        res["eval.pred_count"] = out_e["pred_count"]
        res["eval.seq"] = out_e["seq"]
        res["eval.cap_prob_eval"] = out_e["caption_probs"]["cap_prob_eval"]
        res["eval.topk_query"] = topi // out_e["pred_logits"].shape[2]
        res["eval.count_argmax"] = out_e["pred_count"].argmax(dim=-1).clamp(min=1)
        # inputs (so the test does not depend on weights.synthetic_video_batch staying unchanged)
        res["in.video_tensor"] = dt["video_tensor"]
        res["in.video_mask"] = dt["video_mask"]
        res["in.video_length"] = dt["video_length"]
        res["in.boxes"] = dt["video_target"][0]["boxes"]
        res["in.labels"] = dt["video_target"][0]["labels"]
        res["in.cap_tensor"] = dt["cap_tensor"]
        res["in.cap_mask"] = dt["cap_mask"]
        res["in.gt_boxes"] = dt["gt_boxes"]
        res["in.gt_boxes_mask"] = dt["gt_boxes_mask"]
        res["args"] = np.asarray([f"{k}={v!r}" for k, v in sorted(over.items())] + [f"cfg={cfg!r}"])
        save(name, **res)


def synthetic_translator(vocab):
    """The reference Translator (data/video_dataset.py:152-180) over a synthetic vocabulary w1..w{vocab}."""
    import json
    import tempfile
    from data.video_dataset import Translator
    vocab_json = {"word_to_ix": {f"w{i}": i for i in range(1, vocab + 1)},
                  "ix_to_word": {str(i): f"w{i}" for i in range(1, vocab + 1)}}
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(vocab_json, f)
        path = f.name
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        tr = Translator(path, vocab)
    os.unlink(path)
    return tr


def whole_model_batch_gt():
    """whole_model_batch with transformer_input_type 'gt_proposals' (cfgs/*_gt.yml; pdvc/pdvc.py:138-143,
    misc/utils.py:31-49): the ground-truth segments are the decoder's queries, the refinement is off and the
    class / box / GIoU / length losses weigh 0 (decide_two_stage mutates the criterion)."""
    whole_model_batch("gt_proposals", "pdvc_batch3_anet_gt")


def whole_model_batch(tit="queries", fixture_name="pdvc_batch3_anet"):
    """Reference batch-1 training steps on three different videos (batch_items): per-video losses, matched
    indices of every decoder layer, captioning log-probabilities and heads; the MEAN of the three per-video
    gradients as full tensors (what one 3-video batch of the MI355X path must produce: every loss is the mean
    over videos of the batch-1 value, pdvc/criterion.py:154-198 normalising per video).  Also each video's eval
    forward (greedy captions) and the reference PostProcess (pdvc/pdvc.py:493-546) on it."""
    import io
    import types as _types
    from pdvc.pdvc import build, PostProcess
    from data.video_dataset import collate_fn
    over = dict(feature_dim=32, num_queries=10, enc_layers=2, dec_layers=2, transformer_ff_dim=64,
                vocab_size=29, transformer_dropout_prob=0.0, drop_prob=0.0, max_caption_len=8)
    cfg = "cfgs/anet_tsp_pdvc.yml"
    args = ref_args(cfg, **over)
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        model, criterion, post = build(args)
    W.fill_module(model, overrides={"sampling_offsets": 0.5})
    items = W.batch_items(vocab=args.vocab_size)
    T = max(it[0].shape[0] for it in items)
    captured = {}
    orig_forward = criterion.forward

    def capture(*a, **k):
        r = orig_forward(*a, **k)
        captured["r"] = r
        return r
    criterion.forward = capture
    tr = synthetic_translator(args.vocab_size)
    loader = _types.SimpleNamespace(dataset=_types.SimpleNamespace(translator=tr))
    res = {}
    grads = {}
    wd = criterion.weight_dict
    nv = len(items)
    for v, item in enumerate(items):
        dt = collate_fn([item])
        Tv = dt["video_tensor"].shape[1]
        if Tv < T:  # the batch's padding of this video (collate_fn pads every video to the longest)
            dt["video_tensor"] = torch.cat([dt["video_tensor"], dt["video_tensor"].new_zeros(1, T - Tv, 32)], 1)
            dt["video_mask"] = torch.cat([dt["video_mask"], dt["video_mask"].new_zeros(1, T - Tv)], 1)
        model.train()
        model.zero_grad(set_to_none=True)
        out, loss = model(dt, criterion, tit)
        total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
        total.backward()
        for n, p in model.named_parameters():
            if p.grad is not None:
                grads[n] = grads.get(n, 0) + p.grad.detach().double() / nv
            else:
                grads.setdefault(n, None)
        res[f"v{v}.total_loss"] = total.detach()
        for k, val in loss.items():
            res[f"v{v}.loss.{k}"] = val.detach() if isinstance(val, torch.Tensor) else np.asarray(val)
        res[f"v{v}.pred_logits"] = out["pred_logits"]
        res[f"v{v}.pred_boxes"] = out["pred_boxes"]
        res[f"v{v}.pred_count"] = out["pred_count"]
        res[f"v{v}.cap_prob_train"] = out["caption_probs"]["cap_prob_train"]
        _, last_indices, aux_indices = captured["r"]
        layer_idx = [aux_indices[l][0] for l in range(len(aux_indices))] + [last_indices[0]]
        for l_id, ind in enumerate(layer_idx):
            i, j = ind[0]
            res[f"v{v}.matched.{l_id}.q"] = i
            res[f"v{v}.matched.{l_id}.g"] = j
        # eval forward + PostProcess on this video
        model.eval()
        with torch.no_grad():
            out_e, _ = model(dt, criterion, tit, eval_mode=True)
            pp = post["bbox"](out_e, dt["video_length"][:, 1], loader)[0]
        res[f"v{v}.eval.pred_logits"] = out_e["pred_logits"]
        res[f"v{v}.eval.pred_boxes"] = out_e["pred_boxes"]
        res[f"v{v}.eval.pred_count"] = out_e["pred_count"]
        res[f"v{v}.eval.seq"] = out_e["seq"]
        res[f"v{v}.eval.cap_prob_eval"] = out_e["caption_probs"]["cap_prob_eval"]
        for k in ("scores", "labels", "boxes", "query_id", "vid_duration", "pred_seq_len"):
            res[f"v{v}.post.{k}"] = pp[k]
        res[f"v{v}.post.caption_scores"] = np.asarray(pp["caption_scores"], np.float64)
        res[f"v{v}.post.captions"] = np.asarray(pp["captions"])
    for n, g in grads.items():
        if g is None:
            res["gradnone." + n] = np.zeros(0)
        else:
            pack_grad(res, "grad." + n, g)
    res["param_names"] = np.asarray([n for n, _ in model.named_parameters()])
    res["args"] = np.asarray([f"{k}={v!r}" for k, v in sorted(over.items())] + [f"cfg={cfg!r}"])
    res["n_videos"] = np.asarray(nv)
    res["transformer_input_type"] = np.asarray(tit)
    res["weight_dict_keys"] = np.asarray(list(wd.keys()))
    res["weight_dict_vals"] = np.asarray(list(wd.values()), np.float64)
    save(fixture_name, **res)


INGEST_WORDS = ["a", "man", "is", "cutting", "the", "onion", "with", "knife", "woman", "pours", "water", "into",
                "pot", "and", "stirs", "it", "slowly", "then", "adds", "salt"]
INGEST_SENTENCES = ["A man is cutting the onion.", "The woman pours water into the pot, and stirs it slowly!",
                    "then-adds salt/pepper; \"quickly\"", "  ", "UNKNOWN words: zebra_unicorn?",
                    "a man a man a man a man a man a man a man a man a man", "stirs\\nthe\\pot"]


def data_ingestion():
    """Reference data path (data/video_dataset.py): resizeFeature (:386-397), Translator (:152-180),
    process_time_step (:210-217) and PropSeqDataset.__getitem__ (:232-293) on feature files written to a
    temporary folder; the inputs (feature arrays, annotation and vocabulary JSON text) are stored with the
    outputs so the test rebuilds the same folder."""
    import io
    import json
    import shutil
    import tempfile
    from data.video_dataset import resizeFeature, PropSeqDataset, EDVCdataset
    rng = np.random.RandomState(17)
    res = {}
    for c, (t0, n) in enumerate([(1, 5), (7, 16), (16, 7), (10, 10), (33, 100), (100, 33), (2, 3), (513, 512)]):
        x = rng.randn(t0, 4).astype(np.float32)
        res[f"resize.{c}.in"] = x
        res[f"resize.{c}.n"] = np.asarray(n)
        res[f"resize.{c}.out"] = resizeFeature(x, n, "nearest")
    vocab = {"word_to_ix": {w: i + 1 for i, w in enumerate(INGEST_WORDS)},
             "ix_to_word": {str(i + 1): w for i, w in enumerate(INGEST_WORDS)}}
    vocab_text = json.dumps(vocab)
    tmp = tempfile.mkdtemp(prefix="pdvc_ingest_")
    try:
        vpath = os.path.join(tmp, "vocab.json")
        with open(vpath, "w") as f:
            f.write(vocab_text)
        from data.video_dataset import Translator
        with contextlib.redirect_stdout(io.StringIO()):
            tr = Translator(vpath, len(INGEST_WORDS))
        for i, s in enumerate(INGEST_SENTENCES):
            for ml in (6, 30):
                res[f"translate.{i}.{ml}"] = tr.translate(s, ml)
        ids = [[3, 4, 5, 0, 7], [0, 1], [1, 2, 3], [], [20, 19, 18, 0, 0]]
        for i, s in enumerate(ids):
            res[f"rtranslate.{i}.in"] = np.asarray(s, np.int64)
            res[f"rtranslate.{i}.out"] = np.asarray(tr.rtranslate(np.asarray(s, np.int64)))
        pts = [(120.0, [[0.0, 10.5], [100.0, 130.0]], 100), (33.3, [[1.0, 2.0], [-5.0, 33.3]], 64)]
        for i, (dur, ts, fl) in enumerate(pts):
            res[f"timestep.{i}.out"] = np.asarray(EDVCdataset.process_time_step(None, dur, ts, fl))
        # a feature folder: 4 videos (vggish npy of different lengths, one missing, one of a single row),
        # plus tsn_100 csv files for the two-type dataset
        keys = ["v_QOlSCBRmfWY", "v_ehGHCYKzyZ8", "v_nwznKOuZM7w", "v_missing0000"]
        lengths = [37, 5, 1, None]
        anno = {}
        os.makedirs(os.path.join(tmp, "vgg"))
        os.makedirs(os.path.join(tmp, "tsn"))
        for k, T0 in zip(keys, lengths):
            if T0 is not None:
                f = rng.randn(T0, 128).astype(np.float32)
                res[f"feat.{k}"] = f
                np.save(os.path.join(tmp, "vgg", k[:13] + ".npy"), f)
                ftsn = rng.randn(T0 + 2, 400).astype(np.float64).round(5)
                res[f"tsn.{k}"] = ftsn
                import pandas as pd
                pd.DataFrame(ftsn).to_csv(os.path.join(tmp, "tsn", k[:13] + ".csv"), index=False)
            ne = int(rng.randint(1, 14))
            dur = float(rng.uniform(20, 200))
            ts = np.sort(rng.uniform(0, dur, size=(ne, 2)), 1).round(2).tolist()
            anno[k] = {"duration": round(dur, 2), "timestamps": ts,
                       "sentences": [INGEST_SENTENCES[int(rng.randint(len(INGEST_SENTENCES)))] for _ in range(ne)]}
        anno_text = json.dumps(anno)
        apath = os.path.join(tmp, "anno.json")
        with open(apath, "w") as f:
            f.write(anno_text)
        res["anno_json"] = np.asarray(anno_text)
        res["vocab_json"] = np.asarray(vocab_text)
        res["keys"] = np.asarray(keys)
        for name, vtype, folder, fdim, rescale in (
                ("single", "vggish", os.path.join(tmp, "vgg"), 128, 1),
                ("multi", ["vggish", "tsn_100"], [os.path.join(tmp, "vgg"), os.path.join(tmp, "tsn")], 528, 1),
                ("norescale", "vggish", os.path.join(tmp, "vgg"), 128, 0)):
            opt = types.SimpleNamespace(vocab_size=len(INGEST_WORDS), max_caption_len=8, invalid_video_json=[],
                                        feature_sample_rate=2, train_proposal_sample_num=24,
                                        gt_proposal_sample_num=4, feature_dim=fdim, num_queries=10,
                                        visual_feature_type=vtype, data_rescale=rescale, frame_embedding_num=16,
                                        data_norm=0, num_classes=1)
            with contextlib.redirect_stdout(io.StringIO()):
                ds = PropSeqDataset(apath, folder, vpath, True, "gt", opt)
                np.random.seed(123)
                for i in range(len(ds)):
                    feats, fst, labels, caps, ts, dur, raw, key = ds[i]
                    p = f"ds.{name}.{i}."
                    res[p + "feats"] = np.asarray(feats)
                    res[p + "featstamps"] = np.asarray(fst, np.int64).reshape(-1, 2)
                    res[p + "labels"] = np.asarray(labels, np.int64)
                    res[p + "ncaps"] = np.asarray(len(caps))
                    for j, cp in enumerate(caps):
                        res[p + f"cap{j}"] = np.asarray(cp, np.int64)
                    res[p + "timestamps"] = np.asarray(ts, np.float64).reshape(-1, 2)
                    res[p + "duration"] = np.asarray(dur)
                    res[p + "raw"] = np.asarray(raw)
                    res[p + "key"] = np.asarray(key)
    finally:
        shutil.rmtree(tmp)
    save("data_ingestion", **res)


def state_dict_keys_full():
    """Key list + shapes of the full-size anet_tsp_pdvc model with BASELINE's overrides (C=768, Q=100)."""
    import io
    from pdvc.pdvc import build
    args = ref_args("cfgs/anet_tsp_pdvc.yml", feature_dim=768, num_queries=100)
    with contextlib.redirect_stdout(io.StringIO()):
        model, criterion, _ = build(args)
    sd = model.state_dict()
    save("state_dict_anet_tsp_c768_q100", keys=np.asarray(list(sd.keys())),
         shapes=np.asarray([",".join(str(s) for s in v.shape) for v in sd.values()]),
         param_names=np.asarray([n for n, _ in model.named_parameters()]),
         n_params=np.asarray(sum(p.numel() for p in model.parameters())),
         weight_dict_keys=np.asarray(list(criterion.weight_dict.keys())),
         weight_dict_vals=np.asarray(list(criterion.weight_dict.values()), dtype=np.float64))


def posembed():
    """The encoder's positional input as the reference builds it: PositionEmbeddingSine(256, normalize=True) per
    level on the nearest-interpolated masks (base_encoder.py:54-80, position_encoding.py:20-63), transposed, plus
    the level embedding, concatenated over levels (deformable_transformer.py:84-112).  Three videos, two padded,
    T = 64 -> levels 64/32/16/8; the reference's own duration layer (seeded) and a random level embedding."""
    from misc.detr_utils.misc import NestedTensor
    from pdvc.position_encoding import PositionEmbeddingSine
    torch.manual_seed(11)
    N, T, F_ = 3, 64, 256
    pe = PositionEmbeddingSine(F_, normalize=True)
    d = F_ + pe.max_duration
    mask = torch.zeros(N, T, dtype=torch.bool)
    mask[1, 40:] = True
    mask[2, 21:] = True
    dur = torch.tensor([100.0, 37.0, 12.5])
    level_embed = torch.randn(4, d)
    out = []
    Tl = T
    for lvl in range(4):
        m = mask if lvl == 0 else F.interpolate(mask[None].float(), size=(Tl,)).to(torch.bool)[0]
        src = torch.zeros(N, 8, Tl)
        pos = pe(NestedTensor(src, m, dur))  # (N, d, Tl)
        out.append(pos.transpose(1, 2) + level_embed[lvl].view(1, 1, -1))
        Tl = (Tl + 1) // 2  # kernel-3 / stride-2 / pad-1 conv output length
    save("posembed_levels", mask=mask.numpy(), duration=dur.numpy(), level_embed=level_embed,
         dur_w=pe.duration_embed_layer.weight, dur_b=pe.duration_embed_layer.bias,
         level_T=np.array([64, 32, 16, 8]), lvl_pos=torch.cat(out, 1))


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    which = sys.argv[1:] or ["op_reftest", "op_1d", "op_sample", "module_msdeformattn", "module_layers",
                             "module_captioner", "whole_model", "whole_model_batch", "whole_model_batch_gt", "data_ingestion",
                             "state_dict_keys_full", "posembed"]
    for w in which:
        globals()[w]()
    for k, v in OUT.items():
        print(f"{k:40s} {v / 1024:.1f} KiB")
