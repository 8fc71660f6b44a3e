"""The bf16 mode (pdvc/precision.py) -- BASELINE.json configs[1], yc2_tsp_pdvc on 1 MI355X in
bf16.  The reference is fp32-only, so the fp32 path (pinned to the reference's fixtures elsewhere) is the
oracle here.

Stated tolerances (also in DESIGN.md):
  * every rerouted GEMM form: equal to float64 on operands rounded to bf16 within 1e-5 * sqrt(K) * scale
    (products of bf16 values are exact in fp32, only the fp32 accumulation differs), scale = max|a| * max|b|,
    and within 2^-7 * sqrt(K) * scale of float64 on the unrounded operands;
  * whole training step at the cfg-2 shape (T=256, C=768, Q=100, d=512, 2+2 layers, vocab 5748), dropout off:
    every loss within 2e-2 * max(1, |loss_fp32|) (the non-caption losses also under the bf16 step's own set
    matching -- a random-init model's near-tied costs let bf16 rounding flip matches, so gradients and caption
    losses are compared under the fp32 step's matching); every parameter gradient with ||g_bf16 - g_fp32|| <= 0.1 *
    ||g_fp32|| (relative L2) and cosine >= 0.995 (gradients that vanish in exact arithmetic -- ||g_fp32|| below
    1e-3 of the largest gradient norm, e.g. the soft-attention logit bias under its softmax -- within 1e-3 of
    that largest norm instead); the StepGraph replay of the bf16 step equal to the eager bf16
    step within 1e-2 relative L2 per gradient (the library may pick other GEMM algorithms under capture: an
    fp32 summation-order difference of one ulp can flip the bf16 rounding of the next GEMM's operand, so
    replay-vs-eager noise grows to ~1e-3 -- still 50x below the bf16-vs-fp32 differences); never-used
    parameters None in both.
"""
import math
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "dense-video-captioning_amd")
DEV = "cuda"


def bf16_round(t):
    return t.to(torch.bfloat16).to(torch.float32)


OPS = ["mm", "mm_out", "addmm", "addmm_out", "addmm_", "addmm_relu", "bmm", "baddbmm"]


@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True)])
def test_mode_gemms_vs_float64(op, ta, tb):
    """Every rerouted overload equals float64 on bf16-rounded operands within 1e-5 * sqrt(K) * scale (bf16
    products are exact in fp32; only the fp32 accumulation differs), and float64 on the unrounded operands
    within 2^-7 * sqrt(K) * scale; the fp32 result of each form (out=, in place) lands where it should."""
    from pdvc.precision import bf16_matmul, STATS
    g = torch.Generator(device=DEV).manual_seed(11)
    M, N, K, B = 300, 200, 512, 3
    batched = op in ("bmm", "baddbmm")
    shp = lambda r, c, t: ((B,) if batched else ()) + ((c, r) if t else (r, c))
    a = torch.randn(shp(M, K, ta), device=DEV, generator=g)
    b = torch.randn(shp(K, N, tb), device=DEV, generator=g)
    A = a.transpose(-1, -2) if ta else a
    Bm = b.transpose(-1, -2) if tb else b
    bias = torch.randn(N, device=DEV, generator=g)
    c0 = torch.randn(((B,) if batched else ()) + (M, N), device=DEV, generator=g)
    out = torch.empty_like(c0)
    STATS.clear()
    with bf16_matmul():
        if op == "mm":
            y = torch.mm(A, Bm)
        elif op == "mm_out":
            y = torch.mm(A, Bm, out=out)
        elif op == "addmm":
            y = torch.addmm(bias, A, Bm)
        elif op == "addmm_out":
            y = torch.addmm(bias, A, Bm, out=out)
        elif op == "addmm_":
            y = c0.clone().addmm_(A, Bm)
        elif op == "addmm_relu":
            y = torch._addmm_activation(bias, A, Bm)
        elif op == "bmm":
            y = torch.bmm(A, Bm)
        else:
            y = torch.baddbmm(c0, A, Bm, beta=0.5, alpha=2.0)
    assert sum(v[0] for v in STATS.values()) == 1, f"{op}: not routed to bf16 ({STATS})"
    assert y.dtype == torch.float32
    if op.endswith("_out"):
        assert y.data_ptr() == out.data_ptr()
    r16 = bf16_round(A).double() @ bf16_round(Bm).double()
    r64 = A.double() @ Bm.double()
    extra = {"addmm": bias.double(), "addmm_out": bias.double(), "addmm_relu": bias.double(),
             "addmm_": c0.double()}.get(op, 0)
    if op == "baddbmm":
        r16, r64 = 0.5 * c0.double() + 2 * r16, 0.5 * c0.double() + 2 * r64
    else:
        r16, r64 = r16 + extra, r64 + extra
    if op == "addmm_relu":
        r16, r64 = r16.clamp(min=0), r64.clamp(min=0)
    scale = math.sqrt(K) * float(a.abs().max()) * float(b.abs().max()) * (2 if op == "baddbmm" else 1)
    assert (y.double() - r16).abs().max().item() <= 1e-5 * scale
    assert (y.double() - r64).abs().max().item() <= 2 ** -7 * scale


def test_mode_keeps_tiny_gemms_fp32():
    from pdvc.precision import bf16_matmul, STATS
    a = torch.randn(100, 512, device=DEV)
    w = torch.randn(512, 1, device=DEV)
    STATS.clear()
    with bf16_matmul():
        y = torch.mm(a, w)
    assert torch.equal(y, torch.mm(a, w)) and sum(v[1] for v in STATS.values()) == 1


def test_dispatch_mode_routes_linear_forward_and_backward():
    """nn.Linear forward and both gradient GEMMs under bf16_matmul equal the fp32 results within bf16 rounding,
    and actually differ from them (the bf16 route ran)."""
    from pdvc.precision import bf16_matmul
    g = torch.Generator(device=DEV).manual_seed(5)
    lin = torch.nn.Linear(512, 384).to(DEV)
    x = torch.randn(2, 700, 512, device=DEV, generator=g, requires_grad=True)
    gy = torch.randn(2, 700, 384, device=DEV, generator=g)

    def run():
        lin.zero_grad()
        x.grad = None
        y = lin(x)
        y.backward(gy)
        return y.detach().clone(), x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()

    ref = run()
    with bf16_matmul():
        got = run()
    for r, o, name in zip(ref, got, ("y", "dx", "dW", "db")):
        rel = ((o - r).norm() / r.norm()).item()
        assert rel < 1e-2, f"{name}: relative error {rel:.3e}"
        if name != "db":  # the bias gradient is a reduction, not a GEMM
            assert rel > 1e-6, f"{name}: identical to fp32 -- the bf16 route did not run"


def _cfg2_model_and_batch():
    sys.path.insert(0, PKG)
    import opts
    from pdvc.pdvc import build
    from pdvc.data import collate, synthetic_videos, to_device
    torch.manual_seed(0)
    args = opts.parse_opts(["--cfg_path", "cfgs/yc2_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG, feature_dim=768,
                           num_queries=100, frame_embedding_num=256)
    args.transformer_dropout_prob = 0.0
    args.drop_prob = 0.0
    model, criterion, _ = build(args)
    model = model.to(DEV).train()
    dt = to_device(collate(synthetic_videos(2, 256, 768, 8, 9, args.vocab_size + 1, seed=7)), DEV)
    return model, criterion, dt


def _step(model, criterion, dt, matched=None):
    wd = criterion.weight_dict
    model.zero_grad(set_to_none=True)
    orig = criterion.forward

    def capture(*a, **k):
        r = orig(*a, **k)
        if matched is not None:
            _, last, aux = r
            matched.extend([[(i.tolist(), j.tolist()) for i, j in list(ix[0])] for ix in list(aux) + [last]])
        return r
    criterion.forward = capture
    try:
        _, loss = model(dt, criterion, "queries")
    finally:
        criterion.forward = orig
    total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    total.backward()
    return ({k: float(v) for k, v in loss.items()},
            {n: (None if p.grad is None else p.grad.detach().clone()) for n, p in model.named_parameters()})


REL_L2, COSINE = 0.1, 0.995


def test_cfg2_training_step_bf16_vs_fp32():
    from pdvc.precision import bf16_matmul
    from pdvc.step_graph import StepGraph
    model, criterion, dt = _cfg2_model_and_batch()
    # A random-init model scores every query almost alike, so the set matching is decided by tiny cost
    # differences that bf16 rounding flips; the gradients are compared under the fp32 step's matching
    # (replayed into the bf16 step), the losses under their own.
    m32, m16 = [], []
    l32, g32 = _step(model, criterion, dt, m32)
    with bf16_matmul():
        l16_own, g16_own = _step(model, criterion, dt, m16)
    print("bf16 step matched like fp32:", m32 == m16)
    solve = criterion.matcher.solve_device
    saved = []
    criterion.matcher.solve_device = lambda *a, **k: saved.append(solve(*a, **k)) or saved[-1]
    _step(model, criterion, dt)
    criterion.matcher.solve_device = lambda *a, **k: saved.pop(0)
    try:
        with bf16_matmul():
            l16, g16 = _step(model, criterion, dt)
    finally:
        criterion.matcher.solve_device = solve
    for k, v in l32.items():
        if np.isnan(v):
            continue
        assert abs(l16[k] - v) <= 2e-2 * max(1.0, abs(v)), f"loss {k}: bf16 {l16[k]} vs fp32 {v}"
        if "caption" not in k:  # the caption losses follow the matching's rows
            assert abs(l16_own[k] - v) <= 2e-2 * max(1.0, abs(v)), f"loss {k} (own matching): {l16_own[k]} vs {v}"
    worst = []
    gmax = max(r.norm().item() for r in g32.values() if r is not None)
    for n, r in g32.items():
        assert (r is None) == (g16[n] is None), n
        if r is None:
            continue
        o = g16[n]
        if r.norm().item() < 1e-3 * gmax:
            assert (o - r).norm().item() <= 1e-3 * gmax, n
            continue
        rel = ((o - r).norm() / r.norm()).item()
        cos = torch.nn.functional.cosine_similarity(o.reshape(1, -1).double(), r.reshape(1, -1).double()).item()
        worst.append((round(rel, 4), round(cos, 5), n))
    worst.sort(reverse=True)
    print("largest relative gradient errors (bf16 vs fp32):", worst[:12])
    bad = [w for w in worst if w[0] > REL_L2 or w[1] < COSINE]
    assert not bad, f"gradients outside relative L2 {REL_L2} / cosine {COSINE}: {bad}"
    # the bench path: the bf16 step captured and replayed as one hipGraph
    with bf16_matmul():
        sg = StepGraph(model, criterion, dt)
    for _ in range(2):
        sg.replay()
        torch.cuda.synchronize()
        for n, p in model.named_parameters():  # against the eager bf16 step with its own matching
            if g16_own[n] is None:
                assert p.grad is None
                continue
            err = (p.grad - g16_own[n]).norm().item()
            assert err <= 1e-2 * g16_own[n].norm().item() + 1e-7, f"replayed grad {n}: {err:.3e}"


def test_cfg2_bf16_step_graph_follows_loaded_batch():
    """The bf16 StepGraph fed a SECOND batch through load() equals the eager bf16 step on that batch: every
    operand rounding of the step is a node of the graph, none is a cast cached from the warm-up batch (ADVICE
    round 2: the warm-up's rounding of dt['video_tensor'] was a cache hit at capture, and every replay after a
    load multiplied the first batch's features)."""
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.precision import bf16_matmul
    from pdvc.step_graph import StepGraph
    model, criterion, dt = _cfg2_model_and_batch()
    with bf16_matmul():
        sg = StepGraph(model, criterion, dt)
    dt2 = to_device(collate(synthetic_videos(2, 256, 768, 8, 9, model.opt.vocab_size + 1, seed=8)), DEV)
    assert not torch.equal(dt2["video_tensor"], dt["video_tensor"])
    sg.load(dt2)
    sg.replay()
    torch.cuda.synchronize()
    got = {n: (None if p.grad is None else p.grad.detach().clone()) for n, p in model.named_parameters()}
    dt2 = to_device(collate(synthetic_videos(2, 256, 768, 8, 9, model.opt.vocab_size + 1, seed=8)), DEV)
    with bf16_matmul():
        _, ref = _step(model, criterion, dt2)
    for n, r in ref.items():
        assert (r is None) == (got[n] is None), n
        if r is not None:
            err = (got[n] - r).norm().item()
            assert err <= 1e-2 * r.norm().item() + 1e-7, f"replay after load(): grad {n} {err:.3e} vs |ref| {r.norm().item():.3e}"


def _bits(t):
    return t.contiguous().view(torch.int16)


def test_bf16out_entry_points_round_like_torch():
    """The *_bf16out forms of the add-norm and relu-dropout passes write the same fp32 results as the plain
    forms and, beside them, bit for bit torch's bf16 cast of those results (round to nearest even, ties, NaN,
    +-inf, overflow to inf, subnormals)."""
    from pdvc import _native as _n
    from pdvc.ops.functions.ffn import _parts
    g = torch.Generator(device=DEV).manual_seed(3)
    rows, cols = 777, 512
    # relu-dropout forward, p = 0.1 with a device seed
    h = torch.randn(rows, cols, device=DEV, generator=g) * 3
    h.view(-1)[:6] = torch.tensor([1 + 2 ** -8, 1 + 3 * 2 ** -8, 3.3895e38, 1e-40, float("inf"), 2 ** -130],
                                  device=DEV)
    seed = torch.tensor([12345], device=DEV, dtype=torch.int64)
    h_ref, h_got = h.clone(), h.clone()
    h16 = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
    _n.call("pdvc_relu_dropout_forward_f32", _n.ptr(h_ref), rows, cols, 0.1, 0, _n.ptr(seed), _n.stream())
    _n.call("pdvc_relu_dropout_forward_f32_bf16out", _n.ptr(h_got), rows, cols, 0.1, 0, _n.ptr(seed), _n.ptr(h16),
            _n.stream())
    assert torch.equal(h_got, h_ref)
    assert torch.equal(_bits(h16), _bits(h_ref.to(torch.bfloat16))), "relu-dropout forward bf16 rounding"
    # relu-dropout backward with special gradient values where the forward kept the element
    gr = torch.randn(rows, cols, device=DEV, generator=g)
    keep = (h_ref > 0).nonzero()[:8]
    specials = torch.tensor([float("nan"), float("inf"), -float("inf"), 1 + 2 ** -8, -(1 + 3 * 2 ** -8), 3.39e38,
                             -1e-40, 0.0], device=DEV)
    gr[keep[:, 0], keep[:, 1]] = specials / 0.9  # the pass scales by 1 / (1 - p)
    parts = _parts(rows, cols)
    out = []
    for bf in (False, True):
        gg = gr.clone()
        ws = torch.empty(parts * cols, device=DEV)
        db = torch.empty(cols, device=DEV)
        if bf:
            g16 = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
            _n.call("pdvc_relu_dropout_backward_f32_bf16out", _n.ptr(h_ref), _n.ptr(gg), rows, cols, 0.1, parts,
                    _n.ptr(ws), _n.ptr(db), _n.ptr(g16), _n.stream())
        else:
            _n.call("pdvc_relu_dropout_backward_f32", _n.ptr(h_ref), _n.ptr(gg), rows, cols, 0.1, parts, _n.ptr(ws),
                    _n.ptr(db), _n.stream())
        out.append((gg, db))
    assert torch.equal(out[0][0].nan_to_num(7.0), out[1][0].nan_to_num(7.0))
    assert torch.equal(_bits(g16), _bits(out[1][0].to(torch.bfloat16))), "relu-dropout backward bf16 rounding"
    assert (_bits(g16) == 0x7FC0).sum() >= 1  # the NaN made it through as torch's canonical bf16 NaN
    # add-norm forward and backward (dropout p = 0.1 on s)
    d = 512
    x = torch.randn(rows, d, device=DEV, generator=g)
    s = torch.randn(rows, d, device=DEV, generator=g)
    gam = torch.randn(d, device=DEV, generator=g)
    bet = torch.randn(d, device=DEV, generator=g)
    res = []
    for bf in (False, True):
        y = torch.empty(rows, d, device=DEV)
        mean = torch.empty(rows, device=DEV)
        rstd = torch.empty(rows, device=DEV)
        a = (_n.ptr(x), _n.ptr(s), _n.ptr(gam), _n.ptr(bet), rows, d, 0.1, 0, _n.ptr(seed), 1e-5, _n.ptr(y),
             _n.ptr(mean), _n.ptr(rstd))
        if bf:
            y16 = torch.empty(rows, d, device=DEV, dtype=torch.bfloat16)
            _n.call("pdvc_add_dropout_layernorm_forward_f32_bf16out", *a, _n.ptr(y16), _n.stream())
        else:
            _n.call("pdvc_add_dropout_layernorm_forward_f32", *a, _n.stream())
        res.append((y, mean, rstd))
    for u, v in zip(*res):
        assert torch.equal(u, v)
    assert torch.equal(_bits(y16), _bits(res[1][0].to(torch.bfloat16))), "add-norm forward bf16 rounding"
    y, mean, rstd = res[0]
    dy = torch.randn(rows, d, device=DEV, generator=g)
    grads = []
    for bf in (False, True):
        dx, ds = torch.empty_like(x), torch.empty_like(s)
        dgam, dbet, dcol = (torch.empty(d, device=DEV) for _ in range(3))
        ws = torch.empty(3 * 1024 * d, device=DEV)
        a = (_n.ptr(x), _n.ptr(s), _n.ptr(gam), _n.ptr(mean), _n.ptr(rstd), _n.ptr(dy), rows, d, 0.1, 0, _n.ptr(seed),
             _n.ptr(dx), _n.ptr(ds), _n.ptr(dgam), _n.ptr(dbet), _n.ptr(dcol), _n.ptr(ws))
        if bf:
            ds16 = torch.empty(rows, d, device=DEV, dtype=torch.bfloat16)
            _n.call("pdvc_add_dropout_layernorm_backward_f32_bf16out", *a, _n.ptr(ds16), _n.stream())
        else:
            _n.call("pdvc_add_dropout_layernorm_backward_f32", *a, _n.stream())
        grads.append((dx, ds, dgam, dbet, dcol))
    for u, v in zip(*grads):
        assert torch.equal(u, v)
    assert torch.equal(_bits(ds16), _bits(grads[1][1].to(torch.bfloat16))), "add-norm backward bf16 rounding"


def test_logprob_backward_bf16out_rounds_like_torch():
    """pdvc_logprob_pick_backward_f32_bf16out: the same fp32 logit gradient as the plain form and, beside it, torch's
    bf16 cast of it bit for bit (vocabulary 5748, the cfg-2 size); a row form it cannot serve (V % 4 != 0) is refused
    with nothing written."""
    from pdvc import _native as _n
    g = torch.Generator(device=DEV).manual_seed(9)
    rows, V = 333, 5748
    logits = torch.randn(rows, V, device=DEV, generator=g) * 4
    logp = torch.log_softmax(logits, -1).contiguous()
    tgt = torch.randint(0, V, (rows,), device=DEV, generator=g)
    gp = torch.randn(rows, device=DEV, generator=g)
    ref = torch.empty_like(logp)
    got = torch.empty_like(logp)
    g16 = torch.empty(rows, V, device=DEV, dtype=torch.bfloat16)
    _n.call("pdvc_logprob_pick_backward_f32", _n.ptr(logp), _n.ptr(tgt), _n.ptr(gp), rows, V, _n.ptr(ref), _n.stream())
    _n.call("pdvc_logprob_pick_backward_f32_bf16out", _n.ptr(logp), _n.ptr(tgt), _n.ptr(gp), rows, V, _n.ptr(got),
            _n.ptr(g16), _n.stream())
    assert torch.equal(got, ref)
    assert torch.equal(_bits(g16), _bits(ref.to(torch.bfloat16)))
    odd = torch.empty(rows, V - 1, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(_n.NativeError):
        _n.call("pdvc_logprob_pick_backward_f32_bf16out", _n.ptr(logp[:, :-1].contiguous()), _n.ptr(tgt), _n.ptr(gp),
                rows, V - 1, _n.ptr(torch.empty(rows, V - 1, device=DEV)), _n.ptr(odd), _n.stream())


def test_msda_bf16out_rounds_like_torch():
    """The encoder MSDA's bf16 forms (pdvc_msda1d_forward_f32_bf16out / pdvc_msda1d_backward_ex_f32_bf16out, the
    pyramid path at the cfg-2 shape T = 256): the same fp32 output and gradients as the plain forms, and beside them
    torch's bf16 casts of output, grad_value and grad_proj bit for bit; a decoder-shaped call (Lq != S) is refused."""
    from pdvc import _native as _n
    from pdvc.ops.functions.ms_deform_attn_func import NUM_SAMPLES, _levels
    g = torch.Generator(device=DEV).manual_seed(4)
    T_l = (256, 128, 64, 32)
    N, S, M, D = 3, sum(T_l), 8, 64
    lvl, nl = _levels(T_l)
    value = torch.randn(N, S, M, D, device=DEV, generator=g)
    proj = torch.cat([torch.randn(N, S, M * 16, device=DEV, generator=g) * 2,
                      torch.randn(N, S, M * 16, device=DEV, generator=g)], -1).contiguous()
    ref = torch.cat([(torch.arange(t, device=DEV) + 0.5) / t for t in T_l])[None, :, None, None]
    ref = ref.expand(N, S, 4, 1).contiguous()
    C = proj.shape[2]

    def fwd(bf):
        out = torch.empty(N, S, M * D, device=DEV)
        sa = torch.empty(N, M, nl, S, NUM_SAMPLES // nl, device=DEV)
        sl = torch.empty_like(sa)
        a = (_n.ptr(value), None, _n.ptr(proj), C, 0, M * 16, _n.ptr(ref), 1, lvl, nl, N, S, M, D, NUM_SAMPLES // nl,
             _n.ptr(out), _n.ptr(sa), _n.ptr(sl))
        o16 = torch.empty(N, S, M * D, device=DEV, dtype=torch.bfloat16)
        if bf:
            _n.call("pdvc_msda1d_forward_f32_bf16out", *a, _n.ptr(o16), _n.stream())
        else:
            _n.call("pdvc_msda1d_forward_f32", *a, _n.stream())
        return out, sa, sl, o16

    o0, sa, sl, _ = fwd(False)
    o1, sa1, sl1, o16 = fwd(True)
    assert torch.equal(o0, o1) and torch.equal(sa, sa1) and torch.equal(sl, sl1)
    assert torch.equal(_bits(o16), _bits(o0.to(torch.bfloat16)))
    gout = torch.randn(N, S, M * D, device=DEV, generator=g)

    def bwd(bf):
        gv = torch.empty_like(value)
        gp = torch.empty_like(proj)
        a = (_n.ptr(value), None, _n.ptr(ref), 1, _n.ptr(proj), C, 0, M * 16, lvl, nl, N, S, M, D, NUM_SAMPLES // nl,
             _n.ptr(gout), None, _n.ptr(sa), _n.ptr(sl), _n.ptr(gv), _n.ptr(gp), None, None)
        gv16 = torch.empty(gv.shape, device=DEV, dtype=torch.bfloat16)
        gp16 = torch.empty(gp.shape, device=DEV, dtype=torch.bfloat16)
        if bf:
            _n.call("pdvc_msda1d_backward_ex_f32_bf16out", *a, _n.ptr(gv16), _n.ptr(gp16), _n.stream())
        else:
            _n.call("pdvc_msda1d_backward_ex_f32", *a, _n.stream())
        return gv, gp, gv16, gp16

    gv0, gp0, _, _ = bwd(False)
    gv1, gp1, gv16, gp16 = bwd(True)
    assert torch.equal(gp0, gp1) and (gv1 - gv0).abs().max().item() <= 1e-6 * gv0.abs().max().item()
    assert torch.equal(_bits(gv16), _bits(gv1.to(torch.bfloat16)))
    assert torch.equal(_bits(gp16), _bits(gp1.to(torch.bfloat16)))
    out = torch.empty(N, 100, M * D, device=DEV)
    with pytest.raises(_n.NativeError):
        _n.call("pdvc_msda1d_forward_f32_bf16out", _n.ptr(value), None, _n.ptr(proj[:, :100].contiguous()), C, 0,
                M * 16, _n.ptr(ref[:, :100].contiguous()), 1, lvl, nl, N, 100, M, D, NUM_SAMPLES // nl, _n.ptr(out),
                None, None, _n.ptr(torch.empty(N, 100, M * D, device=DEV, dtype=torch.bfloat16)), _n.stream())


def test_cfg2_bf16_step_with_producer_shadows_equals_cast_passes():
    """The bf16 step with the producing kernels writing the bf16 operands (add-norm, relu-dropout) equals the step
    whose every operand is a cast pass as closely as two runs of the cast-pass step equal each other: the same
    bf16 bits reach the same GEMMs (the entry-point test above pins the rounding bit for bit); what differs run to
    run is the summation order of atomic kernels, whose last-ulp fp32 noise can flip the bf16 rounding of a later
    GEMM operand.  Per tensor, max|shadows - casts| <= 4 * (the largest run-to-run difference of any tensor,
    relative to its max|ref|) * max|ref| + 1e-6 * max|ref|; fewer cast passes ran."""
    from pdvc import precision as P
    model, criterion, dt = _cfg2_model_and_batch()
    runs = []
    for shadows in (False, False, True):
        P.SHADOWS[0] = shadows
        P.STATS_CAST[:] = [0, 0, 0]
        try:
            with P.bf16_matmul():
                losses, grads = _step(model, criterion, dt)
        finally:
            P.SHADOWS[0] = True
        runs.append((losses, grads, list(P.STATS_CAST)))
    (l0, g0, c0), (la, ga, _), (l1, g1, c1) = runs
    assert c0[2] == 0 and c1[2] >= 10 and c1[0] <= c0[0] - 10, (c0, c1)

    def rel(a, b):
        return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)
    noise = max([rel(ga[n], r) for n, r in g0.items() if r is not None]
                + [abs(la[k] - l0[k]) / max(abs(l0[k]), 1e-30) for k in l0])
    bound = 4 * noise + 1e-6
    for k in l0:
        assert abs(l1[k] - l0[k]) <= bound * max(abs(l0[k]), 1e-30), f"loss {k}: {l1[k]} vs {l0[k]} (noise {noise:.2e})"
    for n, r in g0.items():
        assert (r is None) == (g1[n] is None), n
        if r is not None:
            assert rel(g1[n], r) <= bound, f"grad {n}: {rel(g1[n], r):.2e} relative, run-to-run noise {noise:.2e}"


def test_msda_bf16out_decoder_grad_value_only():
    """The decoder's cross-attention shape (Lq = 100 queries on a T = 256 pyramid, the dot backward-query kernel):
    pdvc_msda1d_backward_ex_f32_bf16out with grad_proj16 NULL writes grad_value's bf16 rounding bit for bit beside the
    same fp32 gradients as the plain form; asking for grad_proj16 there is refused with nothing launched."""
    from pdvc import _native as _n
    from pdvc.ops.functions.ms_deform_attn_func import NUM_SAMPLES, _levels
    g = torch.Generator(device=DEV).manual_seed(6)
    T_l = (256, 128, 64, 32)
    N, S, M, D, Lq = 3, sum(T_l), 8, 64, 100
    lvl, nl = _levels(T_l)
    value = torch.randn(N, S, M, D, device=DEV, generator=g)
    proj = torch.cat([torch.randn(N, Lq, M * 16, device=DEV, generator=g) * 2,
                      torch.randn(N, Lq, M * 16, device=DEV, generator=g)], -1).contiguous()
    ref = torch.rand(N, Lq, 1, 2, device=DEV, generator=g).expand(N, Lq, 4, 2).contiguous() * 0.8 + 0.1
    C = proj.shape[2]
    out = torch.empty(N, Lq, M * D, device=DEV)
    sa = torch.empty(N, M, nl, Lq, NUM_SAMPLES // nl, device=DEV)
    sl = torch.empty_like(sa)
    _n.call("pdvc_msda1d_forward_f32", _n.ptr(value), None, _n.ptr(proj), C, 0, M * 16, _n.ptr(ref), 2, lvl, nl, N, Lq,
            M, D, NUM_SAMPLES // nl, _n.ptr(out), _n.ptr(sa), _n.ptr(sl), _n.stream())
    gout = torch.randn(N, Lq, M * D, device=DEV, generator=g)

    def bwd(bf, gp16=None):
        gv = torch.empty_like(value)
        gp = torch.empty_like(proj)
        a = (_n.ptr(value), None, _n.ptr(ref), 2, _n.ptr(proj), C, 0, M * 16, lvl, nl, N, Lq, M, D, NUM_SAMPLES // nl,
             _n.ptr(gout), None, _n.ptr(sa), _n.ptr(sl), _n.ptr(gv), _n.ptr(gp), None, None)
        gv16 = torch.empty(gv.shape, device=DEV, dtype=torch.bfloat16)
        if bf:
            _n.call("pdvc_msda1d_backward_ex_f32_bf16out", *a, _n.ptr(gv16), _n.ptr(gp16), _n.stream())
        else:
            _n.call("pdvc_msda1d_backward_ex_f32", *a, _n.stream())
        return gv, gp, gv16

    gv0, gp0, _ = bwd(False)
    gv1, gp1, gv16 = bwd(True)
    assert (gv1 - gv0).abs().max().item() <= 1e-6 * gv0.abs().max().item()
    assert (gp1 - gp0).abs().max().item() <= 1e-5 * gp0.abs().max().item()
    assert torch.equal(_bits(gv16), _bits(gv1.to(torch.bfloat16)))
    with pytest.raises(_n.NativeError):
        bwd(True, torch.empty(proj.shape, device=DEV, dtype=torch.bfloat16))


@pytest.mark.parametrize("T", [256, 600])
def test_base_encoder_flat_buffer_bf16_shadow(T):
    """bf16 mode: the base encoder's levels write their bf16 rounding beside the flattened (N, sum T_l, d) buffer (the
    single-pass GroupNorm's y16; T = 600 puts level 0 on the chunked forms, whose slice is rounded by a cast) and the
    finished buffer carries it as its cached rounding: torch's bf16 cast of the buffer, bit for bit."""
    from pdvc.base_encoder import BaseEncoder
    from pdvc.precision import bf16_matmul
    torch.manual_seed(T)
    enc = BaseEncoder(4, 768, 512).to(DEV)
    N = 3
    vf = torch.randn(N, T, 768, device=DEV)
    mask = torch.zeros(N, T, dtype=torch.bool, device=DEV)
    dur = torch.tensor([100.0, 37.0, 12.0], device=DEV)
    with bf16_matmul():
        srcs, _, _ = enc(vf, mask, dur)
    flat = srcs[0]._pdvc_flat[0]
    ent = flat.__dict__.get("_pdvc_bf16")
    assert ent is not None and ent[0] == flat._version
    assert torch.equal(_bits(ent[1]), _bits(flat.to(torch.bfloat16)))
