"""GPU parity of the HIP operators against the CPU oracle (oracle/msda_oracle.c) and the golden vectors
generated from the reference (tests/golden).  Tolerances: fp64 1e-10, fp32 1e-4 (north star: 1e-4 fp32).
"""
import os

import numpy as np
import pytest
import torch
from parity import assert_close

from oracle import oracle as O

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def load(name):
    return np.load(os.path.join(G, name + ".npz"), allow_pickle=False)


def cu(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV)


def close(a, b, tol, what=""):
    """Per-tensor relative bound: max|a - b| <= tol * max|b| + 1e-7 (tests/parity.py)."""
    assert_close(a, b, what, tol)


# ------------------------------------------------------------------------------------------------
# drop-in operator MultiScaleDeformableAttention (pdvc/ops/src/vision.cpp:13-16)
# ------------------------------------------------------------------------------------------------
def test_dropin_reftest_inputs_f64():
    """The reference test's own inputs (pdvc/ops/test.py:21-44), fp64, vs the zeros golden vectors."""
    import MultiScaleDeformableAttention as MSDA
    d = load("op_reftest")
    v, lo, a = cu(d["value"]), cu(d["loc"]), cu(d["attn"])
    shapes, lsi = cu(d["shapes"]), cu(d["lsi"])
    out = MSDA.ms_deform_attn_forward(v, shapes, lsi, lo, a, 2)
    close(out, d["zeros_out"], 1e-12, "fwd")
    gv, gl, ga = MSDA.ms_deform_attn_backward(v, shapes, lsi, lo, a, cu(d["grad_out"]), 2)
    close(gv, d["zeros_grad_value"], 1e-12, "grad_value")
    close(gl, d["zeros_grad_loc"], 1e-12, "grad_loc")
    close(ga, d["zeros_grad_attn"], 1e-12, "grad_attn")


@pytest.mark.parametrize("D", [30, 32, 64, 71])
@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_dropin_1d_pyramids(D, dt):
    import MultiScaleDeformableAttention as MSDA
    d = load(f"op_1d_D{D}")
    tdt = torch.float64 if dt == "f64" else torch.float32
    tol = 1e-10 if dt == "f64" else 1e-4
    v, lo, a = cu(d["value"], tdt), cu(d["loc"], tdt), cu(d["attn"], tdt)
    shapes, lsi = cu(d["shapes"]), cu(d["lsi"])
    out = MSDA.ms_deform_attn_forward(v, shapes, lsi, lo, a, 64)
    close(out, d[f"zeros_{dt}_out"], tol, "fwd")
    gv, gl, ga = MSDA.ms_deform_attn_backward(v, shapes, lsi, lo, a, cu(d["grad_out"], tdt), 64)
    close(gv, d[f"zeros_{dt}_grad_value"], tol, "grad_value")
    close(gl, d[f"zeros_{dt}_grad_loc"], tol, "grad_loc")
    close(ga, d[f"zeros_{dt}_grad_attn"], tol, "grad_attn")


@pytest.mark.parametrize("channels", [30, 32, 64, 71, 1025, 2048, 3096])
def test_dropin_gradient_channels_vs_oracle(channels):
    """Every channel count of the reference gradcheck (test.py:85), fp64, against the oracle."""
    import MultiScaleDeformableAttention as MSDA
    rng = np.random.RandomState(channels)
    shapes = np.array([(6, 4), (3, 2)], np.int64)
    lsi = np.array([0, 24], np.int64)
    N, M, Lq, L, P = 1, 2, 2, 2, 2
    v = rng.rand(N, 30, M, channels) * 0.01
    lo = rng.rand(N, Lq, M, L, P, 2)
    a = rng.rand(N, Lq, M, L, P) + 1e-5
    a /= a.sum(-1, keepdims=True).sum(-2, keepdims=True)
    g = rng.randn(N, Lq, M * channels)
    ev = O.msda_forward(v, shapes, lsi, lo, a, "zeros")
    egv, egl, ega = O.msda_backward(v, shapes, lsi, lo, a, g, "zeros")
    out = MSDA.ms_deform_attn_forward(cu(v), cu(shapes), cu(lsi), cu(lo), cu(a), 2)
    gv, gl, ga = MSDA.ms_deform_attn_backward(cu(v), cu(shapes), cu(lsi), cu(lo), cu(a), cu(g), 2)
    close(out, ev, 1e-12, "fwd")
    close(gv, egv, 1e-12, "grad_value")
    close(gl, egl, 1e-11, "grad_loc")
    close(ga, ega, 1e-11, "grad_attn")


def _lifted_inputs(rng, N, M, T_l, Lq, D=64, P=4, y_mode="half"):
    """Drop-in op inputs on PDVC's lifted pyramid (spatial_shapes [[1, T_l]], ms_deform_attn.py:114-117): x over the
    levels and past both ends, kept off cell edges (the location gradient steps there); y = 0.5 as PDVC passes it,
    or (y_mode "mixed") a quarter of the samples at other heights -- inside (-0.5, 1.5), off the kinks at y = 0.5
    and at the ends, and a few outside."""
    L = len(T_l)
    S = sum(T_l)
    shapes = np.array([(1, t) for t in T_l], np.int64)
    lsi = np.concatenate([[0], np.cumsum(T_l)[:-1]]).astype(np.int64)
    value = rng.randn(N, S, M, D)
    Tn = np.asarray(T_l, np.float64)[None, None, None, :, None]
    x = rng.uniform(-0.05, 1.05, size=(N, Lq, M, L, P))
    u = x * Tn - 0.5
    frac = u - np.floor(u)
    u = np.where(np.minimum(frac, 1 - frac) < 2e-3, u + 5e-3, u)
    x = (u + 0.5) / Tn
    y = np.full_like(x, 0.5)
    if y_mode == "mixed":
        pick = rng.rand(*x.shape) < 0.25
        h = rng.uniform(-0.97, 0.97, size=x.shape)
        h = np.where(np.abs(h) < 2e-3, 0.1, h)
        out = rng.rand(*x.shape) < 0.05
        h = np.where(out, rng.choice([-1.3, 1.2], size=x.shape), h)
        y = np.where(pick, h + 0.5, y)
    loc = np.stack([x, y], -1)
    attn = rng.rand(N, Lq, M, L, P) + 1e-3
    attn /= attn.sum((-1, -2), keepdims=True)
    gout = rng.randn(N, Lq, M * D)
    return value, shapes, lsi, loc, attn, gout


@pytest.mark.parametrize("Lq,y_mode", [(960, "half"), (100, "half"), (960, "mixed"), (100, "mixed")])
def test_dropin_fast_path_full_size_vs_oracle(Lq, y_mode):
    """The drop-in operator on PDVC's full lifted pyramid (T = 512: S = 960; the encoder's Lq = S and the decoder's
    Lq = 100, M = 8, D = 64, fp32) -- the shapes a stock MSDeformAttn module hands the extension.  The library takes
    its 1-D fast path (device-side check of the level table, atomic-free value gradient) and must equal the oracle's
    zero-padding CUDA semantics, y at 0.5 and at other heights in the cell."""
    import MultiScaleDeformableAttention as MSDA
    rng = np.random.RandomState(Lq + len(y_mode))
    T_l = [512, 256, 128, 64]
    N, M = 2, 8
    value, shapes, lsi, loc, attn, gout = _lifted_inputs(rng, N, M, T_l, Lq, y_mode=y_mode)
    ev = O.msda_forward(value, shapes, lsi, loc, attn, "zeros")
    egv, egl, ega = O.msda_backward(value, shapes, lsi, loc, attn, gout, "zeros")
    f32 = torch.float32
    v, lo, a = cu(value, f32), cu(loc, f32), cu(attn, f32)
    out = MSDA.ms_deform_attn_forward(v, cu(shapes), cu(lsi), lo, a, 64)
    close(out, ev, 1e-4, "fwd")
    gv, gl, ga = MSDA.ms_deform_attn_backward(v, cu(shapes), cu(lsi), lo, a, cu(gout, f32), 64)
    close(gv, egv, 1e-4, "grad_value")
    close(gl[..., 0], egl[..., 0], 1e-4, "grad_loc x")
    close(gl[..., 1], egl[..., 1], 1e-4, "grad_loc y")
    close(ga, ega, 1e-4, "grad_attn")


@pytest.mark.parametrize("T_l,Lq,y_mode,N", [
    ([256, 128, 64, 32], 480, "half", 2),     # yc2's encoder: whole-pyramid kernels, one staging phase, no fallback
    ([256, 128, 64, 32], 480, "mixed", 2),
    ([512, 256, 128, 64], 1200, "mixed", 2),  # more queries than positions: 3 forward / 2 backward query blocks
    ([512, 256, 128, 64], 240, "half", 2),    # 4 Lq == S: the smallest call the pyramid form takes, a partial block
    ([600, 300, 150, 75], 1125, "half", 4),   # level 0 longer than a staging phase: the gather kernels take the call,
                                              # grid-strided (9 024 waves over 2 048 workgroups)
    ([400, 300, 200, 100], 1000, "mixed", 2),  # levels 1..3 longer than a staging phase: likewise, one pass
])
def test_dropin_pyramid_form_vs_oracle(T_l, Lq, y_mode, N):
    """Encoder-shaped drop-in calls (4 Lq >= S) run on the whole-pyramid kernels (msda_dropin_fwd_pyr_kernel,
    msda_dropin_bwd_query_pyr_kernel) when both staging phases fit 512 rows -- decided on the device from the level
    table -- and on the L2-gather kernels launched after them otherwise; every case must equal the oracle."""
    import MultiScaleDeformableAttention as MSDA
    rng = np.random.RandomState(Lq + sum(T_l) + len(y_mode))
    M = 8
    value, shapes, lsi, loc, attn, gout = _lifted_inputs(rng, N, M, T_l, Lq, y_mode=y_mode)
    ev = O.msda_forward(value, shapes, lsi, loc, attn, "zeros")
    egv, egl, ega = O.msda_backward(value, shapes, lsi, loc, attn, gout, "zeros")
    f32 = torch.float32
    v, lo, a = cu(value, f32), cu(loc, f32), cu(attn, f32)
    out = MSDA.ms_deform_attn_forward(v, cu(shapes), cu(lsi), lo, a, 64)
    close(out, ev, 1e-4, "fwd")
    gv, gl, ga = MSDA.ms_deform_attn_backward(v, cu(shapes), cu(lsi), lo, a, cu(gout, f32), 64)
    close(gv, egv, 1e-4, "grad_value")
    close(gl[..., 0], egl[..., 0], 1e-4, "grad_loc x")
    close(gl[..., 1], egl[..., 1], 1e-4, "grad_loc y")
    close(ga, ega, 1e-4, "grad_attn")


def test_dropin_fast_path_leaves_2d_tables_to_the_general_kernels():
    """A 2-D table of the same sizes (4 levels x 4 points, D = 64) and a 1-D table whose start index is not the prefix
    sum of its lengths: both must take the general kernels (the fast path's device check refuses them) and still
    equal the oracle."""
    import MultiScaleDeformableAttention as MSDA
    rng = np.random.RandomState(5)
    N, M, Lq, D = 2, 2, 37, 64
    for shapes, lsi in ((np.array([(2, 16), (2, 8), (1, 8), (2, 2)], np.int64), np.array([0, 32, 48, 56], np.int64)),
                        (np.array([(1, 16), (1, 8), (1, 8), (1, 4)], np.int64), np.array([0, 16, 20, 28], np.int64))):
        S = 60
        value = rng.randn(N, S, M, D)
        loc = rng.uniform(-0.1, 1.1, size=(N, Lq, M, 4, 4, 2))
        attn = rng.rand(N, Lq, M, 4, 4)
        gout = rng.randn(N, Lq, M * D)
        ev = O.msda_forward(value, shapes, lsi, loc, attn, "zeros")
        egv, egl, ega = O.msda_backward(value, shapes, lsi, loc, attn, gout, "zeros")
        f32 = torch.float32
        v, lo, a = cu(value, f32), cu(loc, f32), cu(attn, f32)
        out = MSDA.ms_deform_attn_forward(v, cu(shapes), cu(lsi), lo, a, 64)
        close(out, ev, 1e-4, "fwd")
        gv, gl, ga = MSDA.ms_deform_attn_backward(v, cu(shapes), cu(lsi), lo, a, cu(gout, f32), 64)
        close(gv, egv, 1e-4, "grad_value")
        close(ga, ega, 1e-4, "grad_attn")


def test_dropin_autograd_gradcheck():
    """torch.autograd.gradcheck through MSDeformAttnFunction (test.py:63-78), fp64."""
    from pdvc.ops.functions import MSDeformAttnFunction
    torch.manual_seed(3)
    shapes = torch.as_tensor([(6, 4), (3, 2)], dtype=torch.long, device=DEV)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    value = (torch.rand(1, 30, 2, 4, device=DEV, dtype=torch.float64) * 0.01).requires_grad_()
    loc = torch.rand(1, 2, 2, 2, 2, 2, device=DEV, dtype=torch.float64).requires_grad_()
    attn = torch.rand(1, 2, 2, 2, 2, device=DEV, dtype=torch.float64) + 1e-5
    attn = (attn / attn.sum(-1, keepdim=True).sum(-2, keepdim=True)).requires_grad_()
    assert torch.autograd.gradcheck(MSDeformAttnFunction.apply, (value, shapes, lsi, loc, attn, 2))


def test_dropin_errors():
    import MultiScaleDeformableAttention as MSDA
    d = load("op_reftest")
    v, lo, a = cu(d["value"]), cu(d["loc"]), cu(d["attn"])
    shapes, lsi = cu(d["shapes"]), cu(d["lsi"])
    v3 = torch.cat([v, v, v], 0)
    lo3, a3 = torch.cat([lo] * 3, 0), torch.cat([a] * 3, 0)
    with pytest.raises(RuntimeError, match="im2col_step"):
        MSDA.ms_deform_attn_forward(v3, shapes, lsi, lo3, a3, 2)  # 3 % min(3,2) != 0
    with pytest.raises(RuntimeError):
        MSDA.ms_deform_attn_forward(v.cpu(), shapes, lsi, lo, a, 2)
    with pytest.raises(RuntimeError):
        MSDA.ms_deform_attn_forward(v.transpose(1, 2), shapes, lsi, lo, a, 2)
    # dtypes the reference's data<int64_t>() / data<scalar_t>() accessors reject
    with pytest.raises(RuntimeError, match="int64"):
        MSDA.ms_deform_attn_forward(v, shapes.int(), lsi, lo, a, 2)
    with pytest.raises(RuntimeError, match="int64"):
        MSDA.ms_deform_attn_forward(v, shapes, lsi.int(), lo, a, 2)
    with pytest.raises(RuntimeError, match="sampling_loc"):
        MSDA.ms_deform_attn_forward(v, shapes, lsi, lo.float(), a, 2)
    with pytest.raises(RuntimeError, match="attn_weight"):
        MSDA.ms_deform_attn_forward(v.float(), shapes, lsi, lo.float(), a, 2)
    g = torch.zeros(1, 2, 4, dtype=torch.float32, device=DEV)
    with pytest.raises(RuntimeError, match="grad_output"):
        MSDA.ms_deform_attn_backward(v, shapes, lsi, lo, a, g, 2)
    # shapes inconsistent with value / sampling_loc
    with pytest.raises(RuntimeError, match="spatial_shapes"):
        MSDA.ms_deform_attn_forward(v, shapes.reshape(-1), lsi, lo, a, 2)
    with pytest.raises(RuntimeError, match="attn_weight"):
        MSDA.ms_deform_attn_forward(v, shapes, lsi, lo, a[..., :1].contiguous(), 2)
    with pytest.raises(RuntimeError, match="grad_output"):
        MSDA.ms_deform_attn_backward(v, shapes, lsi, lo, a, g.double()[..., :3].contiguous(), 2)


def test_dropin_malformed_level_table_reads_nothing_outside_value():
    """A level table pointing past the value rows (the host cannot see device-resident shapes without a sync;
    the reference reads out of bounds) drops that level: no fault, no read outside value."""
    import MultiScaleDeformableAttention as MSDA
    d = load("op_reftest")
    v, lo, a = cu(d["value"]), cu(d["loc"]), cu(d["attn"])
    shapes, lsi = cu(d["shapes"]), cu(d["lsi"])
    bad = lsi.clone()
    bad[1] = 10 ** 9
    out = MSDA.ms_deform_attn_forward(v, shapes, bad, lo, a, 2)
    only0 = a.clone()
    only0[:, :, :, 1] = 0
    ref = MSDA.ms_deform_attn_forward(v, shapes, lsi, lo, only0, 2)
    torch.cuda.synchronize()
    close(out, ref, 1e-12, "level 1 dropped")
    gv, gl, ga = MSDA.ms_deform_attn_backward(v, shapes, bad, lo, a, out, 2)
    torch.cuda.synchronize()
    assert torch.isfinite(gv).all() and torch.count_nonzero(ga[:, :, :, 1]) == 0


def test_dropin_empty_queries():
    import MultiScaleDeformableAttention as MSDA
    d = load("op_reftest")
    v = cu(d["value"])
    shapes, lsi = cu(d["shapes"]), cu(d["lsi"])
    lo = torch.zeros(1, 0, 2, 2, 2, 2, dtype=v.dtype, device=DEV)
    a = torch.zeros(1, 0, 2, 2, 2, dtype=v.dtype, device=DEV)
    out = MSDA.ms_deform_attn_forward(v, shapes, lsi, lo, a, 64)
    assert out.shape == (1, 0, 4)
    gv, gl, ga = MSDA.ms_deform_attn_backward(v, shapes, lsi, lo, a, out, 64)
    assert torch.count_nonzero(gv) == 0


# ------------------------------------------------------------------------------------------------
# border raw-sample core (ms_deform_attn_core_pytorch, return_value=True)
# ------------------------------------------------------------------------------------------------
def test_core_border_samples_vs_golden():
    from pdvc.ops.functions import ms_deform_attn_core_pytorch
    d = load("op_sample")
    v = cu(d["value"], torch.float32).requires_grad_()
    lo = cu(d["loc"], torch.float32).requires_grad_()
    s = ms_deform_attn_core_pytorch(v, cu(d["shapes"]), lo, None, return_value=True)
    close(s, d["f32_samples"], 1e-5, "samples")
    s.backward(cu(d["grad_samples"], torch.float32))
    close(v.grad, d["f32_grad_value"], 1e-4, "grad_value")
    close(lo.grad, d["f32_grad_loc"], 1e-4, "grad_loc")


@pytest.mark.parametrize("D", [30, 64])
def test_core_border_weighted_vs_golden(D):
    from pdvc.ops.functions import ms_deform_attn_core_pytorch
    d = load(f"op_1d_D{D}")
    v = cu(d["value"], torch.float32).requires_grad_()
    lo = cu(d["loc"], torch.float32).requires_grad_()
    a = cu(d["attn"], torch.float32).requires_grad_()
    out = ms_deform_attn_core_pytorch(v, cu(d["shapes"]), lo, a)
    close(out, d["border_f32_out"], 1e-4, "out")
    out.backward(cu(d["grad_out"], torch.float32))
    close(v.grad, d["border_f32_grad_value"], 1e-4, "grad_value")
    close(lo.grad, d["border_f32_grad_loc"], 1e-4, "grad_loc")
    close(a.grad, d["border_f32_grad_attn"], 1e-4, "grad_attn")


# ------------------------------------------------------------------------------------------------
# fused 1-D kernels vs the oracle + the module math restated in numpy (ms_deform_attn.py:163-192)
# ------------------------------------------------------------------------------------------------
def _softmax(x):
    e = np.exp(x - x.max(-1, keepdims=True))
    return e / e.sum(-1, keepdims=True)


def expected_msda1d(value, mask, proj, ref, T_l, M, grad_out):
    """numpy/oracle restatement (float64) of the fused forward and its gradients."""
    N, S, _, D = value.shape
    Lq = proj.shape[1]
    L, P = len(T_l), 4
    NS = L * P
    off = proj[..., :M * NS].reshape(N, Lq, M, L, P)
    logit = proj[..., M * NS:2 * M * NS].reshape(N, Lq, M, NS)
    a = _softmax(logit).reshape(N, Lq, M, L, P)
    Tn = np.asarray(T_l, np.float64)[None, None, None, :, None]
    if ref.shape[-1] == 1:
        loc = ref[:, :, None, :, None, 0] + off / Tn
    else:
        loc = ref[:, :, None, :, None, 0] + off / P * ref[:, :, None, :, None, 1] * 0.5
    v = value * (~mask)[..., None, None] if mask is not None else value
    loc2, shapes, lsi = O.lift_1d(loc, T_l)
    out = O.msda_forward(v, shapes, lsi, loc2, a, "zeros")
    gv, gl, ga = O.msda_backward(v, shapes, lsi, loc2, a, grad_out, "zeros")
    if mask is not None:
        gv = gv * (~mask)[..., None, None]
    glx = gl[..., 0]
    ga_flat = ga.reshape(N, Lq, M, NS)
    a_flat = a.reshape(N, Lq, M, NS)
    glogit = a_flat * (ga_flat - (a_flat * ga_flat).sum(-1, keepdims=True))
    if ref.shape[-1] == 1:
        goff = glx / Tn
        gref = glx.sum(axis=(2, 4))[..., None]
    else:
        goff = glx * 0.5 * ref[:, :, None, :, None, 1] / P
        gc = glx.sum(axis=(2, 4))
        gln = (glx * 0.5 * off / P).sum(axis=(2, 4))
        gref = np.stack([gc, gln], -1)
    gproj = np.concatenate([goff.reshape(N, Lq, M * NS), glogit.reshape(N, Lq, M * NS)], -1)
    return out, gv, gproj, gref


@pytest.mark.parametrize("D", [16, 32, 64, 128])
@pytest.mark.parametrize("ref_dim", [1, 2])
@pytest.mark.parametrize("masked", [False, True])
def test_fused_msda1d_vs_oracle(D, ref_dim, masked):
    from pdvc.ops.functions import MSDA1dFunction
    rng = np.random.RandomState(D * 10 + ref_dim + 100 * masked)
    M = {16: 8, 32: 4, 64: 8, 128: 3}[D]
    T_l = [40, 20, 10, 5]
    N, Lq, S = 2, 37, sum(T_l)
    value = rng.randn(N, S, M, D)
    proj = np.concatenate([rng.randn(N, Lq, M * 16) * 3.0, rng.randn(N, Lq, M * 16)], -1)
    if ref_dim == 1:
        ref = rng.uniform(-0.05, 1.05, size=(N, Lq, 4, 1))
    else:
        ref = np.concatenate([rng.uniform(0, 1, size=(N, Lq, 4, 1)), rng.uniform(0.05, 0.9, size=(N, Lq, 4, 1))], -1)
    mask = None
    if masked:
        mask = np.zeros((N, S), bool)
        mask[1, 30:40] = True
        mask[1, 55:60] = True
    gout = rng.randn(N, Lq, M * D)
    eo, egv, egp, egr = expected_msda1d(value, mask, proj, ref, T_l, M, gout)
    v = cu(value, torch.float32).requires_grad_()
    p = cu(proj, torch.float32).requires_grad_()
    r = cu(ref, torch.float32).requires_grad_()
    mk = None if mask is None else cu(mask).view(torch.uint8)
    out = MSDA1dFunction.apply(v, mk, p, r, tuple(T_l), 0, M * 16)
    close(out, eo, 1e-4, "out")
    out.backward(cu(gout, torch.float32))
    close(v.grad, egv, 1e-4, "grad_value")
    close(p.grad, egp, 1e-4, "grad_proj")
    close(r.grad, egr, 1e-4, "grad_ref")


def test_fused_msda1d_pdvc_shape_vs_oracle():
    """PDVC encoder shape at T=128 (M=8, D=64, S=240, Lq=S), one video."""
    from pdvc.ops.functions import MSDA1dFunction
    rng = np.random.RandomState(1)
    T_l = [128, 64, 32, 16]
    S = sum(T_l)
    M, D, N, Lq = 8, 64, 1, S
    value = rng.randn(N, S, M, D).astype(np.float32)
    proj = np.concatenate([rng.randn(N, Lq, M * 16) * 2, rng.randn(N, Lq, M * 16)], -1).astype(np.float32)
    ref = np.concatenate([(np.arange(t) + 0.5) / t for t in T_l])[None, :, None, None].repeat(4, 2).astype(np.float32)
    gout = rng.randn(N, Lq, M * D).astype(np.float32)
    eo, egv, egp, egr = expected_msda1d(value.astype(np.float64), None, proj.astype(np.float64),
                                        ref.astype(np.float64), T_l, M, gout.astype(np.float64))
    v, p = cu(value).requires_grad_(), cu(proj).requires_grad_()
    out = MSDA1dFunction.apply(v, None, p, cu(ref), tuple(T_l), 0, M * 16)
    close(out, eo, 1e-4, "out")
    out.backward(cu(gout))
    close(v.grad, egv, 1e-4, "grad_value")
    close(p.grad, egp, 1e-4, "grad_proj")


@pytest.mark.parametrize("ref_dim", [1, 2])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("offset_scale", [2.0, 60.0])
def test_fused_msda1d_pyramid_vs_oracle(ref_dim, masked, offset_scale):
    """Self-attention over the pyramid (Lq == S, D = 64) takes the whole-pyramid forward (pick_pyr in
    msda1d.hip: the head's value rows staged in LDS); offset_scale 60 scatters samples over whole levels and
    past both ends (clamped corners, zero padding)."""
    from pdvc.ops.functions import MSDA1dFunction
    rng = np.random.RandomState(7 + ref_dim + 10 * masked + int(offset_scale))
    T_l = [96, 48, 24, 12]
    S = sum(T_l)
    M, D, N, Lq = 4, 64, 3, S
    value = rng.randn(N, S, M, D)
    proj = np.concatenate([rng.randn(N, Lq, M * 16) * offset_scale, rng.randn(N, Lq, M * 16)], -1)
    centre = np.concatenate([(np.arange(t) + 0.5) / t for t in T_l])[None, :, None, None].repeat(4, 2)
    centre = np.repeat(centre, N, 0)
    if ref_dim == 1:
        ref = centre
    else:
        ref = np.concatenate([centre, rng.uniform(0.05, 0.5, size=(N, Lq, 4, 1))], -1)
    mask = None
    if masked:
        mask = np.zeros((N, S), bool)
        mask[1, 80:96] = True
        mask[1, 136:144] = True
        mask[2, 170:] = True
    gout = rng.randn(N, Lq, M * D)
    eo, egv, egp, egr = expected_msda1d(value, mask, proj, ref, T_l, M, gout)
    v = cu(value, torch.float32).requires_grad_()
    p = cu(proj, torch.float32).requires_grad_()
    r = cu(ref, torch.float32).requires_grad_()
    mk = None if mask is None else cu(mask).view(torch.uint8)
    out = MSDA1dFunction.apply(v, mk, p, r, tuple(T_l), 0, M * 16)
    close(out, eo, 1e-4, "out")
    out.backward(cu(gout, torch.float32))
    close(v.grad, egv, 1e-4, "grad_value")
    close(p.grad, egp, 1e-4, "grad_proj")
    close(r.grad, egr, 1e-4, "grad_ref")


@pytest.mark.parametrize("offset_scale,ref_dim", [(1.0, 1), (300.0, 1), (300.0, 2)])
def test_fused_msda1d_windowed_full_size_vs_oracle(offset_scale, ref_dim):
    """PDVC's full pyramid (T = 512: S = 960, two 512-query blocks of the whole-pyramid forward): offsets of
    about one cell, and of hundreds of cells (samples over whole levels and past both ends)."""
    from pdvc.ops.functions import MSDA1dFunction
    rng = np.random.RandomState(int(offset_scale) + ref_dim)
    T_l = [512, 256, 128, 64]
    S = sum(T_l)
    M, D, N, Lq = 2, 64, 1, S
    value = rng.randn(N, S, M, D)
    proj = np.concatenate([rng.randn(N, Lq, M * 16) * offset_scale, rng.randn(N, Lq, M * 16)], -1)
    centre = np.concatenate([(np.arange(t) + 0.5) / t for t in T_l])[None, :, None, None].repeat(4, 2)
    ref = centre if ref_dim == 1 else np.concatenate([centre, rng.uniform(0.05, 0.5, size=(N, Lq, 4, 1))], -1)
    gout = rng.randn(N, Lq, M * D)
    eo, egv, egp, _ = expected_msda1d(value, None, proj, ref, T_l, M, gout)
    v = cu(value, torch.float32).requires_grad_()
    p = cu(proj, torch.float32).requires_grad_()
    out = MSDA1dFunction.apply(v, None, p, cu(ref, torch.float32), tuple(T_l), 0, M * 16)
    close(out, eo, 1e-4, "out")
    out.backward(cu(gout, torch.float32))
    close(v.grad, egv, 1e-4, "grad_value")
    close(p.grad, egp, 1e-4, "grad_proj")


@pytest.mark.parametrize("ref_dim", [1, 2])
def test_fused_msda1d_headline_encoder_backward_vs_oracle(ref_dim):
    """The headline encoder call (T = 512: S = Lq = 960, M = 8, D = 64) over two videos with padded tails (the
    whole-pyramid forward and backward-query kernels, the value gradient's counting sort and walk over 960 queries)
    against the float64 oracle; masked rows get a zero gradient."""
    from pdvc.ops.functions import MSDA1dFunction
    rng = np.random.RandomState(50 + ref_dim)
    T_l = [512, 256, 128, 64]
    S = sum(T_l)
    M, D, N, Lq = 8, 64, 2, S
    value = rng.randn(N, S, M, D)
    proj = np.concatenate([rng.randn(N, Lq, M * 16) * 3.0, rng.randn(N, Lq, M * 16)], -1)
    centre = np.concatenate([(np.arange(t) + 0.5) / t for t in T_l])[None, :, None, None].repeat(4, 2)
    centre = np.repeat(centre, N, 0)
    ref = centre if ref_dim == 1 else np.concatenate([centre, rng.uniform(0.05, 0.5, size=(N, Lq, 4, 1))], -1)
    proj = _away_from_cell_edges(proj, ref, T_l, M)
    mask = np.zeros((N, S), bool)
    mask[1, 400:512] = True
    mask[1, 700:768] = True
    mask[0, 950:960] = True
    gout = rng.randn(N, Lq, M * D)
    eo, egv, egp, egr = expected_msda1d(value, mask, proj, ref, T_l, M, gout)
    v = cu(value, torch.float32).requires_grad_()
    p = cu(proj, torch.float32).requires_grad_()
    r = cu(ref, torch.float32).requires_grad_()
    out = MSDA1dFunction.apply(v, cu(mask).view(torch.uint8), p, r, tuple(T_l), 0, M * 16)
    close(out, eo, 1e-4, "out")
    out.backward(cu(gout, torch.float32))
    close(v.grad, egv, 1e-4, "grad_value")
    close(p.grad, egp, 1e-4, "grad_proj")
    close(r.grad, egr, 1e-4, "grad_ref")
    assert float(v.grad[1, 400:512].abs().max()) == 0.0


def _away_from_cell_edges(proj, ref, T_l, M, margin=2e-3):
    """Nudge the sampling offsets so that no sample's x = loc * T - 0.5 lies within `margin` of an integer: the
    location gradient T * a * (v[x0 + 1] - v[x0]) . g is a step function of x, so at T = 1024 an fp32 location a few
    ulps from a cell edge can take the neighbouring cell where the float64 expectation does not (the reference's
    fp32 CUDA op has the same step) -- a property of the comparison, not of the kernels."""
    P = 4
    N, Lq = proj.shape[:2]
    off = proj[..., :M * 16].reshape(N, Lq, M, len(T_l), P)
    Tn = np.asarray(T_l, np.float64)[None, None, None, :, None]
    r0 = ref[:, :, None, :, None, 0]
    if ref.shape[-1] == 1:
        x = (r0 + off / Tn) * Tn - 0.5
        dxdoff = np.ones_like(x)
    else:
        r1 = ref[:, :, None, :, None, 1]
        x = (r0 + off / P * r1 * 0.5) * Tn - 0.5
        dxdoff = r1 * 0.5 / P * Tn * np.ones_like(x)
    frac = x - np.floor(x)
    near = np.minimum(frac, 1.0 - frac) < margin
    off = off + near * (4 * margin) / dxdoff
    out = proj.copy()
    out[..., :M * 16] = off.reshape(N, Lq, M * 16)
    return out


@pytest.mark.parametrize("T_l,ref_dim,M", [((1024, 512, 256, 128), 1, 2), ((1024, 512, 256, 128), 2, 2),
                                           ((1024, 512, 256, 128), 1, 8), ((1024, 512, 256, 128), 2, 8),
                                           ((700, 512, 256, 200), 1, 8),
                                           ((512, 300, 150, 60), 1, 2), ((512, 300, 150, 60), 2, 2)])
def test_fused_msda1d_long_pyramids_vs_oracle(T_l, ref_dim, M):
    """Long pyramids: anet_c3d's T = 1024 (S = 1920: level 0 past one LDS staging phase, so the forward runs the
    windowed pyramid kernel -- level 0 in two row windows, msda1d_fwd_win_kernel -- and the backward-query the
    dot-product kernel at Lq = S; the value gradient takes two query chunks, the second accumulating into the rows the
    first wrote), a level 0 of 700 rows (second window shorter than the first), and S = 1022 (both pyramid kernels with
    two query blocks).  M = 8 is the headline's head count."""
    from pdvc.ops.functions import MSDA1dFunction
    rng = np.random.RandomState(sum(T_l) + ref_dim + M)
    S = sum(T_l)
    D, N, Lq = 64, 1, S
    value = rng.randn(N, S, M, D)
    proj = np.concatenate([rng.randn(N, Lq, M * 16) * 4.0, rng.randn(N, Lq, M * 16)], -1)
    centre = np.concatenate([(np.arange(t) + 0.5) / t for t in T_l])[None, :, None, None].repeat(4, 2)
    ref = centre if ref_dim == 1 else np.concatenate([centre, rng.uniform(0.05, 0.5, size=(N, Lq, 4, 1))], -1)
    proj = _away_from_cell_edges(proj, ref, T_l, M)
    mask = np.zeros((N, S), bool)
    mask[0, T_l[0] - 40:T_l[0]] = True
    gout = rng.randn(N, Lq, M * D)
    eo, egv, egp, egr = expected_msda1d(value, mask, proj, ref, list(T_l), M, gout)
    v = cu(value, torch.float32).requires_grad_()
    p = cu(proj, torch.float32).requires_grad_()
    r = cu(ref, torch.float32).requires_grad_()
    out = MSDA1dFunction.apply(v, cu(mask).view(torch.uint8), p, r, tuple(T_l), 0, M * 16)
    close(out, eo, 1e-4, "out")
    out.backward(cu(gout, torch.float32))
    close(v.grad, egv, 1e-4, "grad_value")
    close(p.grad, egp, 1e-4, "grad_proj")
    close(r.grad, egr, 1e-4, "grad_ref")


def test_fused_msda1d_pyramid_equals_per_query():
    """The whole-pyramid and the per-query forward share their arithmetic (4 * Lq < S sends a query subset to
    the per-query kernel): equal up to FMA contraction."""
    from pdvc.ops.functions import MSDA1dFunction
    rng = np.random.RandomState(3)
    T_l = [64, 32, 16, 8]
    S = sum(T_l)
    M, D, N = 8, 64, 2
    value = cu(rng.randn(N, S, M, D), torch.float32)
    proj = cu(np.concatenate([rng.randn(N, S, M * 16) * 2, rng.randn(N, S, M * 16)], -1), torch.float32)
    ref = cu(rng.uniform(0, 1, size=(N, S, 4, 1)), torch.float32)
    full = MSDA1dFunction.apply(value, None, proj, ref, tuple(T_l), 0, M * 16)  # whole-pyramid (Lq == S)
    nq = S // 4 - 1
    part = MSDA1dFunction.apply(value, None, proj[:, :nq].contiguous(), ref[:, :nq].contiguous(), tuple(T_l),
                                0, M * 16)  # per-query (4 * Lq < S)
    err = (full[:, :nq] - part).abs().max().item()
    assert err <= 1e-6 * (part.abs().max().item() + 1.0), err


# ------------------------------------------------------------------------------------------------
# caption gather (border raw samples) vs oracle
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("D,M", [(512, 1), (64, 1), (32, 2), (128, 3)])
@pytest.mark.parametrize("ref_dim", [1, 2])
def test_cap_gather_vs_oracle(D, M, ref_dim):
    from pdvc.ops.functions import CapGatherFunction
    rng = np.random.RandomState(D + M + ref_dim)
    T_l = [24, 12, 6, 3]
    S, N, R, L, P = sum(T_l), 3, 11, 4, 4
    value = rng.randn(N, S, M, D)
    row_video = rng.randint(0, N, size=R).astype(np.int32)
    offsets = rng.randn(R, M * 16) * 3.0
    if ref_dim == 1:
        ref = rng.uniform(-0.1, 1.1, size=(R, 4, 1))
    else:
        ref = np.concatenate([rng.uniform(0, 1, size=(R, 4, 1)), rng.uniform(0.05, 0.9, size=(R, 4, 1))], -1)
    gs = rng.randn(R, M, 16, D)
    off = offsets.reshape(R, M, L, P)
    Tn = np.asarray(T_l, np.float64)[None, None, :, None]
    if ref_dim == 1:
        loc = ref[:, None, :, None, 0] + off / Tn
    else:
        loc = ref[:, None, :, None, 0] + off / P * ref[:, None, :, None, 1] * 0.5
    exp_s = np.zeros((R, M, 16, D))
    exp_gv = np.zeros_like(value)
    exp_gl = np.zeros((R, M, L, P))
    for r in range(R):
        b = row_video[r]
        loc2, shapes, lsi = O.lift_1d(loc[r][None, None], T_l)  # (1,1,M,L,P,2)
        s = O.msda_sample(value[b][None], shapes, lsi, loc2, "border")  # (M, D, 1, L, P)
        exp_s[r] = s[:, :, 0].reshape(M, D, 16).transpose(0, 2, 1)
        g = gs[r].transpose(0, 2, 1).reshape(M, D, 1, L, P)
        gv, gl = O.msda_sample_backward(value[b][None], shapes, lsi, loc2, g, "border")
        exp_gv[b] += gv[0]
        exp_gl[r] = gl[0, 0, ..., 0]
    if ref_dim == 1:
        exp_go = exp_gl / Tn
        exp_gr = exp_gl.sum(axis=(1, 3))[..., None]
    else:
        exp_go = exp_gl * 0.5 * ref[:, None, :, None, 1] / P
        exp_gr = np.stack([exp_gl.sum(axis=(1, 3)), (exp_gl * 0.5 * off / P).sum(axis=(1, 3))], -1)
    v = cu(value, torch.float32).requires_grad_()
    o = cu(offsets, torch.float32).requires_grad_()
    rf = cu(ref, torch.float32).requires_grad_()
    s = CapGatherFunction.apply(v, None, cu(row_video), o, rf, tuple(T_l), 0)
    close(s, exp_s, 1e-5, "samples")
    s.backward(cu(gs, torch.float32))
    close(v.grad, exp_gv, 1e-4, "grad_value")
    close(o.grad, exp_go.reshape(R, M * 16), 1e-4, "grad_offsets")
    close(rf.grad, exp_gr, 1e-4, "grad_ref")


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("ref_dim", [1, 2])
@pytest.mark.parametrize("masked", [False, True])
def test_cap_softattn_forward_matches_three_launches(M, ref_dim, masked):
    """pdvc_cap_softattn_forward_f32 (a caption step's value and projected-row samples and its soft attention in one
    launch, 512-wide heads) against pdvc_cap_gather_forward_f32 on the value (with its mask), on U (without) and
    pdvc_softattn_forward_f32: samples, save_loc and the U samples to 1e-6 of their magnitude (the same blends),
    probabilities and the attended rows to 1e-5 (the same sums; the tolerance covers codegen contraction)."""
    from pdvc import _native as _n
    rng = np.random.RandomState(M + 10 * ref_dim + 100 * masked)
    T_l = [24, 12, 6, 3]
    S, N, R, D = sum(T_l), 3, 13, 512
    value = cu(rng.randn(N, S, M, D), torch.float32)
    U = cu(rng.randn(N, S, M, D) * 0.2, torch.float32)
    mask = None
    if masked:
        mk = np.zeros((N, S), np.uint8)
        mk[1, 5:9] = 1
        mk[2, 30:33] = 1
        mask = cu(mk)
    row_video = cu(rng.randint(0, N, size=R).astype(np.int32))
    off_stride = M * 16 + 4 + D  # the offsets at column 0, then the att_h block at a 16-B aligned column
    hp = cu(rng.randn(R, off_stride) * 2.0, torch.float32)
    off_add = cu(rng.randn(R, M * 16) * 0.5, torch.float32)
    if ref_dim == 1:
        ref = cu(rng.uniform(-0.1, 1.1, size=(R, 4, 1)), torch.float32)
    else:
        ref = cu(np.concatenate([rng.uniform(0, 1, size=(R, 4, 1)), rng.uniform(0.05, 0.9, size=(R, 4, 1))], -1),
                 torch.float32)
    rd1 = 4 if ref_dim == 2 else 0
    aw = cu(rng.randn(D) * 0.1, torch.float32)
    ab = cu(rng.randn(1), torch.float32)
    ah, ldh = _n.rows(hp[:, M * 16 + 4:])
    lvl = _n.int_array(T_l)
    geo = (_n.ptr(row_video), _n.ptr(hp), off_stride, 0, _n.ptr(off_add), _n.ptr(ref), ref_dim, rd1, lvl, 4, N, R, M,
           D, 4)
    out = []
    for fused in (False, True):
        smp, loc = torch.empty(R, M, 16, D, device=DEV), torch.empty(R, M, 16, device=DEV)
        att, probs, res = (torch.empty(R * M * 16, D, device=DEV), torch.empty(R, M, 16, device=DEV),
                           torch.empty(R, M * D, device=DEV))
        if fused:
            _n.call("pdvc_cap_softattn_forward_f32", _n.ptr(value), _n.ptr(mask), _n.ptr(U), *geo, ah, ldh, _n.ptr(aw),
                    _n.ptr(ab), _n.ptr(smp), _n.ptr(loc), _n.ptr(att), _n.ptr(probs), _n.ptr(res), _n.stream())
        else:
            _n.call("pdvc_cap_gather_forward_f32", _n.ptr(value), _n.ptr(mask), *geo, _n.ptr(smp), _n.ptr(loc),
                    _n.stream())
            _n.call("pdvc_cap_gather_forward_f32", _n.ptr(U), None, *geo, _n.ptr(att), None, _n.stream())
            _n.call("pdvc_softattn_forward_f32", _n.ptr(att), ah, ldh, _n.ptr(aw), _n.ptr(ab), _n.ptr(smp), R, M, D, D,
                    _n.ptr(res), _n.ptr(probs), _n.stream())
        torch.cuda.synchronize()
        out.append((smp, loc, att, probs, res))
    for name, a, b, tol in zip(("samples", "save_loc", "att", "probs", "res"), *out, (1e-6, 0.0, 1e-6, 1e-5, 1e-5)):
        err = (a - b).abs().max().item()
        assert err <= tol * (a.abs().max().item() + 1.0), (name, err)
    assert out[1][3].max().item() < 0.99  # the soft attention is not degenerate


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("ref_dim", [1, 2])
@pytest.mark.parametrize("masked", [False, True])
def test_cap_softattn_backward_matches_two_launches(M, ref_dim, masked):
    """pdvc_cap_softattn_backward_f32 (the soft attention's and the sampling's backward in one launch, the samples and
    att re-formed from their corner rows) against pdvc_softattn_backward_f32 + pdvc_cap_gather_backward2_f32 (value2
    = U) on the forward's saved tensors: the att and sample gradients, the att_h, alpha_w and alpha_b gradients to
    1e-5 of their magnitude (the same expressions, the dots reduced in another order), the offset and reference
    gradients to 1e-4 (the location gradient's channel sums taken as p_k (dres . dv) + dd_k (w (1 - t^2) . du))."""
    from pdvc import _native as _n
    rng = np.random.RandomState(7 + M + 10 * ref_dim + 100 * masked)
    T_l = [24, 12, 6, 3]
    S, N, R, D = sum(T_l), 3, 13, 512
    value = cu(rng.randn(N, S, M, D), torch.float32)
    U = cu(rng.randn(N, S, M, D) * 0.2, torch.float32)
    mask = None
    if masked:
        mk = np.zeros((N, S), np.uint8)
        mk[1, 5:9] = 1
        mk[2, 30:33] = 1
        mask = cu(mk)
    row_video = cu(rng.randint(0, N, size=R).astype(np.int32))
    off_stride = M * 16 + 4 + D
    hp = cu(rng.randn(R, off_stride) * 2.0, torch.float32)
    off_add = cu(rng.randn(R, M * 16) * 0.5, torch.float32)
    if ref_dim == 1:
        ref = cu(rng.uniform(-0.1, 1.1, size=(R, 4, 1)), torch.float32)
    else:
        ref = cu(np.concatenate([rng.uniform(0, 1, size=(R, 4, 1)), rng.uniform(0.05, 0.9, size=(R, 4, 1))], -1),
                 torch.float32)
    rd1 = 4 if ref_dim == 2 else 0
    aw = cu(rng.randn(D) * 0.1, torch.float32)
    ab = cu(rng.randn(1), torch.float32)
    ah, ldh = _n.rows(hp[:, M * 16 + 4:])
    lvl = _n.int_array(T_l)
    geo = (_n.ptr(row_video), _n.ptr(hp), off_stride, 0, _n.ptr(off_add), _n.ptr(ref), ref_dim, rd1, lvl, 4, N, R, M,
           D, 4)
    smp, loc = torch.empty(R, M, 16, D, device=DEV), torch.empty(R, M, 16, device=DEV)
    att, probs, res = (torch.empty(R * M * 16, D, device=DEV), torch.empty(R, M, 16, device=DEV),
                       torch.empty(R, M * D, device=DEV))
    _n.call("pdvc_cap_softattn_forward_f32", _n.ptr(value), _n.ptr(mask), _n.ptr(U), *geo, ah, ldh, _n.ptr(aw),
            _n.ptr(ab), _n.ptr(smp), _n.ptr(loc), _n.ptr(att), _n.ptr(probs), _n.ptr(res), _n.stream())
    dres = cu(rng.randn(R, M * D), torch.float32)
    out = []
    for fused in (False, True):
        datt, dsmp = torch.empty(R * M * 16, D, device=DEV), torch.empty(R, M, 16, D, device=DEV)
        gaw, gab = torch.empty(R * M, D, device=DEV), torch.empty(R * M, device=DEV)
        dhp = torch.zeros(R, off_stride, device=DEV)
        gr = torch.zeros_like(ref)
        gah, ldgah = _n.rows(dhp[:, M * 16 + 4:])
        if fused:
            _n.call("pdvc_cap_softattn_backward_f32", _n.ptr(value), _n.ptr(mask), _n.ptr(U), *geo, _n.ptr(loc),
                    _n.ptr(probs), _n.ptr(dres), ah, ldh, _n.ptr(aw), _n.ptr(datt), gah, ldgah, _n.ptr(dsmp),
                    _n.ptr(gaw), _n.ptr(gab), _n.ptr(dhp), _n.ptr(gr), _n.stream())
        else:
            _n.call("pdvc_softattn_backward_f32", _n.ptr(att), ah, ldh, _n.ptr(aw), _n.ptr(smp), _n.ptr(probs),
                    _n.ptr(dres), R, M, D, D, _n.ptr(datt), gah, ldgah, _n.ptr(dsmp), _n.ptr(gaw), _n.ptr(gab),
                    _n.stream())
            _n.call("pdvc_cap_gather_backward2_f32", _n.ptr(value), _n.ptr(mask), *geo, _n.ptr(loc), _n.ptr(dsmp),
                    None, _n.ptr(dhp), _n.ptr(gr), _n.ptr(U), _n.ptr(datt), _n.stream())
        torch.cuda.synchronize()
        out.append((datt, dsmp, gaw, gab, dhp[:, M * 16 + 4:], dhp[:, :M * 16], gr))
    names = ("grad_att", "grad_samples", "grad_alpha_w", "grad_alpha_b", "grad_att_h", "grad_offsets", "grad_ref")
    for name, a, b, tol in zip(names, *out, (1e-5,) * 5 + (1e-4, 1e-4)):
        err = (a - b).abs().max().item()
        assert err <= tol * (a.abs().max().item() + 1.0), (name, err)
    assert out[0][5].abs().max().item() > 0 and out[0][6].abs().max().item() > 0


@pytest.mark.parametrize("D,M", [(512, 1), (64, 2)])
@pytest.mark.parametrize("masked", [False, True])
def test_cap_value_grad_rank1_matches_materialised(D, M, masked):
    """pdvc_cap_value_grad_rank1_f32 (sample gradients grad_scale[s] * grad_rows[step, row, head], formed in the
    value-gradient pass) against pdvc_cap_value_grad_ranged_f32 on the materialised (steps, rows, heads, 16, D)
    sample gradients: the same fp32 products; the counting sort places a row's samples in atomic order, so the sums
    agree to rounding (1e-6 of their magnitude), not bitwise, run to run as between the two forms."""
    from pdvc import _native as _n
    rng = np.random.RandomState(D + M + masked)
    T_l = [24, 12, 6, 3]
    S, Nv, R, n = sum(T_l), 3, 10, 3
    rv = rng.randint(0, Nv, size=R)
    order = np.argsort(rv, kind="stable")
    starts = np.concatenate([[0], np.cumsum(np.bincount(rv, minlength=Nv))]).astype(np.int32)
    loc = cu(rng.uniform(-0.1, 1.1, size=(n, R, M, 16)), torch.float32)
    grow = cu(rng.randn(n, R, M, D), torch.float32)
    gsc = cu(rng.uniform(0, 1, size=(n, R, M, 16)), torch.float32)
    gs = (gsc[..., None] * grow[:, :, :, None, :]).contiguous()
    mask = None
    if masked:
        mk = np.zeros((Nv, S), np.uint8)
        mk[1, 3:7] = 1
        mk[2, 40:] = 1
        mask = cu(mk)
    vs, vr = cu(starts), cu(order.astype(np.int32))
    max_rows = int(np.bincount(rv, minlength=Nv).max())
    lvl = _n.int_array(T_l)
    out = []
    for rank1 in (False, True):
        gv = torch.empty(Nv, S, M, D, device=DEV)
        ls = torch.empty(Nv, 4, M * D, device=DEV)
        if rank1:
            _n.call("pdvc_cap_value_grad_rank1_f32", _n.ptr(mask), lvl, 4, Nv, M, D, 4, R, n, max_rows, _n.ptr(vs),
                    _n.ptr(vr), None, _n.ptr(loc), _n.ptr(grow), _n.ptr(gsc), _n.ptr(gv), _n.ptr(ls), _n.stream())
        else:
            _n.call("pdvc_cap_value_grad_ranged_f32", _n.ptr(mask), lvl, 4, Nv, M, D, 4, R, n, max_rows, _n.ptr(vs),
                    _n.ptr(vr), None, _n.ptr(loc), _n.ptr(gs), _n.ptr(gv), _n.ptr(ls), _n.stream())
        torch.cuda.synchronize()
        out.append((gv, ls))
    for a, b in zip(out[0], out[1]):
        assert (a - b).abs().max().item() <= 1e-6 * (a.abs().max().item() + 1.0)
    assert out[0][0].abs().max().item() > 0


@pytest.mark.parametrize("n,R", [(3, 10), (25, 600)])
def test_cap_value_grad_bf16out_rounds_like_torch(n, R):
    """pdvc_cap_value_grad_ranged_f32_bf16out (the bf16 mode's caption dU): grad_value and its level sums as the plain
    form (to the counting sort's rounding), and beside grad_value its bf16 rounding, bit for bit torch's cast of the
    grad_value it wrote; 25 steps of ~200 rows per video split the samples into several accumulating chunks of steps
    (the LDS budget: the last chunk writes the final rows)."""
    from pdvc import _native as _n
    rng = np.random.RandomState(n)
    T_l = [24, 12, 6, 3]
    S, Nv, M, D = sum(T_l), 3, 1, 512
    rv = rng.randint(0, Nv, size=R)
    order = np.argsort(rv, kind="stable")
    starts = np.concatenate([[0], np.cumsum(np.bincount(rv, minlength=Nv))]).astype(np.int32)
    loc = cu(rng.uniform(-0.1, 1.1, size=(n, R, M, 16)), torch.float32)
    gs = cu(rng.randn(n, R, M, 16, D), torch.float32)
    vs, vr = cu(starts), cu(order.astype(np.int32))
    max_rows = int(np.bincount(rv, minlength=Nv).max())
    lvl = _n.int_array(T_l)
    out = []
    for bf in (False, True):
        gv = torch.full((Nv, S, M, D), 3.0, device=DEV)
        ls = torch.empty(Nv, 4, M * D, device=DEV)
        g16 = torch.zeros(gv.shape, device=DEV, dtype=torch.bfloat16)
        args = (None, lvl, 4, Nv, M, D, 4, R, n, max_rows, _n.ptr(vs), _n.ptr(vr), None, _n.ptr(loc), _n.ptr(gs),
                _n.ptr(gv), _n.ptr(ls))
        if bf:
            _n.call("pdvc_cap_value_grad_ranged_f32_bf16out", *args, _n.ptr(g16), _n.stream())
        else:
            _n.call("pdvc_cap_value_grad_ranged_f32", *args, _n.stream())
        torch.cuda.synchronize()
        out.append((gv, ls, g16))
    # the counting sort places a row's samples in atomic order: the two runs' sums agree to fp32 rounding of sums of up
    # to a few thousand terms at the (25, 600) size (measured 1.1e-6 of the magnitude), not bitwise
    for a, b in zip(out[0][:2], out[1][:2]):
        assert (a - b).abs().max().item() <= 1e-5 * (a.abs().max().item() + 1.0)
    gv1, g16 = out[1][0], out[1][2]
    assert torch.equal(g16.view(torch.int16), gv1.to(torch.bfloat16).view(torch.int16))
    assert gv1.abs().max().item() > 0


def test_cap_softattn_forward_rejects_other_widths():
    """the fused step is the 512-wide form only: any other head width is PDVC_ERR_UNSUPPORTED, not a wrong answer"""
    from pdvc import _native as _n
    with pytest.raises(Exception):
        _n.call("pdvc_cap_softattn_forward_f32", *([None] * 5), 80, 0, None, None, 1, 0, _n.int_array([4, 2, 1, 1]),
                4, 1, 1, 1, 64, 4, None, 64, *([None] * 7), _n.stream())


# ------------------------------------------------------------------------------------------------
# modules vs golden vectors generated from the reference modules
# ------------------------------------------------------------------------------------------------
def _fill(module):
    import sys
    sys.path.insert(0, G)
    import weights as W
    W.fill_module(module, overrides={"sampling_offsets": 0.5})


@pytest.mark.parametrize("ref_dim", [1, 2])
def test_module_msdeformattn_vs_golden(ref_dim):
    from pdvc.ops.modules import MSDeformAttn
    d = load(f"module_msdeformattn_ref{ref_dim}")
    m = MSDeformAttn(64, 4, 4, 4).to(DEV)
    _fill(m)
    q = cu(d["query"]).requires_grad_()
    r = cu(d["ref"]).requires_grad_()
    x = cu(d["x"]).requires_grad_()
    T_l = tuple(int(t) for t in d["T_l"])
    shapes = torch.as_tensor(T_l, device=DEV)
    lsi = torch.cat([shapes.new_zeros(1), shapes.cumsum(0)[:-1]])
    out = m(q, r, x, T_l, lsi, cu(d["pad"]))
    close(out, d["out"], 1e-4, "out")
    out.backward(cu(d["grad_out"]))
    close(q.grad, d["grad_query"], 1e-4, "grad_query")
    close(r.grad, d["grad_ref"], 1e-4, "grad_ref")
    close(x.grad, d["grad_x"], 1e-4, "grad_x")
    for n, p in m.named_parameters():
        close(p.grad, d["grad." + n], 1e-4, n)


@pytest.mark.parametrize("D,T_l,Lq,masked", [(64, (40, 20, 10, 5), 37, True), (64, (128, 64, 32, 16), 240, False),
                                             (64, (512, 256, 128, 64), 960, True), (64, (512, 256, 128, 64), 100, True),
                                             (64, (1024, 512, 256, 128), 1920, True), (32, (40, 20, 10, 5), 37, True)])
def test_msda1d_value_level_sums(D, T_l, Lq, masked):
    """pdvc_msda1d_backward_ex_f32's per-(video, level) column sums of grad_value (the value bias gradient's
    partials) against the sums of the grad_value it returns: formed inside the D = 64 value-gradient kernel (one
    query chunk at the encoder's Lq = 960 and the decoder's Lq = 100; two chunks at S = 1920, the second
    accumulating), by a second pass otherwise (D = 32)."""
    from pdvc.ops.functions.ms_deform_attn_func import msda1d_backward, msda1d_forward
    rng = np.random.RandomState(D + Lq)
    M, N = 8 if D == 64 else 4, 2
    S = sum(T_l)
    value = cu(rng.randn(N, S, M, D), torch.float32)
    proj = cu(np.concatenate([rng.randn(N, Lq, M * 16) * 3.0, rng.randn(N, Lq, M * 16)], -1), torch.float32)
    ref = cu(rng.uniform(-0.05, 1.05, size=(N, Lq, 4, 1)), torch.float32)
    mask = None
    if masked:
        mk = np.zeros((N, S), bool)
        mk[1, 3:9] = True
        mk[0, T_l[0]:T_l[0] + 4] = True
        mask = cu(mk).view(torch.uint8)
    gout = cu(rng.randn(N, Lq, M * D), torch.float32)
    out, sa, sl = msda1d_forward(value, mask, proj, ref, T_l, 0, M * 16)
    gv, gp, gr, ls = msda1d_backward(value, mask, proj, ref, sa, sl, out, gout, T_l, 0, M * 16, level_sums=True)
    gv0, gp0, _ = msda1d_backward(value, mask, proj, ref, sa, sl, out, gout, T_l, 0, M * 16)
    # the counting sort's LDS cursors order samples within a bucket arbitrarily: run-to-run ulp differences
    assert torch.equal(gp, gp0) and (gv - gv0).abs().max().item() <= 1e-5
    g = gv.double().view(N, S, M * D)
    starts = np.cumsum((0,) + tuple(T_l))
    exp = torch.stack([g[:, starts[i]:starts[i + 1]].sum(1) for i in range(4)], 1)
    assert ls.shape == exp.shape
    err = (ls.double() - exp).abs().max().item()
    assert err <= 1e-5 * (g.abs().sum(1).max().item() + 1.0), err
