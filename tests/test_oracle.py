"""CPU: pin the oracle (oracle/msda_oracle.c) against the golden vectors generated from the
reference (tests/golden/make_golden.py) -- the reference test's own inputs (pdvc/ops/test.py:21-44)
and 1-D PDVC pyramids -- plus finite differences.  No GPU needed."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("pad", ["zeros", "border"])
def test_reftest_inputs(pad):
    d = load("op_reftest")
    out = O.msda_forward(d["value"], d["shapes"], d["lsi"], d["loc"], d["attn"], pad)
    np.testing.assert_allclose(out, d[f"{pad}_out"], rtol=1e-12, atol=1e-14)
    gv, gl, ga = O.msda_backward(d["value"], d["shapes"], d["lsi"], d["loc"], d["attn"], d["grad_out"], pad)
    np.testing.assert_allclose(gv, d[f"{pad}_grad_value"], rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(gl, d[f"{pad}_grad_loc"], rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(ga, d[f"{pad}_grad_attn"], rtol=1e-10, atol=1e-14)


def test_reftest_padding_modes_differ():
    """the fork's CPU core (border) and the CUDA op (zeros) disagree on test.py's inputs."""
    d = load("op_reftest")
    assert np.abs(d["zeros_out"] - d["border_out"]).max() > 1e-4


@pytest.mark.parametrize("D", [30, 32, 64, 71])
@pytest.mark.parametrize("pad", ["zeros", "border"])
@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_1d_pyramids(D, pad, dt):
    d = load(f"op_1d_D{D}")
    npdt = np.float64 if dt == "f64" else np.float32
    tol = dict(rtol=1e-11, atol=1e-12) if dt == "f64" else dict(rtol=2e-5, atol=2e-5)
    args = [d["value"].astype(npdt), d["shapes"], d["lsi"], d["loc"].astype(npdt), d["attn"].astype(npdt)]
    out = O.msda_forward(*args, pad)
    np.testing.assert_allclose(out, d[f"{pad}_{dt}_out"], **tol)
    gv, gl, ga = O.msda_backward(*args, d["grad_out"].astype(npdt), pad)
    np.testing.assert_allclose(gv, d[f"{pad}_{dt}_grad_value"], **tol)
    np.testing.assert_allclose(ga, d[f"{pad}_{dt}_grad_attn"], **tol)
    # y-gradients: torch's border clip zeroes them (H=1 => iy clipped); the CUDA op reports H*dval/dh
    np.testing.assert_allclose(gl[..., 0], d[f"{pad}_{dt}_grad_loc"][..., 0], **tol)
    if pad == "border":
        np.testing.assert_allclose(gl[..., 1], d[f"{pad}_{dt}_grad_loc"][..., 1], **tol)


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_sample_mode(dt):
    d = load("op_sample")
    npdt = np.float64 if dt == "f64" else np.float32
    tol = dict(rtol=1e-11, atol=1e-12) if dt == "f64" else dict(rtol=2e-5, atol=2e-5)
    v, lo = d["value"].astype(npdt), d["loc"].astype(npdt)
    s = O.msda_sample(v, d["shapes"], d["lsi"], lo, "border")
    np.testing.assert_allclose(s, d[f"{dt}_samples"], **tol)
    gv, gl = O.msda_sample_backward(v, d["shapes"], d["lsi"], lo, d["grad_samples"].astype(npdt), "border")
    np.testing.assert_allclose(gv, d[f"{dt}_grad_value"], **tol)
    np.testing.assert_allclose(gl, d[f"{dt}_grad_loc"], **tol)


def test_zeros_finite_difference():
    """Central differences of the zeros oracle (the reference test's gradcheck, test.py:63-86)."""
    rng = np.random.RandomState(0)
    shapes = np.array([[6, 4], [3, 2]])
    lsi = np.array([0, 24])
    N, M, D, Lq, L, P = 1, 2, 5, 2, 2, 2
    v = rng.rand(N, 30, M, D) * 0.01
    loc = rng.uniform(0.05, 0.95, size=(N, Lq, M, L, P, 2))
    a = rng.rand(N, Lq, M, L, P) + 1e-5
    g = rng.randn(N, Lq, M * D)
    gv, gl, ga = O.msda_backward(v, shapes, lsi, loc, a, g, "zeros")
    f = lambda v_, l_, a_: (O.msda_forward(v_, shapes, lsi, l_, a_, "zeros") * g).sum()
    eps = 1e-6
    for arr, grad in ((v, gv), (loc, gl), (a, ga)):
        flat = arr.reshape(-1)
        for i in rng.choice(flat.size, 12, replace=False):
            old = flat[i]
            flat[i] = old + eps
            fp = f(v, loc, a)
            flat[i] = old - eps
            fm = f(v, loc, a)
            flat[i] = old
            assert abs((fp - fm) / (2 * eps) - grad.reshape(-1)[i]) < 1e-6


@pytest.mark.parametrize("D", [30, 64])
def test_torch_cpu_core_matches_reference_border(D):
    """oracle/torch_core.py (the CPU baseline bench.py times) reproduces the reference's CPU core
    (ms_deform_attn_core_pytorch, border padding) on its fixtures, forward and every gradient, fp64."""
    import torch
    from oracle.torch_core import ms_deform_attn_core_cpu
    d = load(f"op_1d_D{D}")
    shapes = [tuple(int(x) for x in s) for s in d["shapes"]]
    v, lo, a = (torch.tensor(d[k], dtype=torch.float64, requires_grad=True) for k in ("value", "loc", "attn"))
    out = ms_deform_attn_core_cpu(v, shapes, lo, a)
    np.testing.assert_allclose(out.detach().numpy(), d["border_f64_out"], rtol=1e-12, atol=1e-13)
    out.backward(torch.tensor(d["grad_out"]))
    np.testing.assert_allclose(v.grad.numpy(), d["border_f64_grad_value"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(lo.grad.numpy(), d["border_f64_grad_loc"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(a.grad.numpy(), d["border_f64_grad_attn"], rtol=1e-12, atol=1e-13)
    s = load("op_sample")
    vs = torch.tensor(s["value"], dtype=torch.float64)
    samp = ms_deform_attn_core_cpu(vs, [tuple(int(x) for x in r) for r in s["shapes"]],
                                   torch.tensor(s["loc"]), torch.zeros(1, 6, 1, 4, 4, dtype=torch.float64),
                                   return_value=True)
    np.testing.assert_allclose(samp.numpy(), s["f64_samples"], rtol=1e-12, atol=1e-13)


def test_cpu_baseline_timer_runs():
    from oracle.torch_core import time_call_set
    t, info = time_call_set(T=32, Q=10, runs=3, warmup=1, threads=2)
    assert t > 0 and info["threads"] == 2 and info["runs"] == 3


# ---- the caption head's decode step (oracle/cap_step.py) against the reference captioner's fixtures ----------
CAP_SHAPES = {  # the reference LSTMDSACaptioner(small_opt) parameters (tests/golden/make_golden.py::module_captioner)
    "embed.weight": (24, 32), "logit.weight": (24, 64), "logit.bias": (24,),
    "core.rnn.weight_ih_l0": (256, 160), "core.rnn.weight_hh_l0": (256, 64),
    "core.deformable_att.sampling_offsets.weight": (16, 128), "core.deformable_att.sampling_offsets.bias": (16,),
    "core.deformable_att.value_proj.weight": (64, 64), "core.deformable_att.value_proj.bias": (64,),
    "core.ctx2att.weight": (48, 64), "core.ctx2att.bias": (48,), "core.h2att.weight": (48, 64),
    "core.h2att.bias": (48,), "core.alpha_net.weight": (1, 48), "core.alpha_net.bias": (1,),
}


@pytest.mark.parametrize("ref_dim", [1, 2])
def test_caption_step_oracle_matches_reference_captioner(ref_dim):
    """oracle/cap_step.py's float64 restatement of the captioner (soft-attention step, LSTM cell, logits) against
    the reference module's fixture: logprobs, loss and every gradient (the fixture is float32: 1e-5 relative)."""
    import sys
    import torch
    sys.path.insert(0, GOLD)
    import weights as W
    from oracle import cap_step as C
    d = np.load(os.path.join(GOLD, f"module_captioner_ref{ref_dim}.npz"))
    P = {}
    for name, shape in CAP_SHAPES.items():
        scale = 0.5 if "sampling_offsets" in name else None
        P[name] = C.to_f64(W.param_array(name, shape, scale), grad=True)
    hs, ref, memory = C.to_f64(d["hs"], True), C.to_f64(d["ref"], True), C.to_f64(d["memory"], True)
    mask = torch.as_tensor(d["mask"])
    cap = torch.as_tensor(d["cap_tensor"])
    lp = C.captioner_forward(P, hs, ref, memory, mask, [int(t) for t in d["T_l"]], cap)
    np.testing.assert_allclose(lp.detach().numpy(), d["logprobs"], rtol=0, atol=1e-5 * np.abs(d["logprobs"]).max())
    loss = C.build_loss(lp, cap[:, 1:], torch.as_tensor(d["cap_mask"][:, 1:]).double(), 23).mean()
    assert abs(float(loss) - float(d["loss"])) <= 1e-5 * abs(float(d["loss"]))
    loss.backward()
    checks = [("grad_hs", hs.grad), ("grad_ref", ref.grad), ("grad_memory", memory.grad)]
    checks += [(f"grad.{n}", p.grad) for n, p in P.items()]
    for key, g in checks:
        want = d[key]
        err = np.abs(g.numpy() - want).max()
        assert err <= 1e-5 * np.abs(want).max() + 1e-9, (key, err, np.abs(want).max())
