"""GPU parity of the fused feed-forward sub-layer (pdvc/ops/functions/ffn.py, csrc/ffn.hip) against a float64
torch restatement of the reference chain norm(x + dropout(linear2(dropout(relu(linear1(x)))))), reference
deformable_transformer.py:140-145.  The in-kernel dropout mask is recovered by running the relu+dropout kernel
on a tensor of ones with the same seed (the mask depends on (seed, row, column) only)."""
import pytest
import torch
from parity import assert_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


def close(a, b, tol, what):
    """Per-tensor relative bound: max|a - b| <= tol * max|b| + 1e-7 (tests/parity.py)."""
    assert_close(a, b, what, tol)


def act_mask(seed_tensor, rows, cols, p):
    from pdvc import _native as _n
    ones = torch.ones(rows, cols, device=DEV)
    _n.call("pdvc_relu_dropout_forward_f32", _n.ptr(ones), rows, cols, float(p), 0, _n.ptr(seed_tensor), _n.stream())
    return ones


def test_relu_dropout_forward_statistics_and_values():
    from pdvc import _native as _n
    torch.manual_seed(0)
    rows, cols, p = 3000, 512, 0.25
    h = torch.randn(rows, cols, device=DEV)
    seed = torch.tensor([123456789], dtype=torch.int64, device=DEV)
    out = h.clone()
    _n.call("pdvc_relu_dropout_forward_f32", _n.ptr(out), rows, cols, p, 0, _n.ptr(seed), _n.stream())
    m = act_mask(seed, rows, cols, p)
    kept = (m > 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.01, kept
    close(m[m > 0], torch.full_like(m[m > 0], 1 / (1 - p)), 1e-6, "scale")
    close(out, h.clamp_min(0) * m, 0, "relu*mask")
    out0 = h.clone()  # p = 0: plain relu
    _n.call("pdvc_relu_dropout_forward_f32", _n.ptr(out0), rows, cols, 0.0, 7, None, _n.stream())
    close(out0, h.clamp_min(0), 0, "relu")
    # a different seed gives a different mask
    m2 = act_mask(torch.tensor([987654321], dtype=torch.int64, device=DEV), rows, cols, p)
    assert (m2 != m).float().mean().item() > 0.2


@pytest.mark.parametrize("rows,d,f,p_act", [(333, 64, 256, 0.0), (2048, 128, 512, 0.3), (130, 32, 96, 0.1)])
def test_ffn_block_matches_float64_chain(rows, d, f, p_act):
    from pdvc.ops.functions.ffn import FFNBlockFunction
    torch.manual_seed(rows)
    x = torch.randn(2, rows // 2 if rows % 2 == 0 else rows, d, device=DEV)
    lin1, lin2 = torch.nn.Linear(d, f).to(DEV), torch.nn.Linear(f, d).to(DEV)
    norm = torch.nn.LayerNorm(d).to(DEV)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.2, 0.2)
    seeds = torch.tensor([11, 22], dtype=torch.int64, device=DEV)
    params = [lin1.weight, lin1.bias, lin2.weight, lin2.bias, norm.weight, norm.bias]
    xa = x.clone().requires_grad_()
    out = FFNBlockFunction.apply(xa, *params, p_act, 0.0, norm.eps, seeds)
    g = torch.randn_like(out)
    grads = torch.autograd.grad(out, [xa] + params, g)
    R = x.numel() // d
    mask = act_mask(seeds[0:1], R, f, p_act).double() if p_act > 0 else torch.ones(R, f, device=DEV).double()
    x64 = x.double().reshape(R, d).requires_grad_()
    p64 = [t.detach().double().requires_grad_() for t in params]
    h = torch.relu(x64 @ p64[0].t() + p64[1]) * mask
    y = h @ p64[2].t() + p64[3]
    ref = torch.nn.functional.layer_norm(x64 + y, (d,), p64[4], p64[5], norm.eps)
    ref_grads = torch.autograd.grad(ref, [x64] + p64, g.double().reshape(R, d))
    close(out.reshape(R, d), ref, 1e-5, "out")
    names = ["x", "linear1.weight", "linear1.bias", "linear2.weight", "linear2.bias", "norm.weight", "norm.bias"]
    for n, a, b in zip(names, grads, ref_grads):
        close(a.reshape(b.shape), b, 1e-4, n)
