"""GPU parity of the fused caption log-probabilities + target pick (pdvc/ops/functions/logprob.py,
csrc/logprob.hip) against the reference chain log_softmax -> gather -> masked sum (LSTM_DSA.py:48-52,
112-116) in float64 torch: values, the logits gradient through the loss, and a gradient arriving on logp
itself.  All kernel forms: register-resident (V % 4 == 0, V <= 8192: ActivityNet's 5748), streaming float4
(V % 4 == 0, V > 8192) and scalar (V % 4 != 0: YouCook2's 1609)."""
import pytest
import torch
from parity import assert_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5  # fp32 vs float64 reference: max|diff| <= TOL * max|reference| + 1e-7 per tensor


def close(a, b, tol, what):
    """Per-tensor relative bound: max|a - b| <= tol * max|b| + 1e-7 (tests/parity.py)."""
    assert_close(a, b, what, tol)


@pytest.mark.parametrize("V", [5748, 1609, 7, 300, 8200])  # 8200: the streaming float4 form (> 8192)
def test_logprob_pick_matches_log_softmax_gather(V):
    from pdvc.ops.functions.logprob import logprob_pick
    g = torch.Generator().manual_seed(V)
    R, n = 37, 6
    logits = (torch.randn(R, n, V, generator=g) * 4).to(DEV)
    target = torch.randint(0, V, (R, n), generator=g).to(DEV)
    target[0, :] = 0
    target[1, :] = V - 1
    mask = (torch.rand(R, n, generator=g) > 0.3).float().to(DEV)
    x = logits.clone().requires_grad_(True)
    logp, picked = logprob_pick(x, target)
    loss = (-(picked * mask).sum(1) / (mask.sum(1) + 1e-6)).sum()
    loss.backward()
    xr = logits.double().clone().requires_grad_(True)
    lr = torch.log_softmax(xr, -1)
    pr = lr.gather(2, target[:, :, None]).squeeze(2)
    (-(pr * mask.double()).sum(1) / (mask.double().sum(1) + 1e-6)).sum().backward()
    close(logp, lr, TOL, "logp")
    close(picked, pr, TOL, "picked")
    close(x.grad, xr.grad, TOL, "grad logits")


def test_logprob_pick_gradient_on_logp_too():
    from pdvc.ops.functions.logprob import logprob_pick
    g = torch.Generator().manual_seed(3)
    R, n, V = 9, 4, 5748
    logits = torch.randn(R, n, V, generator=g).to(DEV)
    target = torch.randint(0, V, (R, n), generator=g).to(DEV)
    w = torch.randn(R, n, V, generator=g).to(DEV)
    x = logits.clone().requires_grad_(True)
    logp, picked = logprob_pick(x, target)
    ((logp * w).sum() + picked.sum()).backward()
    xr = logits.double().clone().requires_grad_(True)
    lr = torch.log_softmax(xr, -1)
    ((lr * w.double()).sum() + lr.gather(2, target[:, :, None]).sum()).backward()
    close(x.grad, xr.grad, TOL, "grad logits (logp + picked)")


def test_logprob_pick_bad_target_poisons_and_empty_rows():
    from pdvc.ops.functions.logprob import logprob_pick
    x = torch.randn(2, 3, 16, device=DEV)
    t = torch.tensor([[0, 16, 3], [-1, 2, 15]], device=DEV)
    _, picked = logprob_pick(x, t)
    p = picked.cpu()
    assert torch.isnan(p[0, 1]) and torch.isnan(p[1, 0]) and torch.isfinite(p[0, 0]) and torch.isfinite(p[1, 2])
    logp, picked = logprob_pick(torch.randn(0, 3, 16, device=DEV), torch.zeros(0, 3, dtype=torch.long, device=DEV))
    assert logp.shape == (0, 3, 16) and picked.shape == (0, 3)


@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("V", [5749, 1609, 37, 8192, 9000, 3, 4])
def test_logprob_argmax_matches_torch(V, off):
    """pdvc_logprob_argmax_f32 (greedy decoding's word choice, LSTM_DSA.py:149-151) against torch.max over
    log_softmax: identical indices (ties to the first maximal index, rows with repeated maxima included), the
    log-probabilities within 1e-5; the register-resident kernel (V <= 8 192) and the streaming one (9 000), V = 3 and
    4, logits 16-byte aligned or not (off)."""
    from pdvc import _native as _n
    torch.manual_seed(V)
    R = 300
    x = (torch.randn(R * V + off, device="cuda") * 3)[off:].view(R, V)
    x[5, :] = 0.25                      # all tied: index 0
    x[6, V // 2] = x[6].max() + 1.0     # a clear winner in the middle
    x[7, V - 1] = x[7].max() + 1.0      # ... at the end
    if V > 4:
        x[8, 3] = x[8, V - 2] = x[8].max() + 2.0  # tie between two entries: the first
    want_lp, want_i = torch.max(torch.log_softmax(x, 1), 1)
    idx = torch.empty(R, dtype=torch.long, device="cuda")
    lp = torch.empty(R, device="cuda")
    _n.call("pdvc_logprob_argmax_f32", _n.ptr_any(x), R, V, _n.ptr(idx), _n.ptr(lp), _n.stream())
    assert torch.equal(idx, want_i)
    assert (lp - want_lp).abs().max().item() <= 1e-5


@pytest.mark.parametrize("V,rows", [(5748, 9000), (1609, 8200), (37, 300)])
def test_logit_pick_fused_matches_float64(V, rows):
    """LogitPickFunction (the caption logit layer + logprob_pick as one node, its dlogits in rows padded to a multiple
    of 32 columns so that dlogits @ W runs on the in-tree GEMM) against float64 torch: logp, picked and the
    gradients of the input rows, the weight and the bias, with a gradient on logp as well."""
    from pdvc.ops.functions.logprob import logit_pick
    from pdvc.ops.modules.linear import Linear
    g = torch.Generator().manual_seed(V + rows)
    H = 512
    layer = Linear(H, V).to(DEV)
    with torch.no_grad():
        layer.weight.copy_(torch.randn(V, H, generator=g) * 0.05)
        layer.bias.copy_(torch.randn(V, generator=g) * 0.1)
    x0 = torch.randn(rows, H, generator=g).to(DEV)
    target = torch.randint(0, V, (rows,), generator=g).to(DEV)
    gpick = torch.randn(rows, generator=g).to(DEV)
    glogp = (torch.randn(rows, V, generator=g) * 1e-3).to(DEV)
    x = x0.clone().requires_grad_(True)
    logp, picked = logit_pick(x, layer, target)
    ((picked * gpick).sum() + (logp * glogp).sum()).backward()
    xr = x0.double().clone().requires_grad_(True)
    Wr = layer.weight.detach().double().clone().requires_grad_(True)
    br = layer.bias.detach().double().clone().requires_grad_(True)
    lr = torch.log_softmax(xr @ Wr.t() + br, -1)
    pr = lr.gather(1, target[:, None]).squeeze(1)
    ((pr * gpick.double()).sum() + (lr * glogp.double()).sum()).backward()
    close(logp, lr, TOL, "logp")
    close(picked, pr, TOL, "picked")
    close(x.grad, xr.grad, TOL, "grad x")
    close(layer.weight.grad, Wr.grad, TOL, "grad W")
    close(layer.bias.grad, br.grad, TOL, "grad b")
