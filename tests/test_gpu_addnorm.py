"""Fused norm(x + dropout(s)) (csrc/addnorm.hip) against torch float64: p = 0 exactly (forward, all four
gradients), and p > 0 against torch with the kernel's own mask (recovered from where ds vanishes)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def reference(x, s, w, b, mask, p, eps):
    x, s, w, b = (t.detach().double().requires_grad_() for t in (x, s, w, b))
    sd = s * mask.double() / (1 - p) if p > 0 else s
    y = torch.nn.functional.layer_norm(x + sd, (x.shape[-1],), w, b, eps)
    return y, (x, s, w, b)


@pytest.mark.parametrize("rows,d", [(3, 64), (1000, 512), (30720, 512), (77, 256)])
def test_addnorm_p0(rows, d):
    from pdvc.ops.functions import AddDropoutLayerNormFunction
    torch.manual_seed(rows + d)
    x, s = torch.randn(rows, d, device=DEV), torch.randn(rows, d, device=DEV) * 2
    w, b = torch.randn(d, device=DEV), torch.randn(d, device=DEV)
    g = torch.randn(rows, d, device=DEV)
    ins = [t.clone().requires_grad_() for t in (x, s, w, b)]
    y = AddDropoutLayerNormFunction.apply(*ins, 0.0, 1e-5, 0)
    y.backward(g)
    yr, rins = reference(x, s, w, b, None, 0.0, 1e-5)
    yr.backward(g.double())
    assert (y.double() - yr).abs().max().item() < 1e-5
    for got, ref, name in zip(ins, rins, ("dx", "ds", "dgamma", "dbeta")):
        err = (got.grad.double() - ref.grad).abs().max().item()
        assert err < 2e-5 * (ref.grad.abs().max().item() + 1), f"{name}: {err}"


def test_addnorm_dropout_consistent():
    from pdvc.ops.functions import AddDropoutLayerNormFunction
    torch.manual_seed(0)
    rows, d, p = 4096, 512, 0.1
    x, s = torch.randn(rows, d, device=DEV), torch.randn(rows, d, device=DEV)
    w, b = torch.randn(d, device=DEV), torch.randn(d, device=DEV)
    g = torch.randn(rows, d, device=DEV)
    seed = torch.tensor([123456789], device=DEV, dtype=torch.int64)
    ins = [t.clone().requires_grad_() for t in (x, s, w, b)]
    y = AddDropoutLayerNormFunction.apply(*ins, p, 1e-5, seed)
    y2 = AddDropoutLayerNormFunction.apply(x, s, w, b, p, 1e-5, seed)
    assert torch.equal(y, y2), "same seed, same mask"
    y.backward(g)
    mask = ins[1].grad != 0
    frac = mask.float().mean().item()
    assert abs(frac - (1 - p)) < 0.01, frac
    yr, rins = reference(x, s, w, b, mask, p, 1e-5)
    yr.backward(g.double())
    assert (y.double() - yr).abs().max().item() < 1e-5
    for got, ref, name in zip(ins, rins, ("dx", "ds", "dgamma", "dbeta")):
        err = (got.grad.double() - ref.grad).abs().max().item()
        assert err < 2e-5 * (ref.grad.abs().max().item() + 1), f"{name}: {err}"
