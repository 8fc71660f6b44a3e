"""The fp32 matrix-core GEMM (csrc/gemm.hip) against float64 torch: every operand orientation, ragged
shapes (tile and K-slice edges), bias / ReLU epilogues, split-K accumulation, and nn.Linear's backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def ref64(a, b, bias=None, relu=False):
    y = a.double() @ b.double()
    if bias is not None:
        y = y + bias.double()
    return y.clamp(min=0) if relu else y


def check(got, exp, what):
    err = (got.double() - exp).abs().max().item()
    scale = exp.abs().max().item() + 1.0
    assert err <= 2e-6 * scale, f"{what}: max err {err:.3e} (scale {scale:.3g})"


@pytest.mark.parametrize("M,N,K", [(128, 128, 32), (37, 75, 133), (300, 260, 515), (1, 5748, 512), (513, 1, 64)])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_orientations(M, N, K, ta, tb):
    from pdvc.ops.functions import matmul
    torch.manual_seed(M * 7 + N + K)
    A = torch.randn(K, M, device=DEV).t() if ta else torch.randn(M, K, device=DEV)
    B = torch.randn(N, K, device=DEV).t() if tb else torch.randn(K, N, device=DEV)
    check(matmul(A, B), ref64(A, B), f"plain ta={ta} tb={tb}")
    bias = torch.randn(N, device=DEV)
    check(matmul(A, B, bias=bias), ref64(A, B, bias), "bias")
    check(matmul(A, B, bias=bias, relu=True), ref64(A, B, bias, True), "bias+relu")


@pytest.mark.parametrize("M,N,K", [(512, 512, 30720), (256, 2576, 3584), (100, 70, 4099)])
def test_gemm_split_k_accumulate(M, N, K):
    from pdvc.ops.functions import matmul
    torch.manual_seed(K)
    A = torch.randn(K, M, device=DEV).t()  # the weight-gradient orientation: dy^T
    B = torch.randn(K, N, device=DEV)
    C0 = torch.randn(M, N, device=DEV)
    C = C0.clone()
    matmul(A, B, out=C, accumulate=True)
    exp = C0.double() + A.double() @ B.double()
    err = (C.double() - exp).abs().max().item()
    assert err <= 1e-5 * (exp.abs().max().item() + 1.0), err


def test_linear_function_matches_nn_linear():
    from pdvc.ops.functions.linear import linear
    torch.manual_seed(0)
    lin = torch.nn.Linear(512, 256).to(DEV).double()
    x = torch.randn(4, 960, 512, device=DEV, dtype=torch.float64, requires_grad=True)
    g = torch.randn(4, 960, 256, device=DEV, dtype=torch.float64)
    y = lin(x)
    y.backward(g)
    w = lin.weight.detach().float().requires_grad_()
    b = lin.bias.detach().float().requires_grad_()
    xf = x.detach().float().requires_grad_()
    yf = linear(xf, w, b)
    yf.backward(g.float())
    check(yf, y.detach(), "y")
    for got, exp, name in ((xf.grad, x.grad, "dx"), (w.grad, lin.weight.grad, "dW"), (b.grad, lin.bias.grad, "db")):
        err = (got.double() - exp).abs().max().item()
        assert err <= 1e-5 * (exp.abs().max().item() + 1.0), f"{name}: {err}"


@pytest.mark.parametrize("rows,cols", [(30720, 512), (3200, 512), (3200, 2576), (777, 260), (512, 4), (100000, 12)])
def test_colsum_matches_torch(rows, cols):
    """pdvc_colsum_f32 (the bias gradients) against a float64 column sum, ragged slabs and column tiles."""
    from pdvc.ops.functions.linear import colsum
    torch.manual_seed(rows + cols)
    x = torch.randn(rows, cols, device=DEV)
    got = colsum(x)
    exp = x.double().sum(0)
    err = (got.double() - exp).abs().max().item()
    assert err <= 1e-5 * (x.abs().sum(0).max().item() + 1.0), err
