"""GroupNorm on channels-last rows (csrc/groupnorm.hip) against torch's GroupNorm on the reference (N, C, T)
layout in float64: outputs and the gradients of x, weight, bias; ragged T (partial 64-row chunks) and
masked-like constant rows; and the whole channels-last base encoder on the GPU."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,T,C,G", [(3, 512, 512, 32), (2, 37, 512, 32), (4, 64, 256, 16), (1, 1, 512, 32),
                                     (2, 130, 128, 8)])
def test_groupnorm_rows_matches_torch(N, T, C, G):
    from pdvc.ops.functions.conv_rows import GroupNormRowsFunction
    torch.manual_seed(N * T + C)
    x = (torch.randn(N, T, C, device=DEV) * 3 + 1.5).requires_grad_()
    w = torch.rand(C, device=DEV).add_(0.5).requires_grad_()
    b = torch.randn(C, device=DEV).requires_grad_()
    y = GroupNormRowsFunction.apply(x, w, b, G, 1e-5)
    xd, wd, bd = (t.detach().double().requires_grad_() for t in (x, w, b))
    ref = F.group_norm(xd.transpose(1, 2), G, wd, bd, 1e-5).transpose(1, 2)
    assert (y.double() - ref).abs().max().item() < 2e-5
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g.double())
    for got, exp, name in ((x.grad, xd.grad, "dx"), (w.grad, wd.grad, "dw"), (b.grad, bd.grad, "db")):
        err = (got.double() - exp).abs().max().item()
        assert err <= 1e-4 * (exp.abs().max().item() + 1.0), f"{name}: {err}"


def test_base_encoder_rows_gpu_matches_reference_layout():
    from pdvc.base_encoder import BaseEncoder
    torch.manual_seed(0)
    enc = BaseEncoder(4, 768, 512).to(DEV)
    N, T = 3, 512
    vf = torch.randn(N, T, 768, device=DEV)
    mask = torch.zeros(N, T, dtype=torch.bool, device=DEV)
    dur = torch.tensor([100.0, 37.0, 12.0], device=DEV)
    srcs, _, _ = enc(vf, mask, dur)
    x = vf.double().transpose(1, 2)
    encd = BaseEncoder(4, 768, 512).to(DEV).double()
    encd.load_state_dict({k: v.double() for k, v in enc.state_dict().items()})
    ref = [encd.input_proj[0](x)]
    for lvl in range(1, 4):
        ref.append(encd.input_proj[lvl](x if lvl == 1 else ref[-1]))
    for s, r in zip(srcs, ref):
        assert (s.double() - r).abs().max().item() < 1e-4
