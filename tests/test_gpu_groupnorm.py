"""GroupNorm on channels-last rows (csrc/groupnorm.hip) against torch's GroupNorm on the reference (N, C, T)
layout in float64: outputs and the gradients of x, weight, bias; ragged T (partial 64-row chunks) and
masked-like constant rows; and the whole channels-last base encoder on the GPU."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,T,C,G", [(3, 512, 512, 32), (2, 37, 512, 32), (4, 64, 256, 16), (1, 1, 512, 32),
                                     (2, 130, 128, 8), (2, 100, 512, 8), (2, 600, 512, 32), (2, 64, 32, 8)])
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


@pytest.mark.parametrize("T", [512, 37])
def test_base_encoder_flat_buffer_matches_per_level(T, monkeypatch):
    """The levels written straight into one flattened buffer (GroupNormFlatFunction) against the per-level path
    plus torch.cat: values and every gradient (x, conv and GroupNorm parameters), ragged T included."""
    from pdvc.base_encoder import BaseEncoder
    torch.manual_seed(T)
    enc = BaseEncoder(4, 768, 512).to(DEV)
    for p in enc.parameters():  # non-trivial GroupNorm affine parameters
        if p.dim() == 1:
            p.data.normal_()
    N = 3
    vf = torch.randn(N, T, 768, device=DEV)
    mask = torch.zeros(N, T, dtype=torch.bool, device=DEV)
    dur = torch.tensor([100.0, 37.0, 12.0], device=DEV)

    def run(flat_path):
        monkeypatch.setattr(BaseEncoder, "_flat_ok", lambda self, x: flat_path)
        enc.zero_grad(set_to_none=True)
        x = vf.clone().requires_grad_()
        srcs, _, _ = enc(x, mask, dur)
        if flat_path:
            assert all(hasattr(s, "_pdvc_flat") for s in srcs)
            flat = srcs[0]._pdvc_flat[0]
        else:
            flat = torch.cat([s.transpose(1, 2) for s in srcs], 1)
        g = torch.randn(flat.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(1))
        (flat * g).sum().backward()
        return flat.detach(), x.grad, {k: p.grad.clone() for k, p in enc.input_proj.named_parameters()}

    f1, dx1, gp1 = run(True)
    f0, dx0, gp0 = run(False)
    assert f1.shape == f0.shape
    assert (f1 - f0).abs().max().item() == 0.0
    assert (dx1 - dx0).abs().max().item() <= 1e-5 * (dx0.abs().max().item() + 1.0)
    for k in gp0:
        err = (gp1[k] - gp0[k]).abs().max().item()
        assert err <= 1e-5 * (gp0[k].abs().max().item() + 1.0), (k, err)


@pytest.mark.parametrize("N,T", [(64, 512), (5, 37), (1, 256)])
def test_conv_s2_tap_epilogue_matches_conv1d(N, T, monkeypatch):
    """The stride-2 conv with its previous-odd-row tap accumulated in a GEMM epilogue over the shifted rows (each
    video's row 0 restored: its tap is the zero padding) against nn.Conv1d in float64 and against the separate
    product + add (PDVC_CONV_TAP_EPILOGUE=0), every product on gemm3 (MIN_ROWS = 0); ragged T and N = 1 included."""
    import pdvc.ops.functions.gemm3 as G
    import pdvc.ops.functions.conv_rows as CR
    monkeypatch.setattr(G, "MIN_ROWS", 0)
    torch.manual_seed(N + T)
    C, O = 512, 512
    x = torch.randn(N, T, C, device=DEV)
    w = torch.randn(O, C, 3, device=DEV) * C ** -0.5
    b = torch.randn(O, device=DEV)
    g = torch.randn(N, (T + 1) // 2, O, device=DEV)
    outs = {}
    for tap in (True, False):
        monkeypatch.setattr(CR, "_TAP_EPILOGUE", tap)
        xx, ww, bb = (t.clone().requires_grad_() for t in (x, w, b))
        y = CR.ConvS2RowsFunction.apply(xx, ww, bb)
        y.backward(g)
        outs[tap] = (y.detach(), xx.grad, ww.grad, bb.grad)
    ref = F.conv1d(x.double().transpose(1, 2), w.double(), b.double(), stride=2, padding=1).transpose(1, 2)
    scale = F.conv1d(x.double().abs().transpose(1, 2), w.double().abs(), b.double().abs(), stride=2,
                     padding=1).transpose(1, 2)
    for tap in (True, False):
        assert float(((outs[tap][0].double() - ref).abs() / scale).max()) < 1e-6, tap
    torch.testing.assert_close(outs[True][0], outs[False][0], rtol=1e-6, atol=1e-5)
    for a, c in zip(outs[True][1:], outs[False][1:]):
        assert torch.equal(a, c), "the backward does not depend on the forward's form"


def test_groupnorm_single_pass_forms_serve_the_pyramid_shapes():
    """The single-pass kernels (pdvc_groupnorm_rows_*_fused_f32) take every base-encoder level shape (T <= 512, C = 512,
    32 groups) and refuse the rest (T > 512, C not a multiple of 64) with nothing written, so the chunked forms run
    there; the backward's (N, 2C) partials sum to [dgamma | dbeta]."""
    from pdvc import _native as _n
    torch.manual_seed(1)
    for T, C, ok in ((512, 512, True), (64, 512, True), (513, 512, False), (64, 32, False)):
        N, G = 2, 32 if C == 512 else 8
        x = torch.randn(N, T, C, device=DEV)
        w, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
        y = torch.full_like(x, 7.0)
        mean, rstd = torch.empty(N * G, device=DEV), torch.empty(N * G, device=DEV)
        args = (_n.ptr(x), N, T, C, G, 1e-5, _n.ptr(w), _n.ptr(b), _n.ptr(y), T * C, None, _n.ptr(mean), _n.ptr(rstd),
                None, _n.stream())
        if not ok:
            with pytest.raises(_n.NativeError):
                _n.call("pdvc_groupnorm_rows_forward_fused_f32", *args)
            assert bool((y == 7.0).all())
            continue
        _n.call("pdvc_groupnorm_rows_forward_fused_f32", *args)
        ref = F.group_norm(x.double().transpose(1, 2), G, w.double(), b.double(), 1e-5).transpose(1, 2)
        assert (y.double() - ref).abs().max().item() < 2e-5
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        cp = torch.empty(N, 2 * C, device=DEV)
        _n.call("pdvc_groupnorm_rows_backward_fused_f32", _n.ptr(x), _n.ptr(dy), T * C, None, _n.ptr(mean),
                _n.ptr(rstd), _n.ptr(w), N, T, C, G, _n.ptr(cp), _n.ptr(dx), _n.stream())
        xh = ((x.double().view(N, T, G, -1) - mean.double().view(N, 1, G, 1)) * rstd.double().view(N, 1, G, 1))
        dg = (dy.double() * xh.view(N, T, C)).sum((0, 1))
        db = dy.double().sum((0, 1))
        got = cp.double().sum(0)
        assert (got[:C] - dg).abs().max().item() <= 1e-4 * (dg.abs().max().item() + 1.0)
        assert (got[C:] - db).abs().max().item() <= 1e-4 * (db.abs().max().item() + 1.0)


@pytest.mark.parametrize("N,T", [(64, 512), (5, 37), (1, 256), (3, 64)])
def test_conv_s2_backward_on_shifted_views(N, T, monkeypatch):
    """The stride-2 conv's backward on row-shifted views (conv_rows.py _backward_views: no shifted copy of dy; the
    W0 tap's cross-video pairs restored / subtracted) against nn.Conv1d's gradients in float64 and against the
    shifted-copy backward (PDVC_CONV_SHIFT_VIEWS=0), every product on gemm3 (MIN_ROWS = 0); ragged T, N = 1 included
    (shapes whose N * ceil(T/2) rows are not a multiple of 32 take the copy form)."""
    import pdvc.ops.functions.gemm3 as G
    import pdvc.ops.functions.conv_rows as CR
    monkeypatch.setattr(G, "MIN_ROWS", 0)
    torch.manual_seed(N * 7 + T)
    C, O = 512, 512
    x = torch.randn(N, T, C, device=DEV)
    w = torch.randn(O, C, 3, device=DEV) * C ** -0.5
    b = torch.randn(O, device=DEV)
    g = torch.randn(N, (T + 1) // 2, O, device=DEV)
    got = {}
    for views in (True, False):
        monkeypatch.setattr(CR, "_SHIFT_VIEWS", views)
        xx, ww, bb = (t.clone().requires_grad_() for t in (x, w, b))
        CR.ConvS2RowsFunction.apply(xx, ww, bb).backward(g)
        got[views] = (xx.grad, ww.grad, bb.grad)
    xd, wd, bd = (t.double().requires_grad_() for t in (x, w, b))
    F.conv1d(xd.transpose(1, 2), wd, bd, stride=2, padding=1).transpose(1, 2).backward(g.double())
    for views in (True, False):
        for a, r, name in zip(got[views], (xd.grad, wd.grad, bd.grad), ("dx", "dw", "db")):
            err = (a.double() - r).abs().max().item()
            assert err <= 1e-5 * (r.abs().max().item() + 1.0), (views, name, err)
    for a, c in zip(got[True], got[False]):
        assert (a - c).abs().max().item() <= 1e-5 * (c.abs().max().item() + 1.0)
