"""GPU parity of the fused encoder self-attention sub-layer (ops/functions/attn_block.py) against the module chain
it replaces (MSDeformAttn + output projection + residual layer norm, deformable_transformer.py:147-151), dropout
off: layer output and the gradients of src, pos and every parameter; and of the whole encoder with the
level-position gradient handle (ops/functions/posembed.py) against the per-level position path."""
import pytest
import torch
from parity import assert_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


def close(a, b, tol, what):
    """Per-tensor relative bound: max|a - b| <= tol * max|b| + 1e-7 (tests/parity.py)."""
    assert_close(a, b, what, tol)


def _layer(d, heads):
    from pdvc.deformable_transformer import DeformableTransformerEncoderLayer
    layer = DeformableTransformerEncoderLayer(d, 2 * d, 0.0, "relu", 4, heads, 4).to(DEV).train()
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.05 * torch.randn_like(p))
    return layer


@pytest.mark.parametrize("d,heads,masked", [(512, 8, False), (256, 8, True)])
def test_encoder_attn_block_matches_module_chain(d, heads, masked, monkeypatch):
    from pdvc.deformable_transformer import DeformableTransformerEncoder
    torch.manual_seed(d)
    level_T = (64, 32, 16, 8)
    S = sum(level_T)
    N = 2
    layer = _layer(d, heads)
    src = torch.randn(N, S, d, device=DEV)
    pos = torch.randn(N, S, d, device=DEV)
    valid = torch.ones(N, 4, device=DEV)
    mask = None
    if masked:
        mask = torch.zeros(N, S, dtype=torch.bool, device=DEV)
        mask[1, 50:64] = True
        valid[1] = torch.tensor([50 / 64, 25 / 32, 13 / 16, 7 / 8], device=DEV)
    ref_pts = DeformableTransformerEncoder.get_reference_points(level_T, valid, DEV)
    lsi = torch.tensor([0, 64, 96, 112], device=DEV)
    g = torch.randn(N, S, d, device=DEV)
    results = []
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(type(layer), "block_ok", lambda self, s: False)
        a, b = src.clone().requires_grad_(), pos.clone().requires_grad_()
        layer.zero_grad(set_to_none=True)
        out = layer(a, b, ref_pts, level_T, lsi, mask)
        out.backward(g)
        results.append((out.detach(), a.grad, b.grad, {n: p.grad.clone() for n, p in layer.named_parameters()}))
    (o1, gs1, gp1, pg1), (o2, gs2, gp2, pg2) = results
    close(o1, o2, 1e-5, "out")
    close(gs1, gs2, 1e-4, "grad src")
    close(gp1, gp2, 1e-4, "grad pos")
    for n in pg2:
        close(pg1[n], pg2[n], 1e-4, n)


def test_encoder_with_level_position_handle_matches_per_level_path(monkeypatch):
    """prepare_encoder_inputs + encoder: handle path (position gradients returned as per-(video, level) sums)
    vs the materialised position gradient, on the level embedding and the duration embedding layer."""
    import torch.nn.functional as F
    from pdvc.deformable_transformer import DeformableTransformer, DeformableTransformerEncoderLayer
    from pdvc.position_encoding import PositionEmbeddingSine, PyramidPosEmbed
    torch.manual_seed(1)
    d, N, T = 512, 2, 64
    tr = DeformableTransformer(d_model=d, nhead=8, num_encoder_layers=2, num_decoder_layers=1, dim_feedforward=1024,
                               dropout=0.0, activation="relu", return_intermediate_dec=True, num_feature_levels=4,
                               dec_n_points=4, enc_n_points=4).to(DEV).train()
    pe = PositionEmbeddingSine(d // 2, normalize=True).to(DEV)
    mask = torch.zeros(N, T, dtype=torch.bool, device=DEV)
    mask[1, 48:] = True
    masks, srcs = [mask], []
    Tl = T
    for lvl in range(4):
        if lvl:
            Tl = (Tl + 1) // 2
            masks.append(F.interpolate(mask[None].float(), size=(Tl,)).to(torch.bool)[0])
        srcs.append(torch.randn(N, d, Tl, device=DEV))
    dur = torch.tensor([80.0, 31.0], device=DEV)
    results = []
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(DeformableTransformerEncoderLayer, "block_ok", lambda self, s: False)
        tr.zero_grad(set_to_none=True)
        pe.zero_grad(set_to_none=True)
        xs = [s.clone().requires_grad_() for s in srcs]
        pyr = PyramidPosEmbed(pe, masks, dur)
        src_flat, shapes, lsi, vr, lvl_pos, mask_flat = tr.prepare_encoder_inputs(xs, masks, pyr)
        assert hasattr(lvl_pos, "_pdvc_level_grad") == fused
        mem = tr.forward_encoder(src_flat, shapes, lsi, vr, lvl_pos, mask_flat)
        g = torch.randn(mem.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(7))
        mem.backward(g)
        grads = {"level_embed": tr.level_embed.grad.clone(), "dur.weight": pe.duration_embed_layer.weight.grad.clone()}
        grads.update({f"enc.{n}": p.grad.clone() for n, p in tr.encoder.named_parameters()})
        grads.update({f"src{i}": x.grad for i, x in enumerate(xs)})
        results.append((mem.detach(), grads))
    (m1, g1), (m2, g2) = results
    close(m1, m2, 1e-5, "memory")
    for n in g2:
        close(g1[n], g2[n], 1e-4, n)


def test_decoder_value_bias_from_level_sums(monkeypatch):
    """The decoder's value projections (MultiLinearFunction over the encoder memory) take their bias gradients
    from the row sums the fused deformable attention returns with the value gradient: the hand-over happens,
    and the bias gradients equal colsum over the value gradient."""
    from pdvc.ops.functions import linear as L
    from pdvc.ops.functions.linear import multi_dense
    from pdvc.ops.modules.ms_deform_attn import MSDeformAttn
    torch.manual_seed(3)
    N, T_l, Lq = 2, (64, 32, 16, 8), 50
    S = sum(T_l)
    layers = [MSDeformAttn(512, 4, 8, 4).to(DEV) for _ in range(2)]
    mem = torch.randn(N, S, 512, device=DEV, requires_grad=True)
    q = torch.randn(N, Lq, 512, device=DEV)
    ref = torch.rand(N, Lq, 4, 2, device=DEV)
    shapes, lsi = T_l, None
    g = torch.randn(N, Lq, 512, device=DEV)

    def run(handover):
        for m in layers:
            m.zero_grad(set_to_none=True)
        if not handover:
            monkeypatch.setattr(MSDA1dFunction_cls(), "backward", _strip_sums(MSDA1dFunction_cls().backward))
        vals = multi_dense(mem, [m.value_proj for m in layers])
        out = sum(m(q, ref, mem, shapes, lsi, None, value=v) for m, v in zip(layers, vals))
        before = L.LEVEL_SUM_USES[0]
        (out * g).sum().backward()
        return L.LEVEL_SUM_USES[0] - before, [m.value_proj.bias.grad.clone() for m in layers]

    used, gb1 = run(True)
    assert used == 2
    used0, gb0 = run(False)
    assert used0 == 0
    for a, b in zip(gb1, gb0):
        assert (a - b).abs().max().item() <= 1e-4 * (b.abs().max().item() + 1.0)


def MSDA1dFunction_cls():
    from pdvc.ops.functions.ms_deform_attn_func import MSDA1dFunction
    return MSDA1dFunction


def _strip_sums(bwd):
    def backward(ctx, grad_out):
        res = bwd(ctx, grad_out)
        gv = res[0]
        if gv is not None and hasattr(gv, "_pdvc_level_sums"):
            gv = gv.clone()
        return (gv,) + tuple(res[1:])
    return staticmethod(backward)
