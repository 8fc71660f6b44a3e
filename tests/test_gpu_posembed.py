"""GPU parity of the fused encoder positional input (csrc/posembed.hip, ops/functions/posembed.py) against the
reference's per-level computation (position_encoding.py:20-75 + level_embed + cat over levels,
deformable_transformer.py:100-112) in torch: forward values, level-embedding and duration-embedding gradients,
with padded videos (the mask changes the normalised positions)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,T,F_", [(3, 512, 256), (2, 100, 128), (5, 37, 64)])
def test_level_pos_rows_matches_per_level_torch(N, T, F_):
    import torch.nn.functional as F
    from pdvc.ops.functions.posembed import level_pos_rows
    from pdvc.position_encoding import PositionEmbeddingSine, PyramidPosEmbed
    torch.manual_seed(T)
    pe = PositionEmbeddingSine(F_, normalize=True).to(DEV)
    d = F_ + pe.max_duration  # sine features + the 256 duration channels
    mask = torch.zeros(N, T, dtype=torch.bool, device=DEV)
    mask[1, T - T // 3:] = True
    if N > 2:
        mask[2, T // 2:] = True
    masks = [mask]
    for lvl in range(1, 4):
        Tl = (masks[-1].shape[1] + 1) // 2
        masks.append(F.interpolate(mask[None].float(), size=(Tl,)).to(torch.bool)[0])
    dur = torch.tensor([100.0, 37.0, 12.5, 3.0, 250.0][:N], device=DEV)
    level_embed = torch.randn(4, d, device=DEV, requires_grad=True)
    pyr = PyramidPosEmbed(pe, masks, dur)
    got = level_pos_rows(pyr, level_embed)
    ref = torch.cat([pyr[l].transpose(1, 2) + level_embed[l] for l in range(4)], 1)
    assert got.shape == ref.shape
    err = (got - ref).abs().max().item()
    assert err <= 2e-6, err
    g = torch.randn_like(ref)
    params = [level_embed] + list(pe.duration_embed_layer.parameters())
    ga = torch.autograd.grad(got, params, g)
    gb = torch.autograd.grad(ref, params, g)
    for a, b, name in zip(ga, gb, ("level_embed", "dur.weight", "dur.bias")):
        e = (a - b).abs().max().item()
        assert e <= 1e-4 * (1 + b.abs().max().item()), f"{name}: {e}"


def _golden_pyramid(dev):
    """The reference-generated positional input (tests/golden/make_golden.py::posembed) and our modules loaded
    with its parameters: PositionEmbeddingSine(256, normalize=True), the nearest-interpolated level masks."""
    import os
    import numpy as np
    import torch.nn.functional as F
    from pdvc.position_encoding import PositionEmbeddingSine, PyramidPosEmbed
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "posembed_levels.npz"))
    pe = PositionEmbeddingSine(256, normalize=True).to(dev)
    with torch.no_grad():
        pe.duration_embed_layer.weight.copy_(torch.from_numpy(z["dur_w"]))
        pe.duration_embed_layer.bias.copy_(torch.from_numpy(z["dur_b"]))
    mask = torch.from_numpy(z["mask"]).to(dev)
    masks = [mask] + [F.interpolate(mask[None].float(), size=(int(t),)).to(torch.bool)[0] for t in z["level_T"][1:]]
    pyr = PyramidPosEmbed(pe, masks, torch.from_numpy(z["duration"]).to(dev))
    return pyr, torch.from_numpy(z["level_embed"]).to(dev), torch.from_numpy(z["lvl_pos"]).to(dev)


def test_level_pos_rows_matches_reference_fixture():
    """The fused kernel against the reference's own PositionEmbeddingSine + level_embed + cat (pinned)."""
    from pdvc.ops.functions.posembed import level_pos_rows
    pyr, level_embed, want = _golden_pyramid(DEV)
    got = level_pos_rows(pyr, level_embed)
    assert got.shape == want.shape
    err = (got - want).abs().max().item()
    assert err <= 1e-5, err


def test_level_pos_add_matches_materialised_sum():
    """LevelPos.add_to (the position rows generated inside the add, pdvc_level_pos_rows_add_f32) is bit-exact
    against src + the materialised lvl_pos, and materialize() against level_pos_rows; on the reference fixture."""
    from pdvc.ops.functions.posembed import level_pos_rows, level_pos_rows_split
    pyr, level_embed, _ = _golden_pyramid(DEV)
    full = level_pos_rows(pyr, level_embed)
    lazy, handle = level_pos_rows_split(pyr, level_embed)
    assert lazy._pdvc_level_grad is handle and tuple(lazy.shape) == tuple(full.shape)
    assert torch.equal(lazy.materialize(), full)
    src = torch.randn(full.shape, device=DEV)
    assert torch.equal(lazy.add_to(src), src + full)
    rows = src.view(-1, full.shape[-1])
    assert torch.equal(lazy.add_to(rows), (src + full).view(-1, full.shape[-1]))
