"""GPU: destination-sorted row sums (csrc/rowsum.hip, pdvc_sorted_row_sums_f32) and the caption head's word-gate table
(LSTM_DSA._WordTable) built on them.

  * the row sums against float64 index_add over a stable sort of the keys: empty runs written as zeros, keys outside
    [0, n_dst) ignored, strided source rows, a skewed key (half the rows on one word); bit-identical across runs;
  * _WordTable (xe = W_x embed(idx) as rows of the batch's (V + 1) x 4H table, backward through the sorted sums)
    against the per-position form (embedding rows + GEMM): xe within fp32 GEMM rounding, the gradients of the
    embedding and of W_ih within 1e-5 of their scale, and the backward deterministic.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _row_sums(src, keys_flat, n_dst):
    from pdvc import _native as _n
    keys, order = torch.sort(keys_flat, stable=True)
    dst = torch.full((n_dst, src.shape[1]), float("nan"), device=DEV)
    ws = torch.full((int(_n.lib().pdvc_sorted_row_sums_workspace(keys_flat.numel(), src.shape[1])) + 4,), float("nan"),
                    device=DEV)
    _n.call("pdvc_sorted_row_sums_f32", _n.ptr_any(src), src.stride(0), src.shape[1], _n.ptr(keys), _n.ptr(order),
            keys_flat.numel(), n_dst, _n.ptr(dst), dst.stride(0), _n.ptr(ws), _n.stream())
    return dst


@pytest.mark.parametrize("n,cols,n_dst,lead", [(114688, 2048, 5749, 0), (1000, 36, 50, 8), (7, 256, 11, 0),
                                               (0, 64, 5, 0), (4096, 300, 3, 4), (129, 64, 1, 0)])
def test_sorted_row_sums_match_index_add(n, cols, n_dst, lead):
    g = torch.Generator(device=DEV).manual_seed(n + cols)
    base = torch.randn(n, cols + lead, device=DEV, generator=g)
    src = base[:, :cols]
    keys = torch.randint(0, n_dst, (n,), device=DEV, generator=g)
    empty = n >= 1000 and n_dst > 8
    if n >= 1000:
        keys[: n // 2] = min(3, n_dst - 1)       # one heavy word: a run over many 64-position chunks
        keys[n // 2: n // 2 + 5] = n_dst + 4     # out of range: ignored
        keys[n // 2 + 5: n // 2 + 9] = -1
    if empty:
        keys[keys == 7] = 8                      # an empty run
    dst = _row_sums(src, keys, n_dst)
    ok = (keys >= 0) & (keys < n_dst)
    ref = torch.zeros(n_dst, cols, dtype=torch.float64, device=DEV).index_add_(0, keys[ok], src[ok].double())
    scale = torch.zeros(n_dst, cols, dtype=torch.float64, device=DEV).index_add_(0, keys[ok], src[ok].double().abs())
    assert not torch.isnan(dst).any(), "every destination row is written"
    assert float(((dst.double() - ref).abs() / scale.clamp_min(1e-30)).max()) < 1e-5
    if empty:
        assert float(dst[7].abs().max()) == 0.0
    assert torch.equal(dst, _row_sums(src, keys, n_dst)), "deterministic"


def test_word_table_matches_per_position_gates(monkeypatch):
    import pdvc.CaptioningHead.LSTM_DSA as L
    torch.manual_seed(0)
    V, E, H4, n, R = 5749, 512, 2048, 14, 512
    emb = torch.nn.Embedding(V, E).to(DEV)
    W_ih = torch.nn.Parameter(torch.randn(H4, 3 * E, device=DEV) * E ** -0.5)
    idx = torch.randint(0, V, (n, R), device=DEV)
    idx[:, :64] = 0                                  # the end / padding word, frequent
    g = torch.randn(n, R, H4, device=DEV)

    def run(table):
        emb.zero_grad()
        W_ih.grad = None
        W_x = W_ih[:, :E]
        if table:
            xe = L._WordTable.apply(emb.weight, W_x, idx.contiguous())
        else:
            xe = torch.nn.functional.linear(emb(idx), W_x)
        xe.backward(g)
        return xe.detach(), emb.weight.grad.clone(), W_ih.grad.clone()

    x1, de1, dw1 = run(True)
    x0, de0, dw0 = run(False)
    torch.testing.assert_close(x1, x0, rtol=1e-5, atol=1e-5)
    assert float((de1 - de0).abs().max()) <= 1e-5 * (float(de0.abs().max()) + 1.0)
    assert float((dw1 - dw0).abs().max()) <= 1e-5 * (float(dw0.abs().max()) + 1.0)
    x2, de2, dw2 = run(True)
    assert torch.equal(de1, de2) and torch.equal(dw1, dw2), "the table's backward is deterministic"


@pytest.mark.parametrize("table", [True, False])
def test_word_gates_over_listed_positions_gpu(table, monkeypatch):
    """_WordGates on the GPU (the packed-token stream's word gates): the table form (rows of the batch's word-gate
    table, the listed positions' gradients summed per word, padding entries keyed past the table) and the
    per-position form both equal the full autograd backward when the gate gradient is zero off the listed
    positions; fp32 operands, float64 reference, bound 1e-5 of each gradient's scale."""
    import torch.nn.functional as F
    import pdvc.CaptioningHead.LSTM_DSA as L
    monkeypatch.setattr(L, "WORD_TABLE", table)
    g = torch.Generator(device=DEV).manual_seed(5)
    n, R, V, E, G = 13, 640, 5749, 512, 2048
    idx = torch.randint(0, V, (n, R), device=DEV, generator=g)
    idx[0] = 0
    weight = torch.randn(V, E, device=DEV, generator=g).requires_grad_()
    W_ih = torch.randn(G, 2 * E, device=DEV, generator=g).mul_(E ** -0.5).requires_grad_()
    keep = torch.rand(n, R, device=DEV, generator=g) < 0.5
    up = torch.randn(n, R, G, device=DEV, generator=g) * keep[..., None]
    wd, Wd = weight.detach().double().requires_grad_(), W_ih.detach().double().requires_grad_()
    ref_out = F.linear(wd[idx], Wd[:, :E])
    ref = torch.autograd.grad((ref_out * up.double()).sum(), (wd, Wd))
    act = torch.nonzero(keep.reshape(-1)).view(-1)
    act = torch.cat([act, torch.full((5,), n * R, device=DEV)])
    out = L._WordGates.apply(weight, W_ih[:, :E], idx, act)
    assert float((out.detach().double() - ref_out.detach()).abs().max()) <= 1e-5 * float(ref_out.detach().abs().max())
    got = torch.autograd.grad((out * up).sum(), (weight, W_ih))
    for a, e in zip(got, ref):
        assert float((a.double() - e).abs().max()) <= 1e-5 * (float(e.abs().max()) + 1.0)
