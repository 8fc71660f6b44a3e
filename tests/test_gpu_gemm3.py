"""GPU: the fp32 GEMM on the bf16 matrix cores (csrc/gemm3.hip, pdvc/ops/functions/gemm3.py).

Each fp32 operand is split exactly into three bf16 terms (x = x0 + x1 + x2) and the six products of order >= 2^-16
are accumulated in fp32 (the dropped terms are <= 2^-23 |a||b| per product).  The tests check:
  * the split is exact (the three planes sum to the fp32 value, bit for bit, over 80 binades);
  * every entry point and layout against float64 -- the per-element error scaled by sum_k |a_k||b_k| below 1e-6 and
    at most twice hipBLASLt's fp32 error on the same operands (tolerance stated here: the products' own rounding
    is 2^-24 ~ 6e-8 of that scale; K-deep fp32 accumulation adds ~sqrt(K) of it);
  * epilogues (bias, ReLU, accumulate), ragged M / N, strided rows, split-K determinism, argument errors;
  * the encoder nodes and the whole batched training step with every eligible product on gemm3 (MIN_ROWS = 0)
    against the same references as their hipBLASLt runs (tests/parity.py bound, the reference fixture).
"""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib():
    from pdvc import _native as _n
    return _n


def scaled_err(c, ref, scale):
    return float(((c.double() - ref).abs() / scale.clamp_min(1e-300)).max())


def gemm3(M, N, K, A, lda, akc, B, ldb, bkc, C, ldc, bias=None, epi=0, splits=1, ws=None):
    _n = _lib()
    _n.call("pdvc_gemm3_f32", M, N, K, _n.ptr_any(A), lda, akc, _n.ptr_any(B), ldb, bkc, _n.ptr_any(C), ldc,
            _n.ptr(bias), epi, splits, None if ws is None else _n.ptr(ws), _n.stream())


def op_mat(X, kc, rows, cols):
    """The logical (rows, cols) operand of a stored matrix: kc -> X is (rows, ld); else X is (cols, ld) transposed."""
    return X[:rows, :cols] if kc else X[:cols, :rows].t()


def test_split_planes_are_exact():
    from pdvc.ops.functions.gemm3 import split_planes
    torch.manual_seed(0)
    N, K = 96, 128
    W = torch.randn(N, K, device=DEV) * torch.exp2(torch.randint(-40, 40, (N, K), device=DEV).float())
    for kc in (1, 0):
        src = W if kc else W.t().contiguous()
        planes = split_planes(src, kc, N, K)
        bits = planes.view(3, N, K).cpu().numpy().view("uint16").astype("uint32") << 16
        vals = torch.from_numpy(bits.view("float32")).double()
        recon = vals.sum(0)
        assert torch.equal(recon, W.cpu().double()), "x0 + x1 + x2 must equal x exactly"
        assert float((vals[1].abs() - vals[0].abs() * 2.0 ** -8).clamp_min(0).max()) == 0.0
        assert float((vals[2].abs() - vals[0].abs() * 2.0 ** -16).clamp_min(0).max()) == 0.0


CASES = [  # (M, N, K, a_kc, b_kc, epi)
    (4096, 512, 512, 1, 1, 1),
    (1000, 200, 96, 1, 1, 2),
    (4100, 512, 256, 1, 0, 0),
    (300, 64, 1536, 1, 0, 3),
    (512, 256, 4096, 0, 0, 0),
    (260, 132, 64, 0, 1, 3),
]


@pytest.mark.parametrize("M,N,K,akc,bkc,epi", CASES)
def test_gemm3_matches_float64(M, N, K, akc, bkc, epi):
    torch.manual_seed(M + N + K)
    lda = (K if akc else M) + 8
    ldb = (K if bkc else N) + 4
    A = torch.randn((M if akc else K), lda, device=DEV)
    B = torch.randn((N if bkc else K), ldb, device=DEV)
    a, b = op_mat(A, akc, M, K), op_mat(B, bkc, N, K)
    bias = torch.randn(N, device=DEV)
    C0 = torch.randn(M, N + 12, device=DEV)
    C = C0.clone()
    gemm3(M, N, K, A, lda, akc, B, ldb, bkc, C, N + 12, bias if epi in (1, 2) else None, epi)
    ref = a.double() @ b.double().t()
    scale = a.double().abs() @ b.double().abs().t()
    theirs = a @ b.t()
    if epi in (1, 2):
        ref, theirs, scale = ref + bias.double(), theirs + bias, scale + bias.double().abs()
    if epi == 2:
        ref, theirs = ref.clamp_min(0), theirs.clamp_min(0)
    if epi == 3:
        ref, theirs, scale = ref + C0[:, :N].double(), theirs + C0[:, :N], scale + C0[:, :N].double().abs()
    ours_e = scaled_err(C[:, :N], ref, scale)
    blas_e = scaled_err(theirs, ref, scale)
    assert ours_e < 1e-6 and ours_e <= 2 * blas_e + 1e-8, (ours_e, blas_e)
    assert torch.equal(C[:, N:], C0[:, N:]), "columns past N must be untouched"


@pytest.mark.parametrize("M,N,K,bkc,epi", [(4096, 512, 512, 1, 1), (3000, 200, 96, 1, 2), (2500, 512, 256, 0, 3),
                                           (700, 100, 64, 0, 0)])
def test_gemm3p_matches_float64(M, N, K, bkc, epi):
    from pdvc.ops.functions.gemm3 import split_planes
    _n = _lib()
    torch.manual_seed(M + K)
    A = torch.randn(M, K + 4, device=DEV)
    Bst = torch.randn((N, K) if bkc else (K, N), device=DEV)
    b = Bst if bkc else Bst.t()
    a = A[:, :K]
    bias = torch.randn(N, device=DEV)
    C0 = torch.randn(M, N, device=DEV)
    C = C0.clone()
    planes = split_planes(Bst, bkc, N, K)
    _n.call("pdvc_gemm3p_f32", M, N, K, _n.ptr_any(A), K + 4, _n.ptr(planes), _n.ptr(C), N,
            _n.ptr(bias) if epi in (1, 2) else None, epi, _n.stream())
    ref = a.double() @ b.double().t()
    scale = a.double().abs() @ b.double().abs().t()
    theirs = a @ b.t()
    if epi in (1, 2):
        ref, theirs, scale = ref + bias.double(), theirs + bias, scale + bias.double().abs()
    if epi == 2:
        ref, theirs = ref.clamp_min(0), theirs.clamp_min(0)
    if epi == 3:
        ref, theirs, scale = ref + C0.double(), theirs + C0, scale + C0.double().abs()
    ours_e = scaled_err(C, ref, scale)
    blas_e = scaled_err(theirs, ref, scale)
    assert ours_e < 1e-6 and ours_e <= 2 * blas_e + 1e-8, (ours_e, blas_e)


@pytest.mark.parametrize("M,N,K,bkc,epi", [(4096, 512, 512, 1, 1), (3000, 200, 96, 1, 2), (2500, 512, 256, 0, 3),
                                           (700, 100, 64, 0, 0)])
def test_gemm1p_is_the_bf16_operand_product(M, N, K, bkc, epi):
    """pdvc_round_plane_f32 + pdvc_gemm1p_f32 (the bf16 mode's product): the plane is torch's RNE rounding bit for
    bit, and C is the float64 product of the bf16-rounded operands up to fp32 accumulation (each bf16 x bf16 product
    is exact in fp32; bound 1e-6 of sum_k |a||b|, as gemm3), and within the same bound of hipBLASLt's bf16 GEMM."""
    _n = _lib()
    torch.manual_seed(M + K + 1)
    A = torch.randn(M, K + 4, device=DEV)
    Bst = torch.randn((N, K) if bkc else (K, N), device=DEV)
    b = Bst if bkc else Bst.t()
    a = A[:, :K]
    bias = torch.randn(N, device=DEV)
    C0 = torch.randn(M, N, device=DEV)
    C = C0.clone()
    plane = torch.empty((N, K), dtype=torch.int16, device=DEV)
    _n.call("pdvc_round_plane_f32", _n.ptr_any(Bst), Bst.stride(0), bkc, N, K, _n.ptr(plane), _n.stream())
    assert torch.equal(plane.view(torch.bfloat16), b.to(torch.bfloat16))
    _n.call("pdvc_gemm1p_f32", M, N, K, _n.ptr_any(A), K + 4, _n.ptr(plane), _n.ptr(C), N,
            _n.ptr(bias) if epi in (1, 2) else None, epi, _n.stream())
    a16, b16 = a.to(torch.bfloat16), b.to(torch.bfloat16)
    ref = a16.double() @ b16.double().t()
    scale = a16.double().abs() @ b16.double().abs().t()
    theirs = torch.ops.aten.mm.dtype(a16, b16.t(), torch.float32)
    if epi in (1, 2):
        ref, theirs, scale = ref + bias.double(), theirs + bias, scale + bias.double().abs()
    if epi == 2:
        ref, theirs = ref.clamp_min(0), theirs.clamp_min(0)
    if epi == 3:
        ref, theirs, scale = ref + C0.double(), theirs + C0, scale + C0.double().abs()
    assert scaled_err(C, ref, scale) < 1e-6
    assert float(((C - theirs).abs().double() / scale.clamp_min(1e-300)).max()) < 1e-6


def test_wgrad_split_is_deterministic_and_accurate():
    from pdvc.ops.functions.gemm3 import mm_wgrad
    torch.manual_seed(5)
    rows, O, I = 65536, 256, 512
    gy = torch.randn(rows, O, device=DEV)
    x = torch.randn(rows, I + 8, device=DEV)[:, :I]  # strided rows (the base encoder's X2[:, C:] view)
    import pdvc.ops.functions.gemm3 as G
    old = G.MIN_ROWS
    G.MIN_ROWS = 0
    try:
        w1 = mm_wgrad(gy, x)
        w2 = mm_wgrad(gy, x)
    finally:
        G.MIN_ROWS = old
    assert w1 is not None and torch.equal(w1, w2), "split-K weight gradient must be deterministic"
    ref = gy.double().t() @ x.double()
    scale = gy.double().abs().t() @ x.double().abs()
    assert scaled_err(w1, ref, scale) < 1e-6


@pytest.mark.parametrize("rows,O,I,lead", [(65536, 256, 512, 0), (4096, 132, 200, 8), (8192, 516, 64, 4),
                                           (96, 512, 512, 0)])
def test_wgrad_bias_is_the_column_sum(rows, O, I, lead):
    """pdvc_gemm3_wgrad_bias_f32 (mm_wgrad(..., db=)): dW as the plain weight-gradient launch, bit for bit, and db =
    gy.sum(0) within fp32 summation error of float64 (|err| <= 1e-6 sum |gy|: the rounding of a sum of `rows` terms
    in a fixed order is ~sqrt(rows) 2^-24 of it), deterministic; O not a multiple of the 256-wide tile, strided
    rows, one split (rows = 96) and many."""
    from pdvc.ops.functions.gemm3 import mm_wgrad
    import pdvc.ops.functions.gemm3 as G
    torch.manual_seed(rows + O)
    base = torch.randn(rows, O + lead, device=DEV)
    base[:, :O] *= torch.exp2(torch.randint(-6, 6, (O,), device=DEV).float())  # columns of different magnitudes
    gy = base[:, :O]
    x = torch.randn(rows, I + 4, device=DEV)[:, :I]
    old = G.MIN_ROWS
    G.MIN_ROWS = 0
    try:
        w0 = mm_wgrad(gy, x)
        db1 = torch.full((O,), float("nan"), device=DEV)
        w1 = mm_wgrad(gy, x, db=db1)
        db2 = torch.empty(O, device=DEV)
        mm_wgrad(gy, x, db=db2)
    finally:
        G.MIN_ROWS = old
    assert w0 is not None and torch.equal(w0, w1), "the fused bias sum must leave dW unchanged"
    assert torch.equal(db1, db2), "the bias sum must be deterministic"
    ref = gy.double().sum(0)
    assert float(((db1.double() - ref).abs() / gy.double().abs().sum(0)).max()) < 1e-6


def test_linear_bias_gradients_through_the_fused_wgrad(monkeypatch):
    """The nn.Linear backward (TorchLinearFunction) takes its bias gradient from the weight-gradient pass: dW
    unchanged, db within fp32 summation error of float64 (1e-6 of sum |gy|) as the separate colsum pass it replaces
    (PDVC_WGRAD_BIAS A/B switch)."""
    G = _on_gemm3(monkeypatch)
    from pdvc.ops.functions import linear as L
    torch.manual_seed(3)
    x = torch.randn(4096, 256, device=DEV, requires_grad=True)
    lin = torch.nn.Linear(256, 384).to(DEV)
    gy = torch.randn(4096, 384, device=DEV)
    grads = {}
    for fused in (True, False):
        monkeypatch.setattr(G, "WGRAD_BIAS", fused)
        lin.zero_grad()
        L.TorchLinearFunction.apply(x, lin.weight, lin.bias, False).backward(gy)
        grads[fused] = (lin.weight.grad.clone(), lin.bias.grad.clone())
    assert torch.equal(grads[True][0], grads[False][0])
    ref, scale = gy.double().sum(0), gy.double().abs().sum(0)  # fp32 sums in two orders: bound relative to sum |gy|
    for fused in (True, False):
        assert float(((grads[fused][1].double() - ref).abs() / scale).max()) < 1e-6


def test_gemm3_argument_errors():
    _n = _lib()
    A = torch.randn(64, 48, device=DEV)
    B = torch.randn(64, 48, device=DEV)
    C = torch.empty(64, 64, device=DEV)
    with pytest.raises(_n.NativeError, match="multiple of 32"):
        gemm3(64, 64, 48, A, 48, 1, B, 48, 1, C, 64)
    A2 = torch.randn(64 * 64 + 1, device=DEV)[1:].view(64, 64)  # 4-byte aligned, not 16
    with pytest.raises(_n.NativeError, match="16-byte"):
        gemm3(64, 64, 64, A2, 64, 1, A2, 64, 1, C, 64)
    with pytest.raises(_n.NativeError, match="workspace"):
        gemm3(64, 64, 64, C, 64, 1, C, 64, 1, torch.empty(64, 64, device=DEV), 64, None, 0, 2, None)


def _on_gemm3(monkeypatch):
    import pdvc.ops.functions.gemm3 as G
    monkeypatch.setattr(G, "MIN_ROWS", 0)
    monkeypatch.setattr(G, "ENABLED", True)
    return G


def test_ffn_block_on_gemm3(monkeypatch):
    G = _on_gemm3(monkeypatch)
    import test_gpu_ffn
    before = G.CALLS["gemm3"]
    test_gpu_ffn.test_ffn_block_matches_float64_chain(2048, 128, 512, 0.3)
    assert G.CALLS["gemm3"] >= before + 6, "the FFN's six products must run on gemm3"


def test_encoder_attn_block_on_gemm3(monkeypatch):
    G = _on_gemm3(monkeypatch)
    import test_gpu_attn_block
    before = G.CALLS["gemm3"]
    test_gpu_attn_block.test_encoder_attn_block_matches_module_chain(512, 8, False, monkeypatch)
    assert G.CALLS["gemm3"] >= before + 9


def test_batched_step_on_gemm3_equals_reference(monkeypatch):
    """The batched training step of the reference fixture (tests/test_gpu_batch.py) with every eligible product of
    the model on gemm3: the same per-tensor bound against the reference's batch-1 gradients."""
    G = _on_gemm3(monkeypatch)
    import test_gpu_batch as TB
    before = G.CALLS["gemm3"]
    TB.test_batched_step_equals_mean_of_reference_batch1_steps(TB.TM.load(TB.NAME))
    assert G.CALLS["gemm3"] > before + 20


def test_ffn_relu_dropout_epilogue_is_bit_identical(monkeypatch):
    """linear1's relu -> dropout in the gemm3 epilogue (pdvc_gemm3p_relu_dropout_f32) and its backward in linear2's
    data-gradient epilogue (pdvc_gemm3p_dmask_f32) against the GEMMs followed by the relu-dropout passes (ffn.py
    FUSE_RELU_DROPOUT off): the same mask bits and arithmetic, so the block's output and every gradient are
    bit-identical -- except linear1's bias gradient, the same column sums in another summation order; ragged rows."""
    _on_gemm3(monkeypatch)
    import pdvc.ops.functions.ffn as F
    from pdvc.ops.functions.ffn import FFNBlockFunction
    torch.manual_seed(3)
    rows, d, f, p = 3000, 256, 512, 0.3
    x = torch.randn(rows, d, device=DEV)
    lin1, lin2 = torch.nn.Linear(d, f).to(DEV), torch.nn.Linear(f, d).to(DEV)
    norm = torch.nn.LayerNorm(d).to(DEV)
    params = [lin1.weight, lin1.bias, lin2.weight, lin2.bias, norm.weight, norm.bias]
    seeds = torch.tensor([1234567, 7654321], dtype=torch.int64, device=DEV)
    g = torch.randn(rows, d, device=DEV)
    res = []
    for fuse in (True, False):
        monkeypatch.setattr(F, "FUSE_RELU_DROPOUT", fuse)
        xa = x.clone().requires_grad_()
        out = FFNBlockFunction.apply(xa, *params, p, 0.1, norm.eps, seeds)
        res.append([out.detach()] + list(torch.autograd.grad(out, [xa] + params, g)))
    for i, (a, b) in enumerate(zip(*res)):
        if i == 3:  # linear1's bias gradient: the column sums of the same dh, summed in another order
            assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()) + 1e-7
            continue
        assert torch.equal(a, b), f"tensor {i} differs between the fused epilogues and the separate passes"
    kept = (res[0][0] != 0).float().mean()  # sanity: dropout active
    assert kept > 0


@pytest.mark.parametrize("p_out", [0.0, 0.25])
def test_ffn_residual_sum_epilogue_is_bit_identical(monkeypatch, p_out):
    """x + dropout(linear2(h)) formed in linear2's gemm3 epilogue (pdvc_gemm3p_resid_dropout_f32) and the add-norm
    pass on that sum alone (s = NULL) against linear2 followed by the two-input add-norm pass (RESID_EPILOGUE off):
    the same mask bits and the same operations, so the block's output and every gradient are bit-identical;
    ragged rows; dropout off and on."""
    G = _on_gemm3(monkeypatch)
    from pdvc.ops.functions.ffn import FFNBlockFunction
    torch.manual_seed(5)
    rows, d, f = 3000, 256, 512
    x = torch.randn(rows, d, device=DEV)
    lin1, lin2 = torch.nn.Linear(d, f).to(DEV), torch.nn.Linear(f, d).to(DEV)
    norm = torch.nn.LayerNorm(d).to(DEV)
    with torch.no_grad():
        norm.weight.add_(0.1 * torch.randn_like(norm.weight))
        norm.bias.add_(0.1 * torch.randn_like(norm.bias))
    params = [lin1.weight, lin1.bias, lin2.weight, lin2.bias, norm.weight, norm.bias]
    seeds = torch.tensor([1234567, 7654321], dtype=torch.int64, device=DEV)
    g = torch.randn(rows, d, device=DEV)
    res = []
    for fuse in (True, False):
        monkeypatch.setattr(G, "RESID_EPILOGUE", fuse)
        calls = G.CALLS["gemm3"]
        xa = x.clone().requires_grad_()
        out = FFNBlockFunction.apply(xa, *params, 0.1, p_out, norm.eps, seeds)
        res.append([out.detach()] + list(torch.autograd.grad(out, [xa] + params, g)))
        assert G.CALLS["gemm3"] > calls
    for i, (a, b) in enumerate(zip(*res)):
        assert torch.equal(a, b), f"tensor {i} differs between the fused residual sum and the two-input pass"


@pytest.mark.parametrize("p", [0.0, 0.2])
def test_attn_block_residual_sum_epilogue_is_bit_identical(monkeypatch, p):
    """The encoder self-attention node with src + dropout(output_proj(...)) formed in output_proj's gemm3 epilogue
    against the two-input add-norm pass (dropout off and on): the layer output and every gradient that does not pass
    through the MSDA value-gradient walk bit-identical; the rest within 1e-5 of their scale (the walk's counting sort
    places a row's entries by LDS atomics, so its sums are not bitwise reproducible run to run either)."""
    from parity import assert_close
    G = _on_gemm3(monkeypatch)
    from pdvc.deformable_transformer import DeformableTransformerEncoder, DeformableTransformerEncoderLayer
    torch.manual_seed(9)
    d, heads, level_T, N = 256, 8, (64, 32, 16, 8), 2
    S = sum(level_T)
    layer = DeformableTransformerEncoderLayer(d, 2 * d, p, "relu", 4, heads, 4).to(DEV).train()
    src = torch.randn(N, S, d, device=DEV)
    pos = torch.randn(N, S, d, device=DEV)
    ref_pts = DeformableTransformerEncoder.get_reference_points(level_T, torch.ones(N, 4, device=DEV), DEV)
    lsi = torch.tensor([0, 64, 96, 112], device=DEV)
    g = torch.randn(N, S, d, device=DEV)
    res = []
    for fuse in (True, False):
        monkeypatch.setattr(G, "RESID_EPILOGUE", fuse)
        torch.manual_seed(77)  # the same dropout seeds drawn on the device for both runs
        a, b = src.clone().requires_grad_(), pos.clone().requires_grad_()
        layer.zero_grad(set_to_none=True)
        out = layer(a, b, ref_pts, level_T, lsi, None)
        out.backward(g)
        res.append([("out", out.detach()), ("src", a.grad), ("pos", b.grad)] +
                   [(n, q.grad.clone()) for n, q in layer.named_parameters()])
    exact = ("out", "self_attn.output_proj.weight", "self_attn.output_proj.bias", "norm1.weight", "norm1.bias",
             "linear1.weight", "linear1.bias", "linear2.weight", "linear2.bias", "norm2.weight", "norm2.bias")
    for (n, x1), (_, x2) in zip(*res):
        if n in exact:
            assert torch.equal(x1, x2), f"{n} differs between the fused residual sum and the two-input pass"
        else:
            assert_close(x1, x2, f"{n} (fused residual sum vs two-input pass)", 1e-5)


@pytest.mark.parametrize("accumulate", [None, False, True])
def test_dgrad_split_k_few_tiles_deep_reduction(monkeypatch, accumulate):
    """mm_dgrad on a product with few output tiles and a deep reduction (the caption logit layer's input gradient:
    rows x 512 over K = the padded vocabulary) takes the split-K generic kernel (dgrad_splits > 1): float64 bound as
    every gemm3 product, and deterministic (the slabs are summed in a fixed order)."""
    G = _on_gemm3(monkeypatch)
    torch.manual_seed(11)
    M, N, K = 3000, 512, 5760
    assert G.dgrad_splits(M, N, K) > 1
    dy = torch.randn(M, K, device=DEV)
    W = torch.randn(K, N, device=DEV) / K ** 0.5
    ref = dy.double() @ W.double()
    scale = dy.double().abs() @ W.double().abs()
    if accumulate is None:
        out = G.mm_dgrad(dy, W)
        again = G.mm_dgrad(dy, W)
        assert torch.equal(out, again), "split-K must be deterministic"
    else:
        base = torch.randn(M, N, device=DEV)
        out = base.clone()
        G.mm_dgrad(dy, W, out=out, accumulate=accumulate)
        if accumulate:
            ref, scale = ref + base.double(), scale + base.double().abs()
    assert scaled_err(out, ref, scale) < 1e-6


def test_addmm_generic_tile_when_gemm3p_waves_are_ragged(monkeypatch):
    """addmm_nt on a shape whose 256 x 256 tiles leave gemm3p's last wave mostly empty (8 192 x 2 816: 352 tiles)
    takes the generic 256 x 128 kernel (generic_wins): same float64 bound, bias and ReLU epilogues."""
    G = _on_gemm3(monkeypatch)
    torch.manual_seed(13)
    M, N, K = 8192, 2816, 512
    assert G.generic_wins(M, N, K) and not G.generic_wins(983040, 512, 512)
    x = torch.randn(M, K, device=DEV)
    W = torch.randn(N, K, device=DEV) / K ** 0.5
    b = torch.randn(N, device=DEV)
    for relu in (False, True):
        y = G.addmm_nt(b, x, W, relu=relu)
        ref = x.double() @ W.double().t() + b.double()
        if relu:
            ref = ref.clamp_min(0)
        scale = x.double().abs() @ W.double().abs().t() + b.double().abs()
        assert scaled_err(y, ref, scale) < 1e-6


@pytest.mark.parametrize("consumers", [1, 2])
def test_relu_mask_in_next_layers_dgrad_epilogue_is_bit_identical(monkeypatch, consumers):
    """The box MLP (pdvc.py MLP: Linear-ReLU-Linear-ReLU-Linear through TorchLinearFunction): a ReLU layer's backward
    mask (threshold_backward) taken by the next layer's data-gradient epilogue (pdvc_gemm3p_dmask_f32, p = 0) and
    handed over as a tagged gradient (linear.py tag_relu_masked) against the separate threshold_backward passes --
    bit-identical output and gradients.  consumers = 2: the ReLU output also feeds a second product, so autograd
    sums the two gradients and the producer must mask that sum itself (the tag does not survive the sum)."""
    G = _on_gemm3(monkeypatch)
    import pdvc.ops.functions.linear as L
    fused = []
    real = G.mm_dgrad_dmask

    def counting(*a, **k):
        r = real(*a, **k)
        fused.append(r is not None)
        return r
    monkeypatch.setattr(G, "mm_dgrad_dmask", counting)
    torch.manual_seed(5)
    rows, d = 3000, 256
    x = torch.randn(rows, d, device=DEV)
    lins = [torch.nn.Linear(d, d).to(DEV), torch.nn.Linear(d, d).to(DEV), torch.nn.Linear(d, 64).to(DEV)]
    extra = torch.nn.Linear(d, 32).to(DEV)
    params = [p for lin in lins + [extra] for p in (lin.weight, lin.bias)]
    g = torch.randn(rows, 64, device=DEV)
    g2 = torch.randn(rows, 32, device=DEV)
    res = []
    for fuse in (True, False):
        monkeypatch.setattr(L, "_RELU_DMASK", fuse)
        xa = x.clone().requires_grad_()
        h = L.dense(xa, lins[0].weight, lins[0].bias, relu=True)
        h = L.dense(h, lins[1].weight, lins[1].bias, relu=True)
        out = L.dense(h, lins[2].weight, lins[2].bias)
        outs, gs = [out], [g]
        if consumers == 2:
            outs.append(L.dense(h, extra.weight, extra.bias))
            gs.append(g2)
        used = [xa] + params[:6] + (params[6:] if consumers == 2 else [])
        res.append([out.detach()] + list(torch.autograd.grad(outs, used, gs)))
    for i, (a, b) in enumerate(zip(*res)):
        assert torch.equal(a, b), f"tensor {i} differs between the epilogue mask and threshold_backward"
    assert float(res[0][1].abs().max()) > 0
    assert sum(fused) == (2 if consumers == 1 else 3), "the masked data gradients did not run on the fused arm"
