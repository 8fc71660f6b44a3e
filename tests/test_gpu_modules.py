"""GPU parity of the module-level hot path against golden vectors from the reference modules:
DeformableTransformerEncoderLayer / DecoderLayer (MSDA + query self-attention kernels) and the
LSTM-DSA caption head (teacher-forced captioning logits, loss, gradients, greedy decoding); plus the
query self-attention kernel against a float64 torch restatement of nn.MultiheadAttention's core."""
import math
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")
sys.path.insert(0, G)
sys.path.insert(0, HERE)
from parity import assert_close  # noqa: E402
DEV = "cuda"


def load(name):
    return np.load(os.path.join(G, name + ".npz"), allow_pickle=False)


def cu(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return (t.to(dtype) if dtype is not None else t).to(DEV)


def close(a, b, tol, what):
    """Per-tensor relative bound: max|a - b| <= tol * max|b| + 1e-7 (tests/parity.py)."""
    assert_close(a, b, what, tol)


def fill(module):
    import weights as W
    W.fill_module(module, overrides={"sampling_offsets": 0.5})


# ------------------------------------------------------------------------------------------------
# query self-attention kernel
# ------------------------------------------------------------------------------------------------
def torch_mha_core(qk, v, kpm, M):
    N, Q, E2 = qk.shape
    E = E2 // 2
    D = E // M
    q = qk[..., :E].reshape(N, Q, M, D).transpose(1, 2)
    k = qk[..., E:].reshape(N, Q, M, D).transpose(1, 2)
    vv = v.reshape(N, Q, M, D).transpose(1, 2)
    s = (q * math.sqrt(1.0 / D)) @ k.transpose(-1, -2)
    if kpm is not None:
        s = s.masked_fill(kpm[:, None, None, :], float("-inf"))
    p = torch.softmax(s, -1)
    return (p @ vv).transpose(1, 2).reshape(N, Q, E), p


@pytest.mark.parametrize("Q,masked", [(100, False), (100, True), (37, True), (128, True), (129, False), (300, False),
                                      (129, True), (300, True), (257, True)])
def test_query_self_attention_vs_float64(Q, masked):
    from pdvc.ops.functions.attention import query_self_attention
    torch.manual_seed(Q)
    N, M, E = 3, 8, 512
    qk = torch.randn(N, Q, 2 * E, device=DEV)
    v = torch.randn(N, Q, E, device=DEV)
    kpm = None
    if masked:
        kpm = torch.zeros(N, Q, dtype=torch.bool, device=DEV)
        kpm[1, -5:] = True
        kpm[2, :3] = True
    g = torch.randn(N, Q, E, device=DEV)
    a, b = qk.clone().requires_grad_(), v.clone().requires_grad_()
    out = query_self_attention(a, b, kpm, M, 0.0)
    out.backward(g)
    a64, b64 = qk.double().requires_grad_(), v.double().requires_grad_()
    ref, _ = torch_mha_core(a64, b64, kpm, M)
    ref.backward(g.double())
    close(out, ref, 1e-5, "out")
    close(a.grad, a64.grad, 1e-4, "grad_qk")
    close(b.grad, b64.grad, 1e-4, "grad_v")


def test_query_self_attention_dropout_consistent():
    """With dropout the kernel's mask is recovered from its own output (v = one-hot keys); the forward
    equals P_d.v and the backward equals autograd of that expression with the same mask."""
    from pdvc.ops.functions.attention import QuerySelfAttentionFunction
    torch.manual_seed(0)
    N, M, E, Q, p = 2, 8, 512, 64, 0.25
    qk = torch.randn(N, Q, 2 * E, device=DEV)
    onehot = torch.eye(Q, device=DEV)[None, :, None, :].expand(N, Q, M, 64).reshape(N, Q, E).contiguous()
    pd = QuerySelfAttentionFunction.apply(qk, onehot, None, M, p, 1234)  # rows of P_d per head
    pd = pd.view(N, Q, M, Q).transpose(1, 2)  # (N, M, Q, Q)
    _, P = torch_mha_core(qk.double(), onehot.double(), None, M)
    kept = pd > 0
    frac = kept.float().mean().item()
    assert abs(frac - (1 - p)) < 0.03, frac
    Z = kept.double() / (1 - p)
    close(pd, P * Z, 1e-5, "P_d")
    v = torch.randn(N, Q, E, device=DEV)
    g = torch.randn(N, Q, E, device=DEV)
    a, b = qk.clone().requires_grad_(), v.clone().requires_grad_()
    out = QuerySelfAttentionFunction.apply(a, b, None, M, p, 1234)
    out.backward(g)
    a64, b64 = qk.double().requires_grad_(), v.double().requires_grad_()
    _, P64 = torch_mha_core(a64, b64, None, M)
    ref = (P64 * Z) @ b64.view(N, Q, M, 64).transpose(1, 2)
    ref = ref.transpose(1, 2).reshape(N, Q, E)
    ref.backward(g.double())
    close(out, ref, 1e-5, "out")
    close(a.grad, a64.grad, 1e-4, "grad_qk")
    close(b.grad, b64.grad, 1e-4, "grad_v")


@pytest.mark.parametrize("Q,p", [(100, 0.1), (61, 0.0), (128, 0.3), (300, 0.1), (129, 0.3), (200, 0.0)])
def test_query_self_attention_matrix_core_matches_scalar(Q, p, monkeypatch):
    """The MFMA kernels (D = 64: one workgroup per (video, head) at Q <= 128, the flash-style seqattn kernels
    above) and the scalar kernels (PDVC_MHA_MFMA=0) draw the same dropout mask from the same seed: outputs and
    gradients agree to fp32 rounding."""
    from pdvc.ops.functions.attention import QuerySelfAttentionFunction
    torch.manual_seed(Q)
    N, M, E = 3, 8, 512
    qk = torch.randn(N, Q, 2 * E, device=DEV)
    v = torch.randn(N, Q, E, device=DEV)
    kpm = torch.zeros(N, Q, dtype=torch.bool, device=DEV)
    kpm[0, -7:] = True
    kpm[2, 1:4] = True
    g = torch.randn(N, Q, E, device=DEV)
    res = []
    for mode in ("1", "0"):
        monkeypatch.setenv("PDVC_MHA_MFMA", mode)
        a, b = qk.clone().requires_grad_(), v.clone().requires_grad_()
        out = QuerySelfAttentionFunction.apply(a, b, kpm, M, p, 77)
        out.backward(g)
        res.append((out.detach(), a.grad, b.grad))
    for name, x, y in zip(("out", "grad_qk", "grad_v"), res[0], res[1]):
        close(x, y, 2e-5, name)


@pytest.mark.parametrize("Q,p", [(100, 0.1), (61, 0.0), (128, 0.3), (33, 0.1)])
def test_query_self_attention_streaming_backward_matches(Q, p, monkeypatch):
    """The 51-KiB streaming backward (mha_bwd_mfma2_kernel: K / V and q / dO rows in 32-row blocks, own rows as
    register A operands) against the 133-KiB one (PDVC_MHA_BWD2=0): the same dropout mask, products and summation
    order, so the gradients agree to fp32 rounding; both against float64 in the tests above."""
    from pdvc.ops.functions.attention import QuerySelfAttentionFunction
    torch.manual_seed(Q + 7)
    N, M, E = 3, 8, 512
    qk = torch.randn(N, Q, 2 * E, device=DEV)
    v = torch.randn(N, Q, E, device=DEV)
    kpm = torch.zeros(N, Q, dtype=torch.bool, device=DEV)
    kpm[1, -4:] = True
    g = torch.randn(N, Q, E, device=DEV)
    res = []
    for mode in ("1", "0"):
        monkeypatch.setenv("PDVC_MHA_BWD2", mode)
        a, b = qk.clone().requires_grad_(), v.clone().requires_grad_()
        out = QuerySelfAttentionFunction.apply(a, b, kpm, M, p, 99)
        out.backward(g)
        res.append((a.grad, b.grad))
    for name, x, y in zip(("grad_qk", "grad_v"), res[0], res[1]):
        close(x, y, 2e-5, name)


def test_packed_in_proj_matches_per_slice_linears():
    """PackedLinearFunction (the decoder self-attention's in_proj over the (query | key) and value inputs, one
    packed weight gradient) against the per-slice F.linear form torch's nn.MultiheadAttention uses, in float64."""
    from pdvc.ops.functions.linear import PackedLinearFunction
    torch.manual_seed(3)
    E = 512
    w = torch.randn(3 * E, E, device=DEV) * 0.05
    b = torch.randn(3 * E, device=DEV) * 0.1
    a_in = torch.randn(4, 100, E, device=DEV)
    v_in = torch.randn(4, 100, E, device=DEV)
    ga, gv = torch.randn(4, 100, 2 * E, device=DEV), torch.randn(4, 100, E, device=DEV)
    leaves = [t.clone().requires_grad_() for t in (w, b, a_in, v_in)]
    qk, v = PackedLinearFunction.apply(leaves[0], leaves[1], (2 * E, E), leaves[2], leaves[3])
    torch.autograd.backward((qk, v), (ga, gv))
    ref = [t.double().requires_grad_() for t in (w, b, a_in, v_in)]
    rqk = torch.nn.functional.linear(ref[2], ref[0][:2 * E], ref[1][:2 * E])
    rv = torch.nn.functional.linear(ref[3], ref[0][2 * E:], ref[1][2 * E:])
    torch.autograd.backward((rqk, rv), (ga.double(), gv.double()))
    close(qk, rqk, 1e-5, "qk")
    close(v, rv, 1e-5, "v")
    for name, x, r in zip(("weight", "bias", "qk_in", "v_in"), leaves, ref):
        close(x.grad, r.grad, 1e-4, "grad " + name)


@pytest.mark.parametrize("rd", [1, 2])
def test_box_refine_matches_inverse_sigmoid_chain(rd):
    """box_refine (csrc/boxref.hip) against the reference's chain sigmoid(tmp + inverse_sigmoid(ref))
    (misc/detr_utils/misc.py:540-544; a 1-d reference refines only the centre) in float64, forward and both
    gradients, with references at and beyond the clamp edges (0, 1, eps, outside [0, 1])."""
    from pdvc.box_ops import inverse_sigmoid
    from pdvc.ops.functions.boxref import box_refine
    torch.manual_seed(rd)
    tmp = torch.randn(7, 100, 2, device=DEV)
    ref = torch.rand(7, 100, rd, device=DEV)
    edge = torch.tensor([0.0, 1.0, 1e-6, 1 - 1e-6, -0.2, 1.3], device=DEV)
    ref.view(-1)[:edge.numel()] = edge
    g = torch.randn(7, 100, 2, device=DEV)
    t1, r1 = tmp.clone().requires_grad_(), ref.clone().requires_grad_()
    out = box_refine(t1, r1)
    out.backward(g)
    t2, r2 = tmp.double().requires_grad_(), ref.double().requires_grad_()
    r = inverse_sigmoid(r2)
    ref_out = (t2 + r).sigmoid() if rd == 2 else torch.cat([t2[..., :1] + r, t2[..., 1:]], -1).sigmoid()
    ref_out.backward(g.double())
    close(out, ref_out, 1e-5, "out")
    close(t1.grad, t2.grad, 1e-4, "grad tmp")
    close(r1.grad, r2.grad, 1e-4, "grad ref")


# ------------------------------------------------------------------------------------------------
# transformer layers vs the reference layers (tests/golden/make_golden.py::module_layers)
# ------------------------------------------------------------------------------------------------
def test_decoder_layer_vs_golden():
    from pdvc.deformable_transformer import DeformableTransformerDecoderLayer
    d = load("module_decoder_layer")
    layer = DeformableTransformerDecoderLayer(64, 48, 0.0, "relu", 4, 4, 4).to(DEV)
    fill(layer)
    T_l = tuple(int(t) for t in d["T_l"])
    tgt, pos, ref, src = (cu(d[k]).requires_grad_() for k in ("tgt", "query_pos", "ref", "src"))
    lsi = torch.tensor([0, 16, 24, 28], device=DEV)
    # the reference layer hands self_attn's key_padding_mask = ~query_mask (deformable_transformer.py:257)
    out = layer(tgt, pos, ref, src, T_l, lsi, cu(d["pad"]), cu(d["query_mask"]))
    close(out, d["out"], 1e-4, "out")
    out.backward(cu(d["grad_out"]))
    for k, t in (("grad_tgt", tgt), ("grad_query_pos", pos), ("grad_ref", ref), ("grad_src", src)):
        close(t.grad, d[k], 1e-4, k)
    for n, p in layer.named_parameters():
        close(p.grad, d["grad." + n], 1e-4, n)


def test_decoder_layer_shared_query_rows_match_the_expanded_rows():
    """The first decoder layer's in_proj over the Q query rows every video repeats (prepare_decoder_input_query's
    expands, tagged with their (Q, d) rows): projected once and broadcast, against the same layer on materialised
    (N, Q, d) copies of the rows -- output, the rows' gradients (summed over the videos by the expand) and every
    parameter gradient."""
    from pdvc.deformable_transformer import DeformableTransformerDecoderLayer
    d = load("module_decoder_layer")
    layer = DeformableTransformerDecoderLayer(64, 48, 0.0, "relu", 4, 4, 4).to(DEV)
    fill(layer)
    T_l = tuple(int(t) for t in d["T_l"])
    lsi = torch.tensor([0, 16, 24, 28], device=DEV)
    ref, src = cu(d["ref"]), cu(d["src"])
    N, Q, C = d["tgt"].shape
    torch.manual_seed(11)
    rows = [torch.randn(Q, C, device=DEV) for _ in range(2)]
    g = torch.randn(N, Q, C, device=DEV)
    seen = []
    fwd = layer.self_attn.forward
    layer.self_attn.forward = lambda *a, **k: (seen.append(k.get("batch")), fwd(*a, **k))[1]
    results = []
    for shared in (True, False):
        layer.zero_grad()
        t_rows, p_rows = (r.clone().requires_grad_() for r in rows)
        tgt, pos = (r.unsqueeze(0).expand(N, -1, -1) for r in (t_rows, p_rows))
        if shared:
            tgt.__dict__["_pdvc_rows"], pos.__dict__["_pdvc_rows"] = t_rows, p_rows
        else:
            tgt, pos = tgt.contiguous(), pos.contiguous()
        out = layer(tgt, pos, ref, src, T_l, lsi, cu(d["pad"]), cu(d["query_mask"]))
        out.backward(g)
        results.append([out, t_rows.grad, p_rows.grad] + [p.grad.clone() for p in layer.parameters()])
    assert seen == [N, None]
    names = ["out", "grad tgt rows", "grad pos rows"] + [n for n, _ in layer.named_parameters()]
    for name, a, b in zip(names, *results):
        close(a, b, 1e-5, name)


def test_decoder_layer_parameters_named_like_nn_multiheadattention():
    from pdvc.deformable_transformer import DeformableTransformerDecoderLayer
    names = [n for n, _ in DeformableTransformerDecoderLayer(64, 48, 0.0, "relu", 4, 4, 4).named_parameters()]
    assert "self_attn.in_proj_weight" in names and "self_attn.out_proj.weight" in names


def test_encoder_layer_vs_golden():
    from pdvc.deformable_transformer import DeformableTransformerEncoderLayer
    d = load("module_encoder_layer")
    layer = DeformableTransformerEncoderLayer(64, 48, 0.0, "relu", 4, 4, 4).to(DEV)
    fill(layer)
    T_l = tuple(int(t) for t in d["T_l"])
    src, pos = cu(d["src"]).requires_grad_(), cu(d["pos"]).requires_grad_()
    lsi = torch.tensor([0, 16, 24, 28], device=DEV)
    out = layer(src, pos, cu(d["ref"]), T_l, lsi, cu(d["pad"]))
    close(out, d["out"], 1e-4, "out")
    out.backward(cu(d["grad_out"]))
    close(src.grad, d["grad_src"], 1e-4, "grad_src")
    close(pos.grad, d["grad_pos"], 1e-4, "grad_pos")
    for n, p in layer.named_parameters():
        close(p.grad, d["grad." + n], 1e-4, n)


# ------------------------------------------------------------------------------------------------
# caption head vs the reference LSTM_DSA (make_golden.py::module_captioner)
# ------------------------------------------------------------------------------------------------
def small_opt():
    import types
    return types.SimpleNamespace(
        vocab_size=23, input_encoding_size=32, rnn_size=64, num_layers=1, drop_prob=0.0, max_caption_len=6,
        clip_context_dim=64, cap_nheads=1, att_hid_size=48, wordRNN_input_feats_type="C", hidden_dim=64,
        cap_num_feature_levels=4, cap_dec_n_points=4, num_feature_levels=4, event_context_dim=None)


@pytest.mark.parametrize("ref_dim", [1, 2])
def test_captioner_vs_golden(ref_dim):
    from pdvc.CaptioningHead.LSTM_DSA import LSTMDSACaptioner
    d = load(f"module_captioner_ref{ref_dim}")
    cap = LSTMDSACaptioner(small_opt()).to(DEV)
    fill(cap)
    cap.train()
    T_l = tuple(int(t) for t in d["T_l"])
    hs, ref, mem = (cu(d[k]).requires_grad_() for k in ("hs", "ref", "memory"))
    others = {"memory": mem, "mask_flatten": cu(d["mask"]), "spatial_shapes": torch.tensor(T_l, device=DEV),
              "level_T": T_l, "valid_ratios": torch.ones(1, 4, device=DEV)}
    cap_tensor = cu(d["cap_tensor"])
    logprobs = cap(hs, ref, others, cap_tensor)
    close(logprobs, d["logprobs"], 1e-4, "captioning logits (log_softmax)")
    loss = cap.build_loss(logprobs, cap_tensor[:, 1:], cu(d["cap_mask"])[:, 1:].float()).mean()
    close(loss, d["loss"], 1e-4, "loss")
    loss.backward()
    close(hs.grad, d["grad_hs"], 1e-4, "grad_hs")
    close(ref.grad, d["grad_ref"], 1e-4, "grad_ref")
    close(mem.grad, d["grad_memory"], 1e-4, "grad_memory")
    for n, p in cap.named_parameters():
        key = "grad." + n
        if d[key].size == 0:
            assert p.grad is None, f"{n} must get no gradient"
        else:
            close(p.grad, d[key], 1e-4, n)
    cap.eval()
    with torch.no_grad():
        seq, lp = cap.sample(hs.detach(), ref.detach(), {k: (v.detach() if isinstance(v, torch.Tensor) else v)
                                                         for k, v in others.items()})
    assert seq.cpu().tolist() == d["sample_seq"].tolist()
    close(lp, d["sample_logprobs"], 1e-4, "greedy logprobs")


@pytest.mark.parametrize("temperature", [1.0, 0.5])
def test_captioner_multinomial_sampling(temperature):
    """sample_max=0 (LSTM_DSA.py:160-168): words drawn from exp(logprobs / temperature).  The draws are
    random (parity unpinned: torch's device RNG is not the reference's CPU RNG), so the test checks the
    law: 4096 copies of one event row share the first step's distribution; the frequency ratio of two drawn
    words must match exp((lp_a - lp_b) / temperature) within 5 standard errors, every returned log-probability
    must be the untempered log-probability of its word (equal words -> equal values), a seeded generator
    must reproduce the draws, and the unfinished-mask semantics must hold (zeros after a row's first 0)."""
    from pdvc.CaptioningHead.LSTM_DSA import LSTMDSACaptioner
    d = load("module_captioner_ref1")
    cap = LSTMDSACaptioner(small_opt()).to(DEV)
    fill(cap)
    cap.eval()
    T_l = tuple(int(t) for t in d["T_l"])
    R = 4096
    hs = cu(d["hs"])[:, :1].expand(1, R, -1).contiguous()
    ref = cu(d["ref"])[:, :1].expand(1, R, -1).contiguous()
    others = {"memory": cu(d["memory"]), "mask_flatten": cu(d["mask"]), "level_T": T_l,
              "spatial_shapes": torch.tensor(T_l, device=DEV), "valid_ratios": torch.ones(1, 4, device=DEV)}
    gen = torch.Generator(device=DEV).manual_seed(7)
    opt = {"sample_max": 0, "temperature": temperature, "generator": gen}
    with torch.no_grad():
        seq, lp = cap.sample(hs, ref, others, opt)
        gen.manual_seed(7)
        seq2, lp2 = cap.sample(hs, ref, others, opt)
    assert torch.equal(seq, seq2) and torch.equal(lp, lp2), "seeded draws must repeat"
    first, lp1 = seq[:, 0].cpu().numpy(), lp[:, 0].double().cpu().numpy()
    words, counts = np.unique(first, return_counts=True)
    assert len(words) >= 2, "a tempered draw over 24 words should not be constant"
    lp_of = {}
    for w in words:
        vals = lp1[first == w]
        assert np.ptp(vals) < 1e-5, f"word {w}: log-probabilities differ across identical rows"
        lp_of[w] = vals[0]
    a, b = words[np.argsort(-counts)[:2]]
    ca, cb = counts[words == a][0], counts[words == b][0]
    expect = np.exp((lp_of[a] - lp_of[b]) / temperature)
    se = (ca / cb) * np.sqrt(1.0 / ca + 1.0 / cb)
    assert abs(ca / cb - expect) <= 5 * se, f"ratio {ca / cb:.3f} vs exp((lp_a-lp_b)/T) {expect:.3f}"
    s = seq.cpu().numpy()
    for row in s[:256]:
        z = np.flatnonzero(row == 0)
        if z.size:
            assert not row[z[0]:].any(), "tokens after a finished row"


@pytest.mark.parametrize("heads,rd1,deferred", [(1, 3, False), (2, 0, False), (1, 3, True), (2, 0, True)])
def test_caption_decode_function_matches_step_loop(heads, rd1, deferred, monkeypatch):
    """The fused teacher-forced recurrence (ops/functions/caption_decode.py) against the per-step autograd
    loop of the same math (LSTMDSACaptioner._step: cap-gather kernel + torch ops), at the PDVC caption shape
    (d=512, A=512, H=512, 16 samples) with a mix of 1-d and (c, len) reference rows. deferred: the value
    gradient of all steps comes from the destination-sorted pass (pdvc_cap_value_grad_f32) over the per-video
    row CSR instead of per-step atomics; video 2 has no rows."""
    import types
    from pdvc.CaptioningHead.LSTM_DSA import LSTMDSACaptioner
    opt = types.SimpleNamespace(
        vocab_size=50, input_encoding_size=512, rnn_size=512, num_layers=1, drop_prob=0.0, max_caption_len=8,
        clip_context_dim=512, cap_nheads=heads, att_hid_size=512, wordRNN_input_feats_type="C", hidden_dim=512,
        cap_num_feature_levels=4, cap_dec_n_points=4, num_feature_levels=4, event_context_dim=None)
    torch.manual_seed(0)
    cap = LSTMDSACaptioner(opt).to(DEV)
    with torch.no_grad():
        for p in cap.parameters():
            p.normal_(0, 0.03)
    T_l = (64, 32, 16, 8)
    Nv, R, n = 3, 9, 7
    S = sum(T_l)
    memory = torch.randn(Nv, S, 512, device=DEV)
    mask = torch.zeros(Nv, S, dtype=torch.bool, device=DEV)
    mask[1, -5:] = True
    hs = torch.randn(R, 512, device=DEV)
    ref = torch.rand(R, 4, 2, device=DEV) * 0.8 + 0.1
    rv = [0, 1, 0, 1, 0, 1, 1, 0, 0]
    row_video = torch.tensor(rv, dtype=torch.int32, device=DEV)
    starts, flat = [0], []
    for v in range(Nv):
        flat += [i for i in range(R) if rv[i] == v]
        starts.append(len(flat))
    video_csr = (torch.tensor(starts, dtype=torch.int32, device=DEV),
                 torch.tensor(flat, dtype=torch.int32, device=DEV), max(rv.count(v) for v in range(Nv)))
    seq = torch.randint(1, 51, (R, n + 1), device=DEV)
    g = torch.randn(R, n, 51, device=DEV)

    def run(fused):
        ins = [t.clone().requires_grad_() for t in (hs, ref, memory)]
        cap.zero_grad(set_to_none=True)
        if fused:
            out = cap.decode_teacher_forced(ins[0], ins[1], rd1, row_video, ins[2], mask, T_l, seq, n,
                                            video_csr=video_csr if deferred else None)
        else:
            w = cap._step_weights()
            value, mask_u8 = cap._prepare(ins[2], mask)
            xt = cap.embed(seq[:, :n])
            x_gates = torch.nn.functional.linear(xt, w["W_x"])
            hs_part = torch.nn.functional.linear(ins[0], w["W_hs"])
            off_hs = torch.nn.functional.linear(ins[0], w["W_off_hs"], w["b_off"])
            h = ins[0].new_zeros(R, 512)
            c = ins[0].new_zeros(R, 512)
            outs = []
            for i in range(n):
                h, c = cap._step(w, h, c, x_gates[:, i], hs_part, off_hs, value, mask_u8, row_video, ins[1], rd1,
                                 T_l)
                outs.append(h)
            out = torch.log_softmax(cap.logit(torch.stack(outs, 1)), -1)
        loss = (out * g).sum()
        loss.backward()
        grads = {k: p.grad.clone() for k, p in cap.named_parameters() if p.grad is not None}
        return out.detach(), [t.grad.clone() for t in ins], grads

    from pdvc import _native as _nm
    from pdvc.ops.functions import caption_decode as cd
    called, real_call = set(), _nm.call

    def spy(name, *a, **k):
        called.add(name)
        return real_call(name, *a, **k)

    monkeypatch.setattr(_nm, "call", spy)
    o1, gi1, gp1 = run(True)
    monkeypatch.setattr(_nm, "call", real_call)
    # the one-launch caption step is the path taken at the 512-wide head (heads = 1: D = A = 512), its backward
    # with the per-video row CSR (the U-gradient form); the 256-wide heads take the separate launches
    assert ("pdvc_cap_softattn_forward_f32" in called) == (heads == 1 and cd.CAP_FUSED)
    assert ("pdvc_cap_softattn_backward_f32" in called) == (heads == 1 and deferred and cd.CAP_FUSED
                                                            and cd.CAP_FUSED_BWD)
    o0, gi0, gp0 = run(False)
    close(o1, o0, 1e-5, "logprobs")
    for name, a, b in zip(("hs", "ref", "memory"), gi1, gi0):
        close(a, b, 1e-4, "grad_" + name)
    assert set(gp1) == set(gp0)
    for k in gp0:
        if k.endswith("alpha_net.bias"):  # zero in exact arithmetic (softmax shift invariance): both sides are
            # rounding noise, bounded against the scale of the alpha_net weight gradient
            assert_close(gp1[k], gp0[k], k, 1e-4, scale=gp0[k[:-4] + "weight"].abs().max().item())
        else:
            close(gp1[k], gp0[k], 1e-4, k)


def test_caption_value_grad_chunked_steps():
    """Many caption rows on one video (220 rows x 4 points x 12 B per step) overflow the LDS of one launch of
    the destination-sorted value-gradient pass, so its steps run in several accumulating chunks; the memory
    gradient must match the per-step atomic path of the same fused recurrence."""
    import types
    from pdvc.CaptioningHead.LSTM_DSA import LSTMDSACaptioner
    opt = types.SimpleNamespace(
        vocab_size=30, input_encoding_size=512, rnn_size=512, num_layers=1, drop_prob=0.0, max_caption_len=24,
        clip_context_dim=512, cap_nheads=1, att_hid_size=512, wordRNN_input_feats_type="C", hidden_dim=512,
        cap_num_feature_levels=4, cap_dec_n_points=4, num_feature_levels=4, event_context_dim=None)
    torch.manual_seed(1)
    cap = LSTMDSACaptioner(opt).to(DEV)
    with torch.no_grad():
        for p in cap.parameters():
            p.normal_(0, 0.03)
    T_l = (128, 64, 32, 16)
    Nv, R, n = 2, 240, 20
    memory = torch.randn(Nv, sum(T_l), 512, device=DEV)
    mask = torch.zeros(Nv, sum(T_l), dtype=torch.bool, device=DEV)
    mask[0, -7:] = True
    hs = torch.randn(R, 512, device=DEV)
    ref = torch.rand(R, 4, 2, device=DEV) * 0.9 + 0.05
    rv = [0 if i % 12 else 1 for i in range(R)]
    row_video = torch.tensor(rv, dtype=torch.int32, device=DEV)
    starts, flat = [0], []
    for v in range(Nv):
        flat += [i for i in range(R) if rv[i] == v]
        starts.append(len(flat))
    video_csr = (torch.tensor(starts, dtype=torch.int32, device=DEV),
                 torch.tensor(flat, dtype=torch.int32, device=DEV), max(rv.count(v) for v in range(Nv)))
    assert 12 * video_csr[2] * 4 * n > 96 * 1024  # more than one chunk
    seq = torch.randint(1, 31, (R, n + 1), device=DEV)
    g = torch.randn(R, n, 31, device=DEV)

    def run(csr):
        m = memory.clone().requires_grad_()
        out = cap.decode_teacher_forced(hs, ref, 5, row_video, m, mask, T_l, seq, n, video_csr=csr)
        (out * g).sum().backward()
        return m.grad
    close(run(video_csr), run(None), 1e-4, "grad_memory")


@pytest.mark.parametrize("masked,heads", [(False, 1), (True, 1), (False, 2)])
def test_caption_decode_projected_row_backward_equals_per_sample(masked, heads):
    """The caption recurrence's backward in the projected-row form (caption_decode.U_GRAD: dATT scattered onto the
    value rows once, dW_ctx = dU^T value, the value gradient's ctx2att part dU W_ctx, the location gradient of
    att read off U at the sample corners) against the per-sample form (dclip += dATT W_ctx each step, dW_ctx over
    every sample): every input and parameter gradient within 1e-4 * max|ref|, with and without padded frames."""
    import types
    import pdvc.ops.functions.caption_decode as CD
    from pdvc.CaptioningHead.LSTM_DSA import LSTMDSACaptioner
    opt = types.SimpleNamespace(
        vocab_size=40, input_encoding_size=512, rnn_size=512, num_layers=1, drop_prob=0.0, max_caption_len=10,
        clip_context_dim=512, cap_nheads=heads, att_hid_size=512, wordRNN_input_feats_type="C", hidden_dim=512,
        cap_num_feature_levels=4, cap_dec_n_points=4, num_feature_levels=4, event_context_dim=None)
    torch.manual_seed(3)
    cap = LSTMDSACaptioner(opt).to(DEV)
    with torch.no_grad():
        for p in cap.parameters():
            p.normal_(0, 0.03)
    T_l = (64, 32, 16, 8)
    S = sum(T_l)
    Nv, R, n = 3, 24, 8
    memory = torch.randn(Nv, S, 512, device=DEV)
    mask = torch.zeros(Nv, S, dtype=torch.bool, device=DEV)
    if masked:
        mask[1, 50:64] = True
        mask[1, 90:96] = True
    hs = torch.randn(R, 512, device=DEV)
    ref = torch.rand(R, 4, 2, device=DEV) * 0.9 + 0.05
    rv = [i % 3 if i % 7 else 1 for i in range(R)]
    row_video = torch.tensor(rv, dtype=torch.int32, device=DEV)
    starts, flat = [0], []
    for v in range(Nv):
        flat += [i for i in range(R) if rv[i] == v]
        starts.append(len(flat))
    video_csr = (torch.tensor(starts, dtype=torch.int32, device=DEV),
                 torch.tensor(flat, dtype=torch.int32, device=DEV), max(rv.count(v) for v in range(Nv)))
    seq = torch.randint(1, 41, (R, n + 1), device=DEV)
    g = torch.randn(R, n, 41, device=DEV)

    def run(u_grad):
        CD.U_GRAD = u_grad
        try:
            cap.zero_grad(set_to_none=True)
            ins = [t.clone().requires_grad_() for t in (hs, ref, memory)]
            out = cap.decode_teacher_forced(ins[0], ins[1], 5, row_video, ins[2], mask, T_l, seq, n,
                                            video_csr=video_csr)
            (out * g).sum().backward()
            return [t.grad.clone() for t in ins], {k: p.grad.clone() for k, p in cap.named_parameters()
                                                   if p.grad is not None}
        finally:
            CD.U_GRAD = True

    gi0, gp0 = run(False)
    gi1, gp1 = run(True)
    for name, a, b in zip(("hs", "ref", "memory"), gi1, gi0):
        close(a, b, 1e-4, "grad_" + name)
    assert set(gp1) == set(gp0)
    for k in gp0:
        if k.endswith("alpha_net.bias"):
            assert_close(gp1[k], gp0[k], k, 1e-4, scale=gp0[k[:-4] + "weight"].abs().max().item())
        else:
            close(gp1[k], gp0[k], 1e-4, k)


@pytest.mark.parametrize("masked", [False, True])
def test_greedy_ctx2att_gather_equals_gemm(masked):
    """Greedy decoding's ctx2att as a gather of the once-projected memory rows (U = ctx2att(value), blended with
    each sample's border weights, LSTMDSACaptioner._ctx2att_rows) against ctx2att applied to every sample (the
    GEMM path, itself pinned to the reference by test_captioner_vs_golden): same words, log-probabilities
    within 1e-4, at a power-of-two attention width (the gather's) with and without padded memory rows."""
    import pdvc.CaptioningHead.LSTM_DSA as L
    opt = small_opt()
    opt.att_hid_size = 64
    opt.max_caption_len = 8
    torch.manual_seed(5)
    cap = L.LSTMDSACaptioner(opt).to(DEV).eval()
    with torch.no_grad():
        for p in cap.parameters():
            p.copy_(torch.randn_like(p) * 0.1)
    T_l = (32, 16, 8, 4)
    S = sum(T_l)
    Nv, E = 3, 5
    hs = torch.randn(Nv, E, 64, device=DEV)
    ref = torch.rand(Nv, E, 2, device=DEV)
    mask = torch.zeros(Nv, S, dtype=torch.bool, device=DEV)
    if masked:
        mask[1, 24:32] = True
        mask[1, 44:48] = True
    others = {"memory": torch.randn(Nv, S, 64, device=DEV), "mask_flatten": mask, "level_T": T_l,
              "spatial_shapes": torch.tensor(T_l, device=DEV), "valid_ratios": torch.ones(Nv, 4, device=DEV)}
    with torch.no_grad():
        L.GREEDY_CTX2ATT_GATHER = False
        try:
            seq_g, lp_g = cap.sample(hs, ref, others)
        finally:
            L.GREEDY_CTX2ATT_GATHER = True
        seq_u, lp_u = cap.sample(hs, ref, others)
    assert seq_g is not None and torch.equal(seq_u, seq_g)
    # the first step sees the two ctx2att forms alone; later steps carry each form's rounding through the LSTM
    # state (random weights at this scale amplify it), so they get a looser bound
    assert (lp_u[:, 0] - lp_g[:, 0]).abs().max().item() <= 1e-5
    assert (lp_u - lp_g).abs().max().item() <= 1e-3


@pytest.mark.parametrize("masked", [False, True])
def test_teacher_forced_ctx2att_gather_equals_gemm(masked):
    """The training recurrence's ctx2att as a gather of the once-projected value rows (CaptionDecodeFunction,
    CTX2ATT_GATHER) against the per-step GEMM: log-probabilities, and every gradient (the backward is shared),
    within 1e-4."""
    import pdvc.ops.functions.caption_decode as CD
    from pdvc.CaptioningHead.LSTM_DSA import LSTMDSACaptioner
    opt = small_opt()
    opt.att_hid_size = 64
    torch.manual_seed(6)
    cap = LSTMDSACaptioner(opt).to(DEV).train()
    with torch.no_grad():
        for p in cap.parameters():
            p.copy_(torch.randn_like(p) * 0.1)
    T_l = (32, 16, 8, 4)
    S = sum(T_l)
    Nv, E = 2, 4
    mask = torch.zeros(Nv, S, dtype=torch.bool, device=DEV)
    if masked:
        mask[0, 20:32] = True
        mask[0, 44:48] = True
    hs0 = torch.randn(Nv, E, 64, device=DEV)
    ref0 = torch.rand(Nv, E, 2, device=DEV)
    mem0 = torch.randn(Nv, S, 64, device=DEV)
    cap_tensor = torch.randint(1, 23, (Nv * E, 7), device=DEV)
    cap_tensor[:, 0] = 0

    def run(gather):
        CD.CTX2ATT_GATHER = gather
        try:
            cap.zero_grad(set_to_none=True)
            hs, ref, mem = (t.clone().requires_grad_() for t in (hs0, ref0, mem0))
            others = {"memory": mem, "mask_flatten": mask, "level_T": T_l,
                      "spatial_shapes": torch.tensor(T_l, device=DEV), "valid_ratios": torch.ones(Nv, 4, device=DEV)}
            lp = cap(hs, ref, others, cap_tensor)
            lp.sum().backward()
            return lp.detach(), [hs.grad, ref.grad, mem.grad] + [p.grad for p in cap.parameters()]
        finally:
            CD.CTX2ATT_GATHER = True

    lp_g, g_g = run(False)
    lp_u, g_u = run(True)
    close(lp_u, lp_g.cpu().numpy(), 1e-4, "logprobs")
    for a, b in zip(g_u, g_g):
        assert (a is None) == (b is None)
        if a is not None:
            close(a, b.cpu().numpy(), 1e-4, "grad")


# ------------------------------------------------------------------------------------------------
# scheduled sampling (LSTM_DSA.py:88-99): parity unpinned for the draws themselves (torch's device RNG is
# not the reference's CPU RNG); pinned through the realised input words and the law of the draws
# ------------------------------------------------------------------------------------------------
def _ss_setup(R_copies=None):
    from pdvc.CaptioningHead.LSTM_DSA import LSTMDSACaptioner, caption_steps
    d = load("module_captioner_ref1")
    cap = LSTMDSACaptioner(small_opt()).to(DEV)
    fill(cap)
    cap.train()
    T_l = tuple(int(t) for t in d["T_l"])
    hs, ref = cu(d["hs"]), cu(d["ref"])
    cap_tensor = cu(d["cap_tensor"])
    if R_copies:
        hs = hs[:, :1].expand(1, R_copies, -1).contiguous()
        ref = ref[:, :1].expand(1, R_copies, -1).contiguous()
        cap_tensor = cap_tensor[:1].expand(R_copies, -1).contiguous()
    others = {"memory": cu(d["memory"]), "mask_flatten": cu(d["mask"]), "level_T": T_l,
              "spatial_shapes": torch.tensor(T_l, device=DEV), "valid_ratios": torch.ones(1, 4, device=DEV)}
    rows = cap._rows_from_reference(hs, ref, others)
    n = caption_steps(cap_tensor.cpu())
    return cap, rows, others, cap_tensor, n


def test_scheduled_sampling_equals_teacher_forcing_on_the_realised_words():
    """With ss_prob = 0.5 the loop feeds drawn words back; replaying the realised input words through the teacher-forced
    path (CaptionDecodeFunction, pinned to the reference by test_captioner_vs_golden) must give the same log-probabilities
    and every gradient, within 1e-4."""
    cap, (hs_rows, ref, rd1, rv, T), others, cap_tensor, n = _ss_setup()
    gen = torch.Generator(device=DEV).manual_seed(11)
    g = torch.randn(hs_rows.shape[0], n, cap.vocab_size + 1, device=DEV)

    def run(ss, seq, record=None):
        cap.zero_grad(set_to_none=True)
        cap.ss_prob = ss
        h, r, mem = hs_rows.clone().requires_grad_(), ref.clone().requires_grad_(), others["memory"].clone().requires_grad_()
        if ss > 0:
            lp = cap.decode_scheduled_sampling(h, r, rd1, rv, mem, others["mask_flatten"], T, seq, n, generator=gen,
                                               record=record)
        else:
            lp = cap.decode_teacher_forced(h, r, rd1, rv, mem, others["mask_flatten"], T, seq, n)
        (lp * g).sum().backward()
        return lp.detach(), [h.grad, r.grad, mem.grad], {k: p.grad for k, p in cap.named_parameters() if p.grad is not None}

    record = []
    lp_ss, gi_ss, gp_ss = run(0.5, cap_tensor, record)
    assert len(record) == n
    realised = cap_tensor.clone()
    for i, it in enumerate(record):
        realised[:, i] = it
    assert not torch.equal(realised[:, :n], cap_tensor[:, :n]), "no word was drawn at ss_prob 0.5"
    lp_tf, gi_tf, gp_tf = run(0.0, realised)
    close(lp_ss, lp_tf, 1e-4, "logprobs")
    for name, a, b in zip(("hs", "ref", "memory"), gi_ss, gi_tf):
        close(a, b, 1e-4, "grad_" + name)
    assert set(gp_ss) == set(gp_tf)
    for k in gp_tf:
        if k.endswith("alpha_net.bias"):
            assert_close(gp_ss[k], gp_tf[k], k, 1e-4, scale=gp_tf[k[:-4] + "weight"].abs().max().item())
        else:
            close(gp_ss[k], gp_tf[k], 1e-4, k)


def test_scheduled_sampling_draws_follow_the_previous_step():
    """ss_prob = 1: every input word from step 1 on is drawn from exp(previous step's log-probabilities).  4096 copies of
    one row share step 0's distribution: the frequency ratio of the two most drawn step-1 words matches
    exp(lp_a - lp_b) within 5 standard errors; at ss_prob = 0 the words are the ground truth."""
    cap, (hs_rows, ref, rd1, rv, T), others, cap_tensor, n = _ss_setup(R_copies=4096)
    cap.ss_prob = 1.0
    rec = []
    with torch.no_grad():
        lp = cap.decode_scheduled_sampling(hs_rows, ref, rd1, rv, others["memory"], others["mask_flatten"], T,
                                           cap_tensor, n, generator=torch.Generator(device=DEV).manual_seed(3),
                                           record=rec)
    words = rec[1].cpu().numpy()
    lp0 = lp[0, 0].double().cpu().numpy()
    assert np.allclose(lp[:, 0].cpu().numpy(), lp[0:1, 0].cpu().numpy(), atol=1e-6), "copies must share step 0"
    vals, counts = np.unique(words, return_counts=True)
    assert len(vals) >= 2
    a, b = vals[np.argsort(-counts)[:2]]
    ca, cb = counts[vals == a][0], counts[vals == b][0]
    expect = np.exp(lp0[a] - lp0[b])
    se = (ca / cb) * np.sqrt(1.0 / ca + 1.0 / cb)
    assert abs(ca / cb - expect) <= 5 * se, f"ratio {ca / cb:.3f} vs exp(lp_a - lp_b) {expect:.3f}"
    assert torch.equal(rec[0], cap_tensor[:, 0]), "step 0 always takes the ground-truth word"
    cap.ss_prob = 0.0
    rec0 = []
    with torch.no_grad():
        cap.decode_scheduled_sampling(hs_rows[:8], ref[:8], min(rd1, 8), rv[:8], others["memory"],
                                      others["mask_flatten"], T, cap_tensor[:8], n, record=rec0)
    for i, it in enumerate(rec0):
        assert torch.equal(it, cap_tensor[:8, i])


def test_model_step_with_scheduled_sampling():
    """A whole batched training step with Captioner.ss_prob = 0.25 (the decode's per-step path): finite losses and
    gradients for every parameter the teacher-forced step trains."""
    sys.path.insert(0, HERE)
    import test_gpu_model as TM
    d = TM.load("pdvc_small_anet")
    model, criterion = TM.build_filled(d)
    model.train()
    model.caption_head[0].ss_prob = 0.25
    out, loss = model(TM.fixture_dt(d), criterion, "queries")
    total = sum(loss[k] * criterion.weight_dict[k] for k in loss.keys() if k in criterion.weight_dict)
    assert torch.isfinite(total)
    total.backward()
    for n_, p in model.named_parameters():
        assert (p.grad is None) == ("gradnone." + n_ in d.files), n_
        if p.grad is not None:
            assert torch.isfinite(p.grad).all(), n_
