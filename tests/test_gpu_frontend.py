"""GPU parity of the dual-modality front-end of cfgs/yc2_newModel_sound.yml (pdvc/frontend.py over the HIP
attention core csrc/seqattn.hip) against the reference's own construction -- NewModel.visual_self_attention /
visual_sound_attention (NewModel.py:41-65) with torch nn.MultiheadAttention(768, 32, batch_first=True) -- in
float64, loaded from our state_dict with strict=True (same parameter names), forward and every gradient.
HuBERT is not rebuilt (its weights are a network download): synthetic sound features stand in, so parity is
pinned against torch's MultiheadAttention arithmetic, not against a reference run."""
import pytest
import torch
from parity import assert_close
from torch import nn

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4  # fp32 vs float64: max|diff| <= TOL * max|reference| + 1e-7 per tensor


def close(a, b, tol, what):
    """Per-tensor relative bound: max|a - b| <= tol * max|b| + 1e-7 (tests/parity.py)."""
    assert_close(a, b, what, tol)


class RefFrontEnd(nn.Module):
    """NewModel's front-end layers and forward (NewModel.py:21-33, 41-65), restated with the same torch modules."""

    def __init__(self, dim, heads):
        super().__init__()
        self.ln1 = nn.LayerNorm(dim)
        self.mha1 = nn.MultiheadAttention(dim, heads, batch_first=True)
        self.mlp_seq1 = nn.Sequential(nn.Linear(dim, dim), nn.LayerNorm(dim))
        self.ln2 = nn.LayerNorm(dim)
        self.mha2 = nn.MultiheadAttention(dim, heads, batch_first=True)
        self.mlp_seq2 = nn.Sequential(nn.Linear(dim, dim), nn.LayerNorm(dim))

    def forward(self, clips, sound):
        add = clips
        f, _ = self.mha1(query=clips, key=clips, value=clips)
        f = self.ln1(f) + add
        f = self.mlp_seq1(f) + f
        add = f
        g, _ = self.mha2(query=sound, key=f, value=f)
        g = self.ln2(g) + add
        return self.mlp_seq2(g) + g


@pytest.mark.parametrize("T,dim,heads", [(130, 768, 32), (512, 768, 32), (77, 512, 8)])
def test_frontend_matches_multiheadattention_reference(T, dim, heads):
    from pdvc.frontend import DualModalityFrontEnd
    torch.manual_seed(T)
    ours = DualModalityFrontEnd(dim, heads).to(DEV)
    with torch.no_grad():  # non-trivial LayerNorm affine and biases
        for n, p in ours.named_parameters():
            if p.dim() == 1:
                p.normal_(0.0 if "bias" in n else 1.0, 0.1)
    ref = RefFrontEnd(dim, heads).to(DEV).double()
    ref.load_state_dict({k: v.double() for k, v in ours.state_dict().items()}, strict=True)
    N = 2
    clips = torch.randn(N, T, dim, device=DEV)
    sound = torch.randn(N, T, dim, device=DEV)
    gout = torch.randn(N, T, dim, device=DEV)
    c1, s1 = clips.clone().requires_grad_(), sound.clone().requires_grad_()
    out = ours(c1, s1)
    (out * gout).sum().backward()
    c0, s0 = clips.double().requires_grad_(), sound.double().requires_grad_()
    out0 = ref(c0, s0)
    (out0 * gout.double()).sum().backward()
    close(out, out0, TOL, "front-end output")
    close(c1.grad, c0.grad, TOL, "grad clips")
    close(s1.grad, s0.grad, TOL, "grad sound")
    refp = dict(ref.named_parameters())
    for n, p in ours.named_parameters():
        close(p.grad, refp[n].grad, TOL, "grad " + n)


@pytest.mark.parametrize("Tq,Tk,H,D", [(1, 1, 2, 16), (200, 300, 4, 64), (129, 257, 3, 48), (64, 5, 2, 32),
                                       (512, 512, 32, 24), (33, 70, 4, 24), (300, 1, 2, 24), (130, 97, 5, 16)])
def test_seq_attention_core_vs_float64(Tq, Tk, H, D):
    """The attention core alone, queries and keys of different lengths, packed (strided) q/k/v views."""
    from pdvc.ops.functions.seq_attention import seq_attention
    torch.manual_seed(Tq + Tk)
    N, E = 2, H * D
    qx = torch.randn(N, Tq, 2 * E, device=DEV) * 2
    kv = torch.randn(N, Tk, 2 * E, device=DEV) * 2
    q1, kv1 = qx.clone().requires_grad_(), kv.clone().requires_grad_()
    out = seq_attention(q1[..., E:], kv1[..., :E], kv1[..., E:], H)
    g = torch.randn(N, Tq, E, device=DEV)
    (out * g).sum().backward()
    q0, kv0 = qx.double().requires_grad_(), kv.double().requires_grad_()
    qh = q0[..., E:].reshape(N, Tq, H, D).transpose(1, 2)
    kh = kv0[..., :E].reshape(N, Tk, H, D).transpose(1, 2)
    vh = kv0[..., E:].reshape(N, Tk, H, D).transpose(1, 2)
    p = torch.softmax(qh @ kh.transpose(-1, -2) / D ** 0.5, -1)
    ref = (p @ vh).transpose(1, 2).reshape(N, Tq, E)
    (ref * g.double()).sum().backward()
    close(out, ref, TOL, "out")
    if Tk == 1:  # one key: the softmax is constant, the query gradient is zero in exact arithmetic -- its fp32
        # rounding noise is bounded against the scale of the value gradient instead of its own (zero) scale
        assert_close(q1.grad, q0.grad, "grad q (zero)", TOL, scale=kv0.grad.abs().max().item())
    else:
        close(q1.grad, q0.grad, TOL, "grad q")
    close(kv1.grad, kv0.grad, TOL, "grad kv")


def test_seq_attention_rejects_unsupported_head_dim():
    from pdvc.ops.functions.seq_attention import seq_attention
    x = torch.randn(1, 4, 40, device=DEV)
    with pytest.raises(RuntimeError, match="head_dim"):
        seq_attention(x, x, x, 2)  # head_dim 20
