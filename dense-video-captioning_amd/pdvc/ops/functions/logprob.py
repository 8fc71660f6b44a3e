"""Caption word log-probabilities and the target word's log-probability as one autograd node:
    logp = log_softmax(logits, -1);  picked = logp.gather(-1, target)
(reference: Captioner.get_logprobs_state, pdvc/CaptioningHead/LSTM_DSA.py:112-116, and the gather inside
LanguageModelCriterion, LSTM_DSA.py:48-52).  csrc/logprob.hip does both in one pass over the logits and the
backward in one pass over logp (dlogits = g_picked * (onehot(target) - exp(logp))) -- no (rows, V) zero fill,
scatter or log_softmax_backward.  A gradient arriving on logp itself (only if a caller differentiates the
returned caption_probs) is added with the closed-form log_softmax backward.
"""
import torch
from torch.autograd import Function

from pdvc import _native as _n
from pdvc.precision import attach_bf16, bf16_active, shadow_for


class LogProbPickFunction(Function):
    @staticmethod
    def forward(ctx, logits, target):
        V = logits.shape[-1]
        x = logits.contiguous()
        tgt = target.to(torch.int64).contiguous()
        if tgt.shape != x.shape[:-1]:
            raise RuntimeError(f"logprob_pick: target shape {tuple(tgt.shape)} != logits rows {tuple(x.shape[:-1])}")
        if x.dtype != torch.float32 or not x.is_cuda:
            raise RuntimeError("logprob_pick: float32 GPU logits required")
        rows = tgt.numel()
        logp = torch.empty_like(x)
        picked = x.new_empty(tgt.shape)
        _n.call("pdvc_logprob_pick_forward_f32", _n.ptr(x), _n.ptr(tgt), rows, V, _n.ptr(logp), _n.ptr(picked),
                _n.stream())
        ctx.save_for_backward(logp, tgt)
        ctx.set_materialize_grads(False)
        return logp, picked

    @staticmethod
    def backward(ctx, g_logp, g_picked):
        logp, tgt = ctx.saved_tensors
        V = logp.shape[-1]
        if g_picked is None:
            g_picked = logp.new_zeros(tgt.shape)
        g_picked = g_picked.contiguous()
        grad = torch.empty_like(logp)
        g16 = shadow_for(grad) if g_logp is None else None  # bf16 mode: the logit GEMMs' operand, same pass
        done = False
        if g16 is not None:
            try:
                _n.call("pdvc_logprob_pick_backward_f32_bf16out", _n.ptr(logp), _n.ptr(tgt), _n.ptr(g_picked),
                        tgt.numel(), V, _n.ptr(grad), _n.ptr(g16), _n.stream())
                attach_bf16(grad, g16)
                done = True
            except _n.NativeError:  # not the register-resident row form: the GEMMs cast grad themselves
                pass
        if not done:
            _n.call("pdvc_logprob_pick_backward_f32", _n.ptr(logp), _n.ptr(tgt), _n.ptr(g_picked), tgt.numel(), V,
                    _n.ptr(grad), _n.stream())
        if g_logp is not None:
            grad.add_(g_logp - logp.exp() * g_logp.sum(-1, keepdim=True))
        return grad, None


def logprob_pick(logits, target):
    """(log_softmax(logits, -1), its entries at target) -- logits (..., V) fp32 on the GPU, target (...) int."""
    return LogProbPickFunction.apply(logits, target)


def _pick_forward(logits2, target):
    rows, V = logits2.shape
    tgt = target.to(torch.int64).reshape(-1).contiguous()
    if tgt.numel() != rows:
        raise RuntimeError(f"logprob_pick: target of {tgt.numel()} entries != {rows} logit rows")
    logp = torch.empty_like(logits2)
    picked = logits2.new_empty(rows)
    _n.call("pdvc_logprob_pick_forward_f32", _n.ptr(logits2), _n.ptr(tgt), rows, V, _n.ptr(logp), _n.ptr(picked),
            _n.stream())
    return logp, picked, tgt


class LogitPickFunction(Function):
    """The caption head's logit layer and logprob_pick as one node: logits = x W^T + b (LSTM_DSA.py:112-116), logp,
    picked.  The backward writes dlogits into rows padded to a multiple of 32 columns (zeros past V) so that the
    input-gradient product dlogits @ W runs on the in-tree GEMM (its K = V = vocab + 1 is not a multiple of 32: the
    unpadded product went to hipBLASLt at ~140 TF/s); the weight and bias gradients read the same buffer."""

    @staticmethod
    def forward(ctx, x, weight, bias, target):
        from .gemm3 import addmm_nt
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        logits = addmm_nt(bias, x2, weight)
        logp, picked, tgt = _pick_forward(logits, target)
        del logits
        ctx.save_for_backward(x2, weight, logp, tgt)
        ctx.has_bias = bias is not None
        ctx.lead = lead
        ctx.set_materialize_grads(False)
        return logp.view(*lead, -1), picked.view(lead)

    @staticmethod
    def backward(ctx, g_logp, g_picked):
        from .gemm3 import mm_dgrad
        from .linear import colsum, wgrad_mm
        x2, weight, logp, tgt = ctx.saved_tensors
        rows, V = logp.shape
        Vp = (V + 31) // 32 * 32
        gp = logp.new_zeros(rows) if g_picked is None else g_picked.reshape(-1).contiguous()
        G = torch.empty(rows, Vp, dtype=logp.dtype, device=logp.device)
        _n.call("pdvc_logprob_pick_backward_ld_f32", _n.ptr(logp), _n.ptr(tgt), _n.ptr(gp), rows, V, Vp, _n.ptr(G),
                _n.stream())
        Gv = G[:, :V]
        if g_logp is not None:
            gl = g_logp.reshape(rows, V)
            Gv.add_(gl - logp.exp() * gl.sum(-1, keepdim=True))
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            Wp = weight.new_zeros(Vp, weight.shape[1])
            Wp[:V] = weight
            gx = mm_dgrad(G, Wp).view(*ctx.lead, weight.shape[1])
        want_gb = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            # on the padded (rows, Vp) buffer (zeros past V): its width qualifies for gemm3w, where the strided
            # (rows, V) view made wgrad_mm fall back to a reshaped copy and a library GEMM; the
            # bias gradient from the same pass over G
            gbp = G.new_empty(G.shape[1]) if want_gb else None
            gw = wgrad_mm(G, x2, db=gbp)[:V]
            gb = gbp[:V] if want_gb else None
        elif want_gb:
            gb = colsum(G)[:V]
        return gx, gw, gb, None


def logit_pick(x, logit_layer, target):
    """logprob_pick(logit_layer(x), target) -- as one fused node on fp32 GPU tensors outside the bf16 mode (the bf16
    mode keeps the two nodes: its GEMMs read the bf16 shadow of dlogits)."""
    w, b = logit_layer.weight, logit_layer.bias
    if (x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and not bf16_active()
            and w.is_contiguous()):
        return LogitPickFunction.apply(x, w, b, target)
    return logprob_pick(logit_layer(x), target)
