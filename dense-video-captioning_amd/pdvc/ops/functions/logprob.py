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
from pdvc.precision import attach_bf16, shadow_for


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
