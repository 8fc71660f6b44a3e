"""The encoder's self-attention sub-layer as one autograd node:
    out = norm(src + dropout(output_proj(MSDA(value_proj(src), proj(src + pos)))))
(reference: DeformableTransformerEncoderLayer.forward, deformable_transformer.py:147-151, and MSDeformAttn.forward,
ms_deform_attn.py:79-126).  Same kernels and GEMMs as the module chain; what the single node changes is where the
gradients of src meet:
  * src's three gradient paths (residual from the layer norm, value projection, query projection) accumulate in
    the epilogues of the two input-gradient GEMMs (beta = 1) instead of two autograd adds over (N*S, d);
  * output_proj's bias gradient comes out of the layer-norm backward pass (pdvc_add_dropout_layernorm ds_colsum);
  * the residual sum src + dropout(output_proj(...)) is formed in output_proj's gemm3 epilogue
    (pdvc_gemm3p_resid_dropout_f32), so the add-norm pass reads one tensor instead of two each way;
  * with a level-position handle (ops/functions/posembed.py) the position gradient is returned as per-(video,
    level) sums, sum_rows(d_proj) @ W_q, so the (N*S, d) position gradient is never formed nor accumulated over
    layers.
"""
import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from pdvc import _native as _n
from .addnorm import BWD_PARTS, an_backward, an_forward
from .gemm3 import addmm_nt, addmm_resid_dropout_nt, mm_dgrad
from .linear import wgrad_mm
from .ms_deform_attn_func import NUM_SAMPLES, msda1d_backward, msda1d_forward
from .posembed import LevelPos, level_row_sums


class EncoderAttnBlockFunction(Function):
    @staticmethod
    def forward(ctx, src, pos, handle, ref, pad_mask, Wv, bv, Wq, bq, Wo, bo, gamma, beta, p, eps, seed, level_T, M):
        N, S, d = src.shape
        R = N * S
        D = d // M
        src2 = src.reshape(R, d).contiguous()
        q = pos.add_to(src2) if isinstance(pos, LevelPos) else src2 + pos.reshape(R, d)
        value = addmm_nt(bv, src2, Wv)
        proj = addmm_nt(bq, q, Wq)
        nq = M * NUM_SAMPLES
        ref = ref.contiguous()
        out, save_attn, save_loc = msda1d_forward(value.view(N, S, M, D), pad_mask, proj.view(N, S, -1), ref,
                                                  level_T, 0, nq)
        y = torch.empty_like(src2)
        mean = torch.empty(R, dtype=src.dtype, device=src.device)
        rstd = torch.empty_like(mean)
        seed_dev = seed if isinstance(seed, torch.Tensor) else None
        seed_int = 0 if seed_dev is not None else int(seed)
        # output_proj's epilogue forms src + dropout(s2) (the add-norm pass's mask bits, device seed), and the pass
        # reads that sum alone each way; s2 then holds the sum
        s2 = None
        if seed_dev is not None or p == 0:
            s2 = addmm_resid_dropout_nt(bo, out.view(R, d), Wo, src2, float(p),
                                        _n.ptr(seed_dev) if seed_dev is not None else None)
        fused_sum = s2 is not None
        if fused_sum:
            an_forward(s2, None, gamma, beta, 0.0, 0, None, eps, y, mean, rstd)
        else:
            s2 = addmm_nt(bo, out.view(R, d), Wo)
            an_forward(src2, s2, gamma, beta, p, seed_int, seed_dev, eps, y, mean, rstd)
        ctx.save_for_backward(src2, q, value, proj, ref, pad_mask, save_attn, save_loc, out, s2, Wv, Wq, Wo, gamma,
                              mean, rstd, seed_dev)
        ctx.meta = (N, S, d, M, float(p), seed_int, tuple(level_T), handle is not None, fused_sum)
        return y.view(N, S, d)

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        (src2, q, value, proj, ref, pad_mask, save_attn, save_loc, out, s2, Wv, Wq, Wo, gamma, mean, rstd,
         seed_dev) = ctx.saved_tensors
        N, S, d, M, p, seed_int, level_T, has_handle, fused_sum = ctx.meta
        R = N * S
        D = d // M
        dy2 = dy.reshape(R, d).contiguous()
        d_src = torch.empty_like(src2)
        d_s2 = torch.empty_like(s2)
        dgamma = torch.empty_like(gamma)
        dbeta = torch.empty_like(gamma)
        dbo = torch.empty_like(gamma)
        ws = torch.empty(3 * BWD_PARTS * d, dtype=src2.dtype, device=src2.device)
        if fused_sum:  # s2 holds src + dropout(output_proj(out))
            an_backward(s2, None, gamma, mean, rstd, dy2, p, seed_int, seed_dev, d_src, d_s2, dgamma, dbeta, dbo, ws)
        else:
            an_backward(src2, s2, gamma, mean, rstd, dy2, p, seed_int, seed_dev, d_src, d_s2, dgamma, dbeta, dbo, ws)
        dWo = wgrad_mm(d_s2, out.view(R, d))
        d_out = mm_dgrad(d_s2, Wo)
        nq = M * NUM_SAMPLES
        gv, gp, _, vsums = msda1d_backward(value.view(N, S, M, D), pad_mask, proj.view(N, S, -1), ref, save_attn,
                                           save_loc, out, d_out.view(N, S, d), level_T, 0, nq,
                                           level_sums=d % 4 == 0)
        gv2 = gv.view(R, d)
        gp2 = gp.view(R, -1)
        # the value bias gradient from the value-gradient kernel's per-(video, level) row sums
        if vsums is not None:
            dbv = vsums.view(-1, d).sum(0)
            dWv = wgrad_mm(gv2, src2)
        else:
            dbv = gv2.new_empty(d)
            dWv = wgrad_mm(gv2, src2, db=dbv)
        dbq = gp2.new_empty(gp2.shape[1])  # the sampling / attention-weight bias gradient, from dWq's pass over gp2
        dWq = wgrad_mm(gp2, q, db=dbq)
        d_pos = d_handle = None
        if has_handle:
            d_handle = torch.matmul(level_row_sums(gp.view(N, S, -1), level_T), Wq)
            mm_dgrad(gp2, Wq, out=d_src)
        elif ctx.needs_input_grad[1]:
            d_q = mm_dgrad(gp2, Wq)
            d_pos = d_q.view(N, S, d)
            d_src.add_(d_q)
        else:
            mm_dgrad(gp2, Wq, out=d_src)
        mm_dgrad(gv2, Wv, out=d_src)  # residual + value path + query path, accumulated in the GEMM epilogues
        return (d_src.view(N, S, d), d_pos, d_handle, None, None, dWv, dbv, dWq, dbq, dWo, dbo, dgamma, dbeta,
                None, None, None, None, None)


def use_attn_block(src, layer):
    """EncoderAttnBlockFunction serves fp32 GPU rows whose MSDeformAttn takes the fused 1-D kernels, on the
    torch/hipBLASLt GEMM backend."""
    from . import linear as _lin
    return (src.is_cuda and src.dtype == torch.float32 and layer.self_attn.fused and _lin.BACKEND != "hip"
            and layer.self_attn.d_model % layer.self_attn.n_heads == 0)


def encoder_attn_block(layer, src, pos, handle, reference_points, level_T, padding_mask):
    """norm1(src + dropout1(self_attn(src + pos, ...))) of a DeformableTransformerEncoderLayer."""
    sa = layer.self_attn
    mask = None if padding_mask is None else padding_mask.contiguous().view(torch.uint8)
    Wq = torch.cat([sa.sampling_offsets.weight, sa.attention_weights.weight], 0)
    bq = torch.cat([sa.sampling_offsets.bias, sa.attention_weights.bias], 0)
    p = float(layer.dropout1.p) if layer.training else 0.0
    seed = torch.randint(0, 2 ** 62, (1,), device=src.device, dtype=torch.int64) if p > 0 else 0
    return EncoderAttnBlockFunction.apply(src, pos, handle, reference_points, mask, sa.value_proj.weight,
                                          sa.value_proj.bias, Wq, bq, sa.output_proj.weight, sa.output_proj.bias,
                                          layer.norm1.weight, layer.norm1.bias, p, layer.norm1.eps, seed,
                                          tuple(level_T), sa.n_heads)
