// capgather.hip -- caption-head deformable sampling (MSDeformAttnCap) for MI355X (gfx950).
//
// Replaces MSDeformAttnCap.forward after value_proj (pdvc/ops/modules/ms_deform_attn_for_caption.py:92-121):
// sampling locations from the offset projection (ref dim 1: ref + off / T_l; dim 2: c + off / P * len * 0.5)
// and the *raw* bilinear samples with grid_sample's border padding (the reference always calls its Python
// core here, ms_deform_attn_func.py:58-59, even on a GPU).  The attention_weights softmax the reference
// computes is never used by the caption head, so it is not computed.
//
// Output layout is the one ShowAttendTellCore consumes after its reshape/permute (LSTM_DSA.py:241-242):
// samples (rows, M, L*P, D) -- each sample is one contiguous D-float row, written by one wave.
// Query rows come from many videos (ragged events per video): row_video maps a row to its video.
#include "pdvc_common.h"

namespace pdvc {

constexpr int cNS = 16, cP = 4, cL = 4;

struct CapLevels {
    int T[cL];
    int start[cL];
};

// grid_sampler_compute_source_index for border padding, align_corners=False, applied to grid = 2*loc-1.
// Returns the clipped pixel coordinate; gm = d(ix)/d(grid) (T/2, or 0 where clipped).
__device__ __forceinline__ float border_ix(float loc, int T, float& gm) {
    float ix = ((2.f * loc - 1.f) + 1.f) * (float)T;
    ix = (ix - 1.f) / 2.f;
    gm = (float)T / 2.f;
    if (ix <= 0.f) { ix = 0.f; gm = 0.f; }
    else if (ix >= (float)(T - 1)) { ix = (float)(T - 1); gm = 0.f; }
    return ix;
}

template <int CPL>
__device__ __forceinline__ void ld(VecF<CPL>& v, const float* __restrict__ p, bool ok) {
    if (ok) v.load(p);
    else v.zero();
}

template <int CPL, int LPH, int RD>
__global__ __launch_bounds__(256) void cap_gather_fwd_kernel(const float* __restrict__ value,
                                                              const uint8_t* __restrict__ vmask,
                                                              const int32_t* __restrict__ row_video,
                                                              const float* __restrict__ offsets, int off_stride,
                                                              int off_col0, const float* __restrict__ off_add,
                                                              const float* __restrict__ ref, int rd1_rows,
                                                              CapLevels lv, int S, int M, int D, int waves_per_row,
                                                              int total_waves, float* __restrict__ samples,
                                                              float* __restrict__ save_loc) {
    constexpr int HPW = 64 / LPH;
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wave >= total_waves) return;
    const int r = wave / waves_per_row;
    const int hg = wave - r * waves_per_row;
    const int sub = lane % LPH;
    const int m = hg * HPW + lane / LPH;
    if (m >= M) return;
    const int c0 = sub * CPL;
    const int b = row_video[r];
    const size_t MD = (size_t)M * D;
    const float* vbase = value + (size_t)b * S * MD + (size_t)m * D + c0;
    const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
    const float* orow = offsets + (size_t)r * off_stride + off_col0 + m * cNS;
    const bool centre_only = (RD == 1) || (r < rd1_rows);  // wave-uniform
#pragma unroll
    for (int l = 0; l < cL; ++l) {
        const int T = lv.T[l], st = lv.start[l];
        const float r0 = ref[((size_t)r * cL + l) * RD];
        const float r1 = (RD == 2) ? ref[((size_t)r * cL + l) * RD + 1] : 0.f;
        int x0[cP];
        float nw[cP], ne[cP];
#pragma unroll
        for (int p = 0; p < cP; ++p) {
            const int j = l * cP + p;
            const float off = off_add ? orow[j] + off_add[((size_t)r * M + m) * cNS + j] : orow[j];
            const float loc = centre_only ? r0 + off / (float)T : r0 + ((off / (float)cP) * r1) * 0.5f;
            if (save_loc && sub == (j % LPH)) save_loc[((size_t)r * M + m) * cNS + j] = loc;
            float gm;
            const float ix = border_ix(loc, T, gm);
            const float xf = floorf(ix);
            x0[p] = (int)xf;
            // iy == 0 (H == 1): nw = (x0+1-ix)*1, ne = (ix-x0)*1, the y0+1 row is outside
            nw[p] = ((float)(x0[p] + 1) - ix);
            ne[p] = (ix - xf);
        }
        VecF<CPL> v0[cP], v1[cP];
        bool ok0[cP], ok1[cP];
#pragma unroll
        for (int p = 0; p < cP; ++p) {  // the level's 2*P rows in flight together (clamped, selected after)
            const int a1 = min(x0[p] + 1, T - 1);
            v0[p].load(vbase + (size_t)(st + x0[p]) * MD);
            v1[p].load(vbase + (size_t)(st + a1) * MD);
            ok0[p] = !(mbase && mbase[st + x0[p]]);
            ok1[p] = x0[p] + 1 < T && !(mbase && mbase[st + a1]);
        }
#pragma unroll
        for (int p = 0; p < cP; ++p) {
            VecF<CPL> o;
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                o.v[c] = (ok0[p] ? v0[p].v[c] : 0.f) * nw[p] + (ok1[p] ? v1[p].v[c] : 0.f) * ne[p];
            o.store(samples + (((size_t)r * M + m) * cNS + l * cP + p) * D + c0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int CPL, int LPH, int RD>
__global__ __launch_bounds__(256) void cap_gather_bwd_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const int32_t* __restrict__ row_video,
    const float* __restrict__ offsets, int off_stride, int off_col0, const float* __restrict__ off_add,
    const float* __restrict__ ref, int rd1_rows, CapLevels lv, int S, int M, int D, int waves_per_row,
    int total_waves, const float* __restrict__ save_loc,
    const float* __restrict__ gsamp, float* __restrict__ grad_value, float* __restrict__ grad_off,
    float* __restrict__ grad_ref) {
    constexpr int HPW = 64 / LPH;
    constexpr int G = LPH < 16 ? LPH : 16;  // reduce-scatter group; the rest is an all-reduce
    constexpr int SPL = cNS / G;
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wave >= total_waves) return;
    const int r = wave / waves_per_row;
    const int hg = wave - r * waves_per_row;
    const int sub = lane % LPH;
    const int m_raw = hg * HPW + lane / LPH;
    const bool active = m_raw < M;
    const int m = active ? m_raw : 0;
    const int c0 = sub * CPL;
    const int b = row_video[r];
    const size_t MD = (size_t)M * D;
    const float* vbase = value + (size_t)b * S * MD + (size_t)m * D + c0;
    float* gvbase = grad_value + (size_t)b * S * MD + (size_t)m * D + c0;
    const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;

    float part[cNS];
#pragma unroll
    for (int l = 0; l < cL; ++l) {
        const int T = lv.T[l], st = lv.start[l];
        int x0[cP];
        float nw[cP], ne[cP];
#pragma unroll
        for (int p = 0; p < cP; ++p) {
            const float loc = active ? save_loc[((size_t)r * M + m) * cNS + l * cP + p] : 0.f;
            float gm;
            const float ix = border_ix(loc, T, gm);
            const float xf = floorf(ix);
            x0[p] = (int)xf;
            nw[p] = ((float)(x0[p] + 1) - ix);
            ne[p] = (ix - xf);
        }
        VecF<CPL> g[cP], v0[cP], v1[cP];
        bool ok0[cP], ok1[cP];
#pragma unroll
        for (int p = 0; p < cP; ++p) {
            const int a1 = min(x0[p] + 1, T - 1);
            g[p].load(gsamp + (((size_t)r * M + m) * cNS + l * cP + p) * D + c0);
            v0[p].load(vbase + (size_t)(st + x0[p]) * MD);
            v1[p].load(vbase + (size_t)(st + a1) * MD);
            ok0[p] = active && !(mbase && mbase[st + x0[p]]);
            ok1[p] = active && x0[p] + 1 < T && !(mbase && mbase[st + a1]);
        }
#pragma unroll
        for (int p = 0; p < cP; ++p) {
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const float gv = active ? g[p].v[c] : 0.f;
                if (ok0[p]) atomicAdd(gvbase + (size_t)(st + x0[p]) * MD + c, nw[p] * gv);
                if (ok1[p]) atomicAdd(gvbase + (size_t)(st + x0[p] + 1) * MD + c, ne[p] * gv);
                s += gv * ((ok1[p] ? v1[p].v[c] : 0.f) - (ok0[p] ? v0[p].v[c] : 0.f));  // gix = -vnw + vne
            }
            part[l * cP + p] = s;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    group_reduce_scatter<cNS, G>(part, lane);
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
#pragma unroll
        for (int d = G; d < LPH; d <<= 1) part[k] += __shfl_xor(part[k], d, PDVC_WAVE);
    }
    float gr0[cL], gr1[cL];
#pragma unroll
    for (int l = 0; l < cL; ++l) { gr0[l] = 0.f; gr1[l] = 0.f; }
    const bool owner = active && sub < G;
    const int gsub = sub % G;
    const bool centre_only = (RD == 1) || (r < rd1_rows);
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        const int j = gsub * SPL + k;
        const int l = j / cP;
        const int T = lv.T[l];
        const float loc = active ? save_loc[((size_t)r * M + m) * cNS + j] : 0.f;
        float gm;
        border_ix(loc, T, gm);
        const float gloc = 2.f * (gm * part[k]);  // grid = 2*loc - 1
        float goff;
        if (centre_only) {
            goff = gloc / (float)T;
#pragma unroll
            for (int ll = 0; ll < cL; ++ll) if (ll == l && owner) gr0[ll] += gloc;
        } else {
            const float r1 = ref[((size_t)r * cL + l) * 2 + 1];
            const float t2 = gloc * 0.5f;
            goff = (t2 * r1) / (float)cP;
            float o = active ? offsets[(size_t)r * off_stride + off_col0 + m * cNS + j] : 0.f;
            if (active && off_add) o += off_add[((size_t)r * M + m) * cNS + j];
#pragma unroll
            for (int ll = 0; ll < cL; ++ll)
                if (ll == l && owner) { gr0[ll] += gloc; gr1[ll] += t2 * (o / (float)cP); }
        }
        if (owner) grad_off[(size_t)r * off_stride + off_col0 + m * cNS + j] = goff;
    }
    if (grad_ref) {
#pragma unroll
        for (int l = 0; l < cL; ++l) {
            float v0 = gr0[l], v1 = gr1[l];
#pragma unroll
            for (int d = 32; d > 0; d >>= 1) {
                v0 += __shfl_xor(v0, d, PDVC_WAVE);
                if (RD == 2) v1 += __shfl_xor(v1, d, PDVC_WAVE);
            }
            if (lane == 0) {
                atomicAdd(grad_ref + ((size_t)r * cL + l) * RD, v0);
                if (RD == 2) atomicAdd(grad_ref + ((size_t)r * cL + l) * RD + 1, v1);
            }
        }
    }
}

static int cap_setup(const int32_t* level_T, int num_levels, int num_point, int head_dim, int num_heads, int ref_dim,
                     CapLevels& lv, int& S, int& lph, int& wpr) {
    PDVC_CHECK_ARG(level_T != nullptr, "level_T must not be NULL");
    if (num_levels != cL || num_point != cP)
        return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "caption gather needs %d levels x %d points (got %d x %d)", cL, cP,
                              num_levels, num_point);
    PDVC_CHECK_ARG(ref_dim == 1 || ref_dim == 2, "ref_dim must be 1 or 2, got %d", ref_dim);
    S = 0;
    for (int l = 0; l < cL; ++l) {
        PDVC_CHECK_ARG(level_T[l] > 0, "level %d has non-positive length", l);
        lv.T[l] = level_T[l];
        lv.start[l] = S;
        S += level_T[l];
    }
    if (head_dim % 8 != 0 || head_dim < 32 || head_dim > 512 || (head_dim & (head_dim - 1)) != 0)
        return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "caption gather supports head_dim 32..512 (power of 2), got %d",
                              head_dim);
    lph = head_dim / 8;
    const int hpw = 64 / lph;
    wpr = (num_heads + hpw - 1) / hpw;
    return PDVC_OK;
}

}  // namespace pdvc

using namespace pdvc;

#define CAP_DISPATCH(KERNEL, RD, grid, s, ...)                                                                   \
    switch (lph) {                                                                                               \
        case 4: hipLaunchKernelGGL((KERNEL<8, 4, RD>), grid, dim3(256), 0, s, __VA_ARGS__); break;              \
        case 8: hipLaunchKernelGGL((KERNEL<8, 8, RD>), grid, dim3(256), 0, s, __VA_ARGS__); break;              \
        case 16: hipLaunchKernelGGL((KERNEL<8, 16, RD>), grid, dim3(256), 0, s, __VA_ARGS__); break;            \
        case 32: hipLaunchKernelGGL((KERNEL<8, 32, RD>), grid, dim3(256), 0, s, __VA_ARGS__); break;            \
        default: hipLaunchKernelGGL((KERNEL<8, 64, RD>), grid, dim3(256), 0, s, __VA_ARGS__); break;            \
    }

extern "C" int pdvc_cap_gather_forward_f32(const float* value, const uint8_t* value_pad_mask, const int32_t* row_video,
                                           const float* offsets, int off_stride, int off_col0, const float* off_add,
                                           const float* ref,
                                           int ref_dim, int rd1_rows, const int32_t* level_T, int num_levels, int batch, int rows,
                                           int num_heads, int head_dim, int num_point, float* samples, float* save_loc,
                                           void* stream) {
    CapLevels lv;
    int S, lph, wpr;
    int rc = cap_setup(level_T, num_levels, num_point, head_dim, num_heads, ref_dim, lv, S, lph, wpr);
    if (rc) return rc;
    PDVC_CHECK_ARG(batch >= 0 && rows >= 0, "negative sizes");
    PDVC_CHECK_ARG(off_col0 >= 0 && off_col0 + num_heads * cNS <= off_stride, "offset columns out of range");
    const long tw = (long)rows * wpr;
    if (tw == 0) return PDVC_OK;
    dim3 grid((unsigned)((tw + 3) / 4));
    hipStream_t s = (hipStream_t)stream;
    if (ref_dim == 1) {
        CAP_DISPATCH(cap_gather_fwd_kernel, 1, grid, s, value, value_pad_mask, row_video, offsets, off_stride, off_col0,
                     off_add, ref, rd1_rows, lv, S, num_heads, head_dim, wpr, (int)tw, samples, save_loc)
    } else {
        CAP_DISPATCH(cap_gather_fwd_kernel, 2, grid, s, value, value_pad_mask, row_video, offsets, off_stride, off_col0,
                     off_add, ref, rd1_rows, lv, S, num_heads, head_dim, wpr, (int)tw, samples, save_loc)
    }
    PDVC_CHECK_LAUNCH("cap_gather_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_cap_gather_backward_f32(const float* value, const uint8_t* value_pad_mask,
                                            const int32_t* row_video, const float* offsets, int off_stride,
                                            int off_col0, const float* off_add, const float* ref, int ref_dim,
                                            int rd1_rows,
                                            const int32_t* level_T,
                                            int num_levels, int batch, int rows, int num_heads, int head_dim,
                                            int num_point, const float* save_loc, const float* grad_samples,
                                            float* grad_value, float* grad_offsets, float* grad_ref, void* stream) {
    CapLevels lv;
    int S, lph, wpr;
    int rc = cap_setup(level_T, num_levels, num_point, head_dim, num_heads, ref_dim, lv, S, lph, wpr);
    if (rc) return rc;
    PDVC_CHECK_ARG(save_loc != nullptr, "backward needs save_loc from the forward");
    PDVC_CHECK_ARG(off_col0 >= 0 && off_col0 + num_heads * cNS <= off_stride, "offset columns out of range");
    hipStream_t s = (hipStream_t)stream;
    const long tw = (long)rows * wpr;
    if (tw == 0) return PDVC_OK;
    dim3 grid((unsigned)((tw + 3) / 4));
    if (ref_dim == 1) {
        CAP_DISPATCH(cap_gather_bwd_kernel, 1, grid, s, value, value_pad_mask, row_video, offsets, off_stride, off_col0,
                     off_add, ref, rd1_rows, lv, S, num_heads, head_dim, wpr, (int)tw, save_loc, grad_samples,
                     grad_value, grad_offsets, grad_ref)
    } else {
        CAP_DISPATCH(cap_gather_bwd_kernel, 2, grid, s, value, value_pad_mask, row_video, offsets, off_stride, off_col0,
                     off_add, ref, rd1_rows, lv, S, num_heads, head_dim, wpr, (int)tw, save_loc, grad_samples,
                     grad_value, grad_offsets, grad_ref)
    }
    PDVC_CHECK_LAUNCH("cap_gather_bwd_kernel");
    return PDVC_OK;
}
