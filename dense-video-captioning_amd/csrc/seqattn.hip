// seqattn.hip -- long-sequence multi-head attention core for the dual-modality front-end of cfgs/yc2_newModel_sound
// (reference: NewModel.visual_self_attention / visual_sound_attention, NewModel.py:41-65: nn.MultiheadAttention(768,
// 32 heads, batch_first) over the T clip features, queries = clips or sound features).  T = 512 queries and keys,
// head_dim 24: outside the decoder kernel's range (mha.hip: Q <= 300), and a (T x T) score matrix per head is
// 1 MB, so nothing of size T^2 is ever written: flash-style, one lane per query (forward, dq) or per key (dk, dv),
// the other side streamed through LDS in 128-row tiles that every lane of the workgroup reads as a broadcast.
//   forward:  out_i = sum_j softmax_j(scale q_i.k_j) v_j, lse_i saved (running max / sum, rescaled on a new max)
//   backward: delta_i = dout_i.out_i;  p_ij = exp(scale q_i.k_j - lse_i);  ds_ij = p_ij (dout_i.v_j - delta_i)
//             dq_i = scale sum_j ds_ij k_j  (query lanes);  dk_j = scale sum_i ds_ij q_i, dv_j = sum_i p_ij dout_i
//             (key lanes) -- every gradient row has exactly one writer, no atomics.
// Exponentials on the hardware exp2 (__expf: ~1 ulp of expf, well inside the 1e-4 parity bound).
// No dropout and no key padding: the front-end uses neither (nn.MultiheadAttention defaults, all clips valid).
#include <math.h>

#include "pdvc_common.h"

namespace pdvc {

constexpr int kSqT = 128;   // lanes (queries or keys) per workgroup
constexpr int kSqTile = 128;  // rows of the other side per LDS tile

// rows [r0, r0 + n) of a (T, ld) head slice -> LDS [n][D]; missing rows zero
template <int D>
__device__ __forceinline__ void sq_stage(float* lds, const float* src, long ld, int r0, int n, int T) {
    for (int e = threadIdx.x; e < n * D; e += kSqT) {
        const int r = e / D, c = e - r * D;
        lds[e] = (r0 + r < T) ? src[(long)(r0 + r) * ld + c] : 0.f;
    }
}

template <int D, int R>
__global__ __launch_bounds__(kSqT) void seqattn_fwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                           const float* __restrict__ v, int H, int Tq, int Tk,
                                                           long ldq, long ldk, long ldv, float scale,
                                                           float* __restrict__ out, float* __restrict__ lse) {
    __shared__ float ks[kSqTile * D], vs[kSqTile * D];
    const int nh = blockIdx.y, n = nh / H, h = nh - n * H;
    const float* qh = q + (long)n * Tq * ldq + h * D;
    const float* kh = k + (long)n * Tk * ldk + h * D;
    const float* vh = v + (long)n * Tk * ldv + h * D;
    float qi[R][D], acc[R][D], m[R], l[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = blockIdx.x * kSqT * R + r * kSqT + threadIdx.x;
#pragma unroll
        for (int c = 0; c < D; ++c) {
            qi[r][c] = i < Tq ? qh[(long)i * ldq + c] * scale : 0.f;
            acc[r][c] = 0.f;
        }
        m[r] = -INFINITY;
        l[r] = 0.f;
    }
    for (int t0 = 0; t0 < Tk; t0 += kSqTile) {
        const int nt = min(kSqTile, Tk - t0);
        __syncthreads();
        sq_stage<D>(ks, kh, ldk, t0, nt, Tk);
        sq_stage<D>(vs, vh, ldv, t0, nt, Tk);
        __syncthreads();
        for (int j = 0; j < nt; ++j) {
            float kv[D];
#pragma unroll
            for (int c = 0; c < D; ++c) kv[c] = ks[j * D + c];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float s = 0.f;
#pragma unroll
                for (int c = 0; c < D; ++c) s += qi[r][c] * kv[c];
                if (s > m[r]) {
                    const float corr = __expf(m[r] - s);
                    l[r] *= corr;
#pragma unroll
                    for (int c = 0; c < D; ++c) acc[r][c] *= corr;
                    m[r] = s;
                }
                const float p = __expf(s - m[r]);
                l[r] += p;
#pragma unroll
                for (int c = 0; c < D; ++c) acc[r][c] += p * vs[j * D + c];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = blockIdx.x * kSqT * R + r * kSqT + threadIdx.x;
        if (i < Tq) {
            const float inv = 1.f / l[r];
            float* o = out + ((long)n * Tq + i) * H * D + h * D;
#pragma unroll
            for (int c = 0; c < D; ++c) o[c] = acc[r][c] * inv;
            lse[(long)nh * Tq + i] = m[r] + logf(l[r]);
        }
    }
}

template <int D, int R>
__global__ __launch_bounds__(kSqT) void seqattn_bwd_dq_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                              const float* __restrict__ v,
                                                              const float* __restrict__ dout,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ out,
                                                              float* __restrict__ delta, int H, int Tq, int Tk,
                                                              long ldq, long ldk, long ldv, float scale,
                                                              float* __restrict__ dq, long lddq) {
    __shared__ float ks[kSqTile * D], vs[kSqTile * D];
    const int nh = blockIdx.y, n = nh / H, h = nh - n * H;
    const float* qh = q + (long)n * Tq * ldq + h * D;
    const float* kh = k + (long)n * Tk * ldk + h * D;
    const float* vh = v + (long)n * Tk * ldv + h * D;
    const float* gh = dout + (long)n * Tq * H * D + h * D;
    float qi[R][D], gi[R][D], acc[R][D], li[R], di[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = blockIdx.x * kSqT * R + r * kSqT + threadIdx.x;
        const bool act = i < Tq;
#pragma unroll
        for (int c = 0; c < D; ++c) {
            qi[r][c] = act ? qh[(long)i * ldq + c] * scale : 0.f;
            gi[r][c] = act ? gh[(long)i * H * D + c] : 0.f;
            acc[r][c] = 0.f;
        }
        li[r] = act ? lse[(long)nh * Tq + i] : 0.f;
        // delta_i = dout_i . out_i, from the lane's own rows; published for the dk/dv kernel launched after this
        float dsum = 0.f;
        if (act) {
            const float* oh = out + ((long)n * Tq + i) * H * D + h * D;
#pragma unroll
            for (int c = 0; c < D; ++c) dsum += gi[r][c] * oh[c];
            delta[(long)nh * Tq + i] = dsum;
        }
        di[r] = dsum;
    }
    for (int t0 = 0; t0 < Tk; t0 += kSqTile) {
        const int nt = min(kSqTile, Tk - t0);
        __syncthreads();
        sq_stage<D>(ks, kh, ldk, t0, nt, Tk);
        sq_stage<D>(vs, vh, ldv, t0, nt, Tk);
        __syncthreads();
        for (int j = 0; j < nt; ++j) {
            float kv[D], vv[D];
#pragma unroll
            for (int c = 0; c < D; ++c) {
                kv[c] = ks[j * D + c];
                vv[c] = vs[j * D + c];
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float s = 0.f, dp = 0.f;
#pragma unroll
                for (int c = 0; c < D; ++c) {
                    s += qi[r][c] * kv[c];
                    dp += gi[r][c] * vv[c];
                }
                const float ds = __expf(s - li[r]) * (dp - di[r]);
#pragma unroll
                for (int c = 0; c < D; ++c) acc[r][c] += ds * kv[c];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = blockIdx.x * kSqT * R + r * kSqT + threadIdx.x;
        if (i < Tq) {
            float* o = dq + ((long)n * Tq + i) * lddq + h * D;
#pragma unroll
            for (int c = 0; c < D; ++c) o[c] = acc[r][c] * scale;
        }
    }
}

template <int D, int R>
__global__ __launch_bounds__(kSqT) void seqattn_bwd_dkv_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                               const float* __restrict__ v,
                                                               const float* __restrict__ dout,
                                                               const float* __restrict__ lse,
                                                               const float* __restrict__ delta, int H, int Tq, int Tk,
                                                               long ldq, long ldk, long ldv, float scale,
                                                               float* __restrict__ dk, long lddk,
                                                               float* __restrict__ dv, long lddv) {
    __shared__ float qs[kSqTile * D], gs[kSqTile * D], ls[kSqTile], dls[kSqTile];
    const int nh = blockIdx.y, n = nh / H, h = nh - n * H;
    const float* qh = q + (long)n * Tq * ldq + h * D;
    const float* kh = k + (long)n * Tk * ldk + h * D;
    const float* vh = v + (long)n * Tk * ldv + h * D;
    const float* gh = dout + (long)n * Tq * H * D + h * D;
    float kj[R][D], vj[R][D], ak[R][D], av[R][D];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = blockIdx.x * kSqT * R + r * kSqT + threadIdx.x;
        const bool act = j < Tk;
#pragma unroll
        for (int c = 0; c < D; ++c) {
            kj[r][c] = act ? kh[(long)j * ldk + c] * scale : 0.f;
            vj[r][c] = act ? vh[(long)j * ldv + c] : 0.f;
            ak[r][c] = 0.f;
            av[r][c] = 0.f;
        }
    }
    for (int t0 = 0; t0 < Tq; t0 += kSqTile) {
        const int nt = min(kSqTile, Tq - t0);
        __syncthreads();
        sq_stage<D>(qs, qh, ldq, t0, nt, Tq);
        sq_stage<D>(gs, gh, (long)H * D, t0, nt, Tq);
        for (int e = threadIdx.x; e < nt; e += kSqT) {
            ls[e] = lse[(long)nh * Tq + t0 + e];
            dls[e] = delta[(long)nh * Tq + t0 + e];
        }
        __syncthreads();
        for (int i = 0; i < nt; ++i) {
            float qv[D], gv[D];
#pragma unroll
            for (int c = 0; c < D; ++c) {
                qv[c] = qs[i * D + c];
                gv[c] = gs[i * D + c];
            }
            const float li = ls[i], di = dls[i];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float s = 0.f, dp = 0.f;
#pragma unroll
                for (int c = 0; c < D; ++c) {
                    s += kj[r][c] * qv[c];
                    dp += vj[r][c] * gv[c];
                }
                const float p = __expf(s - li);
                const float ds = p * (dp - di);
#pragma unroll
                for (int c = 0; c < D; ++c) {
                    av[r][c] += p * gv[c];
                    ak[r][c] += ds * qv[c];
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = blockIdx.x * kSqT * R + r * kSqT + threadIdx.x;
        if (j < Tk) {
            float* ok = dk + ((long)n * Tk + j) * lddk + h * D;
            float* ov = dv + ((long)n * Tk + j) * lddv + h * D;
#pragma unroll
            for (int c = 0; c < D; ++c) {
                ok[c] = ak[r][c] * scale;
                ov[c] = av[r][c];
            }
        }
    }
}

#define PDVC_SQ_DISPATCH(D_, CALL) \
    switch (D_) {                  \
        case 16: CALL(16); break;  \
        case 24: CALL(24); break;  \
        case 32: CALL(32); break;  \
        case 48: CALL(48); break;  \
        case 64: CALL(64); break;  \
        default: break;            \
    }

// query rows per lane in the forward and dq kernels: 2 for head_dim <= 32 (each key row read from LDS serves two
// queries), 1 above (register budget)
static constexpr int sq_rows_per_lane(int D) { return D <= 32 ? 2 : 1; }

// key rows per lane in the dk/dv kernel: 2 for head_dim <= 24 (four D-vectors per key row live in registers)
static constexpr int sq_keys_per_lane(int D) { return D <= 24 ? 2 : 1; }

static bool sq_head_dim_ok(int D) { return D == 16 || D == 24 || D == 32 || D == 48 || D == 64; }

}  // namespace pdvc

using namespace pdvc;

extern "C" int pdvc_seq_attention_forward_f32(const float* q, long ldq, const float* k, long ldk, const float* v,
                                              long ldv, int batch, int num_query, int num_key, int num_heads,
                                              int head_dim, float* out, float* lse, void* stream) {
    PDVC_CHECK_ARG(batch >= 0 && num_query >= 0 && num_key > 0 && num_heads > 0, "invalid sizes");
    PDVC_CHECK_ARG(sq_head_dim_ok(head_dim), "head_dim must be 16, 24, 32, 48 or 64, got %d", head_dim);
    const long E = (long)num_heads * head_dim;
    PDVC_CHECK_ARG(ldq >= E && ldk >= E && ldv >= E, "row strides must be >= num_heads * head_dim");
    PDVC_CHECK_ARG((long)batch * num_heads < 65536, "batch * num_heads must be < 65536");
    if (batch == 0 || num_query == 0) return PDVC_OK;
    const float scale = 1.f / sqrtf((float)head_dim);
    const int R = sq_rows_per_lane(head_dim);
    dim3 grid((unsigned)((num_query + kSqT * R - 1) / (kSqT * R)), (unsigned)(batch * num_heads));
    hipStream_t s = (hipStream_t)stream;
#define PDVC_SQ_FWD(DD)                                                                                              \
    if (sq_rows_per_lane(DD) == 2)                                                                                   \
        hipLaunchKernelGGL((seqattn_fwd_kernel<DD, 2>), grid, dim3(kSqT), 0, s, q, k, v, num_heads, num_query,       \
                           num_key, ldq, ldk, ldv, scale, out, lse);                                                \
    else                                                                                                             \
        hipLaunchKernelGGL((seqattn_fwd_kernel<DD, 1>), grid, dim3(kSqT), 0, s, q, k, v, num_heads, num_query,       \
                           num_key, ldq, ldk, ldv, scale, out, lse)
    PDVC_SQ_DISPATCH(head_dim, PDVC_SQ_FWD)
#undef PDVC_SQ_FWD
    PDVC_CHECK_LAUNCH("seqattn_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_seq_attention_backward_f32(const float* q, long ldq, const float* k, long ldk, const float* v,
                                               long ldv, const float* out, const float* grad_out, const float* lse,
                                               int batch, int num_query, int num_key, int num_heads, int head_dim,
                                               float* workspace, float* grad_q, long ld_grad_q, float* grad_k,
                                               long ld_grad_k, float* grad_v, long ld_grad_v, void* stream) {
    PDVC_CHECK_ARG(batch >= 0 && num_query >= 0 && num_key > 0 && num_heads > 0, "invalid sizes");
    PDVC_CHECK_ARG(sq_head_dim_ok(head_dim), "head_dim must be 16, 24, 32, 48 or 64, got %d", head_dim);
    const long E = (long)num_heads * head_dim;
    PDVC_CHECK_ARG(ldq >= E && ldk >= E && ldv >= E && ld_grad_q >= E && ld_grad_k >= E && ld_grad_v >= E,
                   "row strides must be >= num_heads * head_dim");
    PDVC_CHECK_ARG((long)batch * num_heads < 65536, "batch * num_heads must be < 65536");
    if (batch == 0) return PDVC_OK;
    hipStream_t s = (hipStream_t)stream;
    const float scale = 1.f / sqrtf((float)head_dim);
    if (num_query == 0) {  // no query: the key and value gradients are zero
        hipError_t e1 = hipMemset2DAsync(grad_k, sizeof(float) * ld_grad_k, 0, sizeof(float) * E,
                                         (size_t)batch * num_key, s);
        hipError_t e2 = hipMemset2DAsync(grad_v, sizeof(float) * ld_grad_v, 0, sizeof(float) * E,
                                         (size_t)batch * num_key, s);
        if (e1 != hipSuccess || e2 != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "memset grad_k/grad_v");
        return PDVC_OK;
    }
    float* delta = workspace;  // (N, H, Tq): written by the dq kernel, read by the dk/dv kernel
    const int R = sq_rows_per_lane(head_dim);
    dim3 gq((unsigned)((num_query + kSqT * R - 1) / (kSqT * R)), (unsigned)(batch * num_heads));
    const int RK = sq_keys_per_lane(head_dim);
    dim3 gk((unsigned)((num_key + kSqT * RK - 1) / (kSqT * RK)), (unsigned)(batch * num_heads));
#define PDVC_SQ_DQ(DD)                                                                                               \
    if (sq_rows_per_lane(DD) == 2)                                                                                   \
        hipLaunchKernelGGL((seqattn_bwd_dq_kernel<DD, 2>), gq, dim3(kSqT), 0, s, q, k, v, grad_out, lse, out, delta, \
                           num_heads, num_query, num_key, ldq, ldk, ldv, scale, grad_q, ld_grad_q);                 \
    else                                                                                                             \
        hipLaunchKernelGGL((seqattn_bwd_dq_kernel<DD, 1>), gq, dim3(kSqT), 0, s, q, k, v, grad_out, lse, out, delta, \
                           num_heads, num_query, num_key, ldq, ldk, ldv, scale, grad_q, ld_grad_q)
#define PDVC_SQ_DKV(DD)                                                                                              \
    if (sq_keys_per_lane(DD) == 2)                                                                                   \
        hipLaunchKernelGGL((seqattn_bwd_dkv_kernel<DD, 2>), gk, dim3(kSqT), 0, s, q, k, v, grad_out, lse, delta,     \
                           num_heads, num_query, num_key, ldq, ldk, ldv, scale, grad_k, ld_grad_k, grad_v,          \
                           ld_grad_v);                                                                              \
    else                                                                                                             \
        hipLaunchKernelGGL((seqattn_bwd_dkv_kernel<DD, 1>), gk, dim3(kSqT), 0, s, q, k, v, grad_out, lse, delta,     \
                           num_heads, num_query, num_key, ldq, ldk, ldv, scale, grad_k, ld_grad_k, grad_v, ld_grad_v)
    PDVC_SQ_DISPATCH(head_dim, PDVC_SQ_DQ)
    PDVC_CHECK_LAUNCH("seqattn_bwd_dq_kernel");
    PDVC_SQ_DISPATCH(head_dim, PDVC_SQ_DKV)
    PDVC_CHECK_LAUNCH("seqattn_bwd_dkv_kernel");
#undef PDVC_SQ_DQ
#undef PDVC_SQ_DKV
    return PDVC_OK;
}
