// capstep.hip -- the per-step pieces of the caption decoder (ShowAttendTellCore) for MI355X (gfx950).
//
// softattn: the soft attention over the L*P = 16 deformable samples of every (row, head)
//   (pdvc/CaptioningHead/LSTM_DSA.py:245-258):
//     dot_j = alpha_net(tanh(att_j + att_h)) = sum_a tanh(att[j,a] + att_h[a]) * w_a + b
//     p = softmax_j(dot);  att_res = sum_j p_j * clip_j
//   with att = ctx2att(clip) (a GEMM, hipBLASLt) and att_h = h2att(h) given.  One wave per (row, head):
//   lanes cover the hidden width for the 16 dots (reduce-scatter over lanes) and the value width for the
//   weighted sum.  Replaces an add, tanh, the 1-wide alpha_net GEMM, softmax and a bmm (+ their backward).
// lstm_cell: nn.LSTM's cell for 1 layer, 1 step, no bias (LSTM_DSA.py:206-207,261): gates = sum of up to
//   three pre-activation parts (the GEMM outputs of the hoisted input part, the attention part and W_hh h),
//   gate order (i, f, g, o), c' = f c + i g, h' = o tanh(c').  One lane per (row, unit).
#include "pdvc_common.h"

namespace pdvc {

constexpr int sNS = 16;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// att (R, M, 16, A) contiguous; att_h (R, ldh) [A values at column 0 of the pointer]; clip (R, M, 16, D).
// APL / DPL are the per-lane maxima (A <= 64*APL, D <= 64*DPL); columns past A / D are masked.
template <int APL, int DPL>
__global__ __launch_bounds__(256) void softattn_fwd_kernel(const float* __restrict__ att, const float* __restrict__ att_h,
                                                           int ldh, const float* __restrict__ aw,
                                                           const float* __restrict__ ab, const float* __restrict__ clip,
                                                           int R, int M, int A, int D, float* __restrict__ res,
                                                           float* __restrict__ probs) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wave >= R * M) return;
    const int r = wave / M;
    float hv[APL], wv[APL];
#pragma unroll
    for (int k = 0; k < APL; ++k) {
        const int a = lane + 64 * k;
        hv[k] = a < A ? att_h[(size_t)r * ldh + a] : 0.f;
        wv[k] = a < A ? aw[a] : 0.f;
    }
    const float* ab_ = att + (size_t)wave * sNS * A;
    float part[sNS];
#pragma unroll
    for (int j = 0; j < sNS; ++j) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < APL; ++k) {
            const int a = lane + 64 * k;
            if (a < A) s += tanhf(ab_[j * A + a] + hv[k]) * wv[k];
        }
        part[j] = s;
    }
    group_reduce_scatter<sNS, 16>(part, lane);   // lane%16 -> dot of sample lane%16 (partial over 16-lane group)
    float dot = part[0];
    dot += __shfl_xor(dot, 16, PDVC_WAVE);
    dot += __shfl_xor(dot, 32, PDVC_WAVE);
    dot += ab[0];
    // softmax over the 16 samples (each value replicated on 4 lanes)
    float mx = dot;
#pragma unroll
    for (int d = 8; d > 0; d >>= 1) mx = fmaxf(mx, __shfl_xor(mx, d, PDVC_WAVE));
    const float e = expf(dot - mx);
    float sum = e;
#pragma unroll
    for (int d = 8; d > 0; d >>= 1) sum += __shfl_xor(sum, d, PDVC_WAVE);
    const float p = e / sum;
    if (lane < sNS) probs[(size_t)wave * sNS + lane] = p;
    float o[DPL];
#pragma unroll
    for (int k = 0; k < DPL; ++k) o[k] = 0.f;
    const float* cb = clip + (size_t)wave * sNS * D;
#pragma unroll
    for (int j = 0; j < sNS; ++j) {
        const float pj = __shfl(p, j, PDVC_WAVE);
#pragma unroll
        for (int k = 0; k < DPL; ++k) {
            const int d = lane + 64 * k;
            if (d < D) o[k] += pj * cb[j * D + d];
        }
    }
#pragma unroll
    for (int k = 0; k < DPL; ++k) {
        const int d = lane + 64 * k;
        if (d < D) res[(size_t)wave * D + d] = o[k];
    }
}

// backward: grad_res (R, M*D) -> grad_att (R,M,16,A), grad_att_h (R,A) (summed over heads), grad_clip
// (R,M,16,D) = p_j * grad_res (the caller adds the ctx2att-path term grad_att @ W_ctx2att with a GEMM),
// per-wave partial sums of the alpha_net weight gradient (R*M, A) and bias gradient (R*M).
template <int APL, int DPL>
__global__ __launch_bounds__(256) void softattn_bwd_kernel(const float* __restrict__ att, const float* __restrict__ att_h,
                                                           int ldh, const float* __restrict__ aw,
                                                           const float* __restrict__ clip,
                                                           const float* __restrict__ probs,
                                                           const float* __restrict__ gres, int R, int M, int A, int D,
                                                           float* __restrict__ gatt, float* __restrict__ gatt_h,
                                                           int ldgh, float* __restrict__ gclip,
                                                           float* __restrict__ gaw_part, float* __restrict__ gab_part) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wave >= R * M) return;
    const int r = wave / M;
    const float* cb = clip + (size_t)wave * sNS * D;
    float* gcb = gclip + (size_t)wave * sNS * D;
    float g[DPL];
#pragma unroll
    for (int k = 0; k < DPL; ++k) {
        const int d = lane + 64 * k;
        g[k] = d < D ? gres[(size_t)wave * D + d] : 0.f;
    }
    const float p = (lane < sNS) ? probs[(size_t)wave * sNS + lane] : 0.f;
    // d p_j = sum_d g_d clip_j[d]; grad_clip_j = p_j g
    float part[sNS];
#pragma unroll
    for (int j = 0; j < sNS; ++j) {
        const float pj = __shfl(p, j, PDVC_WAVE);
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < DPL; ++k) {
            const int d = lane + 64 * k;
            if (d < D) {
                const size_t idx = (size_t)j * D + d;
                s += g[k] * cb[idx];
                gcb[idx] = pj * g[k];
            }
        }
        part[j] = s;
    }
    group_reduce_scatter<sNS, 16>(part, lane);
    float dp = part[0];
    dp += __shfl_xor(dp, 16, PDVC_WAVE);
    dp += __shfl_xor(dp, 32, PDVC_WAVE);
    // softmax backward: ddot_j = p_j (dp_j - sum_k p_k dp_k); lanes j (mod 16) hold sample j
    const float pj_l = __shfl(p, lane & 15, PDVC_WAVE);
    float t = pj_l * dp;
#pragma unroll
    for (int d = 8; d > 0; d >>= 1) t += __shfl_xor(t, d, PDVC_WAVE);
    const float ddot = pj_l * (dp - t);
    float sb = ddot;
#pragma unroll
    for (int d = 8; d > 0; d >>= 1) sb += __shfl_xor(sb, d, PDVC_WAVE);
    if (lane == 0) gab_part[wave] = sb;
    float hv[APL], wv[APL], gh[APL], gw[APL];
#pragma unroll
    for (int k = 0; k < APL; ++k) {
        const int a = lane + 64 * k;
        hv[k] = a < A ? att_h[(size_t)r * ldh + a] : 0.f;
        wv[k] = a < A ? aw[a] : 0.f;
        gh[k] = 0.f;
        gw[k] = 0.f;
    }
    const float* ab_ = att + (size_t)wave * sNS * A;
    float* gab_ = gatt + (size_t)wave * sNS * A;
#pragma unroll
    for (int j = 0; j < sNS; ++j) {
        const float dj = __shfl(ddot, j, PDVC_WAVE);
#pragma unroll
        for (int k = 0; k < APL; ++k) {
            const int a = lane + 64 * k;
            if (a < A) {
                const float th = tanhf(ab_[j * A + a] + hv[k]);
                const float dpre = dj * wv[k] * (1.f - th * th);
                gab_[j * A + a] = dpre;
                gh[k] += dpre;
                gw[k] += dj * th;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < APL; ++k) {
        const int a = lane + 64 * k;
        if (a < A) {
            if (M == 1) gatt_h[(size_t)r * ldgh + a] = gh[k];
            else atomicAdd(&gatt_h[(size_t)r * ldgh + a], gh[k]);
            gaw_part[(size_t)wave * A + a] = gw[k];
        }
    }
}

// gates = a + b + c (each (R,4H) with its own row stride; b or c may be NULL); acts <- (i,f,g,o) activations
__global__ __launch_bounds__(256) void lstm_fwd_kernel(const float* __restrict__ ga, int lda, const float* __restrict__ gb,
                                                       int ldb, const float* __restrict__ gc, int ldc,
                                                       const float* __restrict__ c_prev, int R, int H,
                                                       float* __restrict__ h_out, int ldho, float* __restrict__ c_out,
                                                       float* __restrict__ acts) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)R * H) return;
    const int r = (int)(idx / H), u = (int)(idx - (long)r * H);
    float z[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int col = q * H + u;
        float v = ga[(size_t)r * lda + col];
        if (gb) v += gb[(size_t)r * ldb + col];
        if (gc) v += gc[(size_t)r * ldc + col];
        z[q] = v;
    }
    const float i = sigm(z[0]), f = sigm(z[1]), g = tanhf(z[2]), o = sigm(z[3]);
    const float c = f * c_prev[idx] + i * g;
    const float h = o * tanhf(c);
    c_out[idx] = c;
    h_out[(size_t)r * ldho + u] = h;
    float* a = acts + (size_t)r * 4 * H;
    a[u] = i;
    a[H + u] = f;
    a[2 * H + u] = g;
    a[3 * H + u] = o;
}

// dh (R,H) [+ dh2 (R, ld2) if given], dc_next (R,H) or NULL, acts, c_prev, c -> dgates (R,4H), dc_prev (R,H)
__global__ __launch_bounds__(256) void lstm_bwd_kernel(const float* __restrict__ dh, int lddh, const float* __restrict__ dh2,
                                                       int lddh2, const float* __restrict__ dc_next,
                                                       const float* __restrict__ acts, const float* __restrict__ c_prev,
                                                       const float* __restrict__ c, int R, int H,
                                                       float* __restrict__ dgates, int ldg, float* __restrict__ dc_prev) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)R * H) return;
    const int r = (int)(idx / H), u = (int)(idx - (long)r * H);
    const float* a = acts + (size_t)r * 4 * H;
    const float i = a[u], f = a[H + u], g = a[2 * H + u], o = a[3 * H + u];
    float gh = dh[(size_t)r * lddh + u];
    if (dh2) gh += dh2[(size_t)r * lddh2 + u];
    const float tc = tanhf(c[idx]);
    float dc = gh * o * (1.f - tc * tc);
    if (dc_next) dc += dc_next[idx];
    const float dO = gh * tc, dI = dc * g, dG = dc * i, dF = dc * c_prev[idx];
    float* d = dgates + (size_t)r * ldg;
    d[u] = dI * i * (1.f - i);
    d[H + u] = dF * f * (1.f - f);
    d[2 * H + u] = dG * (1.f - g * g);
    d[3 * H + u] = dO * o * (1.f - o);
    dc_prev[idx] = dc * f;
}

}  // namespace pdvc

using namespace pdvc;

static int pow2_lanes(int n) {  // per-lane maximum for n columns over 64 lanes: 1, 2, 4 or 8 (0 if n > 512)
    const int k = (n + 63) / 64;
    return k <= 1 ? 1 : k <= 2 ? 2 : k <= 4 ? 4 : k <= 8 ? 8 : 0;
}

#define SA_CASE(KERNEL, PA, PD, ...) \
    else if (pa == PA && pd == PD) hipLaunchKernelGGL((KERNEL<PA, PD>), __VA_ARGS__)
#define SA_DISPATCH(KERNEL, A, D, ...)                                                                       \
    do {                                                                                                     \
        const int pa = pow2_lanes(A), pd = pow2_lanes(D);                                                    \
        if (A <= 0 || D <= 0 || pa == 0 || pd == 0)                                                          \
            return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "soft attention: need 0 < A, D <= 512 (A=%d, D=%d)", A, D); \
        SA_CASE(KERNEL, 1, 1, __VA_ARGS__); SA_CASE(KERNEL, 1, 2, __VA_ARGS__); SA_CASE(KERNEL, 1, 4, __VA_ARGS__); \
        SA_CASE(KERNEL, 1, 8, __VA_ARGS__); SA_CASE(KERNEL, 2, 1, __VA_ARGS__); SA_CASE(KERNEL, 2, 2, __VA_ARGS__); \
        SA_CASE(KERNEL, 2, 4, __VA_ARGS__); SA_CASE(KERNEL, 2, 8, __VA_ARGS__); SA_CASE(KERNEL, 4, 1, __VA_ARGS__); \
        SA_CASE(KERNEL, 4, 2, __VA_ARGS__); SA_CASE(KERNEL, 4, 4, __VA_ARGS__); SA_CASE(KERNEL, 4, 8, __VA_ARGS__); \
        SA_CASE(KERNEL, 8, 1, __VA_ARGS__); SA_CASE(KERNEL, 8, 2, __VA_ARGS__); SA_CASE(KERNEL, 8, 4, __VA_ARGS__); \
        SA_CASE(KERNEL, 8, 8, __VA_ARGS__);                                                                  \
    } while (0)

extern "C" int pdvc_softattn_forward_f32(const float* att, const float* att_h, int ld_att_h, const float* alpha_w,
                                         const float* alpha_b, const float* clip, int rows, int num_heads,
                                         int att_hid, int head_dim, float* att_res, float* probs, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && num_heads > 0, "invalid sizes");
    const long waves = (long)rows * num_heads;
    if (waves == 0) return PDVC_OK;
    dim3 grid((unsigned)((waves + 3) / 4)), block(256);
    hipStream_t s = (hipStream_t)stream;
    SA_DISPATCH(softattn_fwd_kernel, att_hid, head_dim, grid, block, 0, s, att, att_h, ld_att_h, alpha_w, alpha_b,
                clip, rows, num_heads, att_hid, head_dim, att_res, probs);
    PDVC_CHECK_LAUNCH("softattn_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_softattn_backward_f32(const float* att, const float* att_h, int ld_att_h, const float* alpha_w,
                                          const float* clip, const float* probs, const float* grad_res, int rows,
                                          int num_heads, int att_hid, int head_dim, float* grad_att,
                                          float* grad_att_h, int ld_grad_att_h, float* grad_clip,
                                          float* grad_alpha_w_part, float* grad_alpha_b_part, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && num_heads > 0, "invalid sizes");
    const long waves = (long)rows * num_heads;
    if (waves == 0) return PDVC_OK;
    hipStream_t s = (hipStream_t)stream;
    if (num_heads > 1) {
        // grad_att_h is accumulated over heads with atomics: zero it first (rows x att_hid, strided)
        hipError_t e = hipMemset2DAsync(grad_att_h, sizeof(float) * ld_grad_att_h, 0, sizeof(float) * att_hid, rows, s);
        if (e != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "memset grad_att_h: %s", hipGetErrorString(e));
    }
    dim3 grid((unsigned)((waves + 3) / 4)), block(256);
    SA_DISPATCH(softattn_bwd_kernel, att_hid, head_dim, grid, block, 0, s, att, att_h, ld_att_h, alpha_w, clip, probs,
                grad_res, rows, num_heads, att_hid, head_dim, grad_att, grad_att_h, ld_grad_att_h, grad_clip, grad_alpha_w_part,
                grad_alpha_b_part);
    PDVC_CHECK_LAUNCH("softattn_bwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_lstm_cell_forward_f32(const float* gates_a, int lda, const float* gates_b, int ldb,
                                          const float* gates_c, int ldc, const float* c_prev, int rows, int hidden,
                                          float* h_out, int ld_h_out, float* c_out, float* acts, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && hidden > 0 && lda >= 4 * hidden, "invalid sizes");
    const long n = (long)rows * hidden;
    if (n == 0) return PDVC_OK;
    hipLaunchKernelGGL(lstm_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, gates_a,
                       lda, gates_b, ldb, gates_c, ldc, c_prev, rows, hidden, h_out, ld_h_out, c_out, acts);
    PDVC_CHECK_LAUNCH("lstm_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_lstm_cell_backward_f32(const float* grad_h, int ld_grad_h, const float* grad_h2, int ld_grad_h2,
                                           const float* grad_c_next, const float* acts, const float* c_prev,
                                           const float* c, int rows, int hidden, float* grad_gates,
                                           int ld_grad_gates, float* grad_c_prev, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && hidden > 0 && ld_grad_gates >= 4 * hidden, "invalid sizes");
    const long n = (long)rows * hidden;
    if (n == 0) return PDVC_OK;
    hipLaunchKernelGGL(lstm_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, grad_h,
                       ld_grad_h, grad_h2, ld_grad_h2, grad_c_next, acts, c_prev, c, rows, hidden, grad_gates,
                       ld_grad_gates, grad_c_prev);
    PDVC_CHECK_LAUNCH("lstm_bwd_kernel");
    return PDVC_OK;
}
