// capstep.hip -- the per-step pieces of the caption decoder (ShowAttendTellCore) for MI355X (gfx950).
//
// softattn: the soft attention over the L*P = 16 deformable samples of every (row, head)
//   (pdvc/CaptioningHead/LSTM_DSA.py:245-258):
//     dot_j = alpha_net(tanh(att_j + att_h)) = sum_a tanh(att[j,a] + att_h[a]) * w_a + b
//     p = softmax_j(dot);  att_res = sum_j p_j * clip_j
//   with att = ctx2att(clip) (a GEMM, hipBLASLt) and att_h = h2att(h) given.  One 512-thread workgroup per
//   (row, head): threads cover the hidden width for the 16 dots and the value width for the weighted sum.  Replaces an add, tanh, the 1-wide alpha_net GEMM, softmax and a bmm (+ their backward).
// lstm_cell: nn.LSTM's cell for 1 layer, 1 step, no bias (LSTM_DSA.py:206-207,261): gates = sum of up to
//   three pre-activation parts (the GEMM outputs of the hoisted input part, the attention part and W_hh h),
//   gate order (i, f, g, o), c' = f c + i g, h' = o tanh(c').  One lane per (row, unit).
#include <stdlib.h>

#include "pdvc_common.h"

namespace pdvc {

constexpr int sNS = 16;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// One 512-thread workgroup per (row, head); threads run over the hidden (A) and value (D) channels, so every
// global access is a coalesced row segment and no reduction crosses a thread except the 16 dot products
// (wave reduce-scatter + an 8-wave LDS sum).  att (R, M, 16, A) contiguous; att_h (R, ldh) [A values at
// column 0 of the pointer]; clip (R, M, 16, D); any A, D (loops stride 512).
constexpr int kSAT = 512;            // threads per soft-attention workgroup
constexpr int kSAW = kSAT / 64;      // waves

// sum over the workgroup of 16 per-thread partials; result (all 16) in red[0..15]
__device__ __forceinline__ void block_sum16(float (&part)[sNS], float* red, int lane, int wid) {
    group_reduce_scatter<sNS, 16>(part, lane);  // lane%16 -> partial of sample lane%16 over its 16-lane group
    float v = part[0];
    v += lane_swap(v, 16);
    v += __shfl_xor(v, 32, PDVC_WAVE);
    if (lane < sNS) red[wid * sNS + lane] = v;
    __syncthreads();
    if (threadIdx.x < sNS) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kSAW; ++w) t += red[w * sNS + threadIdx.x];
        red[kSAW * sNS + threadIdx.x] = t;
    }
    __syncthreads();
}

__global__ __launch_bounds__(kSAT) void softattn_fwd_kernel(const float* __restrict__ att, const float* __restrict__ att_h,
                                                            int ldh, const float* __restrict__ aw,
                                                            const float* __restrict__ ab, const float* __restrict__ clip,
                                                            int R, int M, int A, int D, float* __restrict__ res,
                                                            float* __restrict__ probs) {
    __shared__ float red[(kSAW + 1) * sNS];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wg = blockIdx.x;  // (row, head)
    const int r = wg / M;
    const float* ab_ = att + (size_t)wg * sNS * A;
    float part[sNS];
#pragma unroll
    for (int j = 0; j < sNS; ++j) part[j] = 0.f;
    for (int a = threadIdx.x; a < A; a += kSAT) {
        const float hv = att_h[(size_t)r * ldh + a], wv = aw[a];
#pragma unroll
        for (int j = 0; j < sNS; ++j) part[j] += tanhf(ab_[(size_t)j * A + a] + hv) * wv;
    }
    block_sum16(part, red, lane, wid);
    const float* dots = red + kSAW * sNS;
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < sNS; ++j) mx = fmaxf(mx, dots[j] + ab[0]);
    float p[sNS], sum = 0.f;
#pragma unroll
    for (int j = 0; j < sNS; ++j) {
        p[j] = expf(dots[j] + ab[0] - mx);
        sum += p[j];
    }
    const float inv = 1.f / sum;
#pragma unroll
    for (int j = 0; j < sNS; ++j) p[j] = p[j] * inv;
    if (threadIdx.x < sNS) {
        float pj = 0.f;
#pragma unroll
        for (int j = 0; j < sNS; ++j) pj = (j == (int)threadIdx.x) ? p[j] : pj;
        probs[(size_t)wg * sNS + threadIdx.x] = pj;
    }
    const float* cb = clip + (size_t)wg * sNS * D;
    for (int d = threadIdx.x; d < D; d += kSAT) {
        float o = 0.f;
#pragma unroll
        for (int j = 0; j < sNS; ++j) o += p[j] * cb[(size_t)j * D + d];
        res[(size_t)wg * D + d] = o;
    }
}

// backward: grad_res (R, M*D) -> grad_att (R,M,16,A), grad_att_h (R,A) (summed over heads), grad_clip
// (R,M,16,D) = p_j * grad_res (the caller adds the ctx2att-path term grad_att @ W_ctx2att with a GEMM),
// per-(row, head) partial sums of the alpha_net weight gradient (R*M, A) and bias gradient (R*M).
__global__ __launch_bounds__(kSAT) void softattn_bwd_kernel(const float* __restrict__ att, const float* __restrict__ att_h,
                                                            int ldh, const float* __restrict__ aw,
                                                            const float* __restrict__ clip,
                                                            const float* __restrict__ probs,
                                                            const float* __restrict__ gres, int R, int M, int A, int D,
                                                            float* __restrict__ gatt, float* __restrict__ gatt_h,
                                                            int ldgh, float* __restrict__ gclip,
                                                            float* __restrict__ gaw_part, float* __restrict__ gab_part) {
    __shared__ float red[(kSAW + 1) * sNS];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wg = blockIdx.x;
    const int r = wg / M;
    float p[sNS];
#pragma unroll
    for (int j = 0; j < sNS; ++j) p[j] = probs[(size_t)wg * sNS + j];
    // dp_j = sum_d g_d clip_j[d];  grad_clip_j = p_j g
    const float* cb = clip + (size_t)wg * sNS * D;
    float* gcb = gclip + (size_t)wg * sNS * D;
    float part[sNS];
#pragma unroll
    for (int j = 0; j < sNS; ++j) part[j] = 0.f;
    for (int d = threadIdx.x; d < D; d += kSAT) {
        const float g = gres[(size_t)wg * D + d];
#pragma unroll
        for (int j = 0; j < sNS; ++j) {
            part[j] += g * cb[(size_t)j * D + d];
            gcb[(size_t)j * D + d] = p[j] * g;
        }
    }
    block_sum16(part, red, lane, wid);
    const float* dp = red + kSAW * sNS;
    // softmax backward: ddot_j = p_j (dp_j - sum_k p_k dp_k)
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < sNS; ++j) t += p[j] * dp[j];
    float dd[sNS], sb = 0.f;
#pragma unroll
    for (int j = 0; j < sNS; ++j) {
        dd[j] = p[j] * (dp[j] - t);
        sb += dd[j];
    }
    if (threadIdx.x == 0) gab_part[wg] = sb;
    const float* ab_ = att + (size_t)wg * sNS * A;
    float* gab_ = gatt + (size_t)wg * sNS * A;
    for (int a = threadIdx.x; a < A; a += kSAT) {
        const float hv = att_h[(size_t)r * ldh + a], wv = aw[a];
        float gh = 0.f, gw = 0.f;
#pragma unroll
        for (int j = 0; j < sNS; ++j) {
            const float th = tanhf(ab_[(size_t)j * A + a] + hv);
            const float dpre = dd[j] * wv * (1.f - th * th);
            gab_[(size_t)j * A + a] = dpre;
            gh += dpre;
            gw += dd[j] * th;
        }
        if (M == 1) gatt_h[(size_t)r * ldgh + a] = gh;
        else atomicAdd(&gatt_h[(size_t)r * ldgh + a], gh);
        gaw_part[(size_t)wg * A + a] = gw;
    }
}

// float4 forms of the two kernels above (A, D, the row strides and the pointers 16-byte aligned -- PDVC's
// A = D = 512): one 128-thread workgroup per (row, head), a lane owns 4 consecutive channels and issues the 16
// samples' float4 loads together.  The 512-thread form gave each lane one float per sample row, 8 waves per
// (row, head) and two workgroup barriers for ~8 KB of reads: latency-bound at ~3x its HBM time.
template <int NW>
__device__ __forceinline__ void block_sum16w(float (&part)[sNS], float* red, int lane, int wid) {
    group_reduce_scatter<sNS, 16>(part, lane);
    float v = part[0];
    v += lane_swap(v, 16);
    v += __shfl_xor(v, 32, PDVC_WAVE);
    if (lane < sNS) red[wid * sNS + lane] = v;
    __syncthreads();
    if (threadIdx.x < sNS) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += red[w * sNS + threadIdx.x];
        red[NW * sNS + threadIdx.x] = t;
    }
    __syncthreads();
}

constexpr int kSA4T = 128;
constexpr int kSA4W = kSA4T / 64;

__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

__global__ __launch_bounds__(kSA4T) void softattn_fwd4_kernel(const float* __restrict__ att,
                                                              const float* __restrict__ att_h, int ldh,
                                                              const float* __restrict__ aw, const float* __restrict__ ab,
                                                              const float* __restrict__ clip, int R, int M, int A,
                                                              int D, float* __restrict__ res,
                                                              float* __restrict__ probs) {
    __shared__ float red[(kSA4W + 1) * sNS];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wg = blockIdx.x;
    const int r = wg / M;
    const int A4 = A / 4, D4 = D / 4;
    const float4* at4 = reinterpret_cast<const float4*>(att + (size_t)wg * sNS * A);
    const float4* h4 = reinterpret_cast<const float4*>(att_h + (size_t)r * ldh);
    const float4* w4 = reinterpret_cast<const float4*>(aw);
    float part[sNS];
#pragma unroll
    for (int j = 0; j < sNS; ++j) part[j] = 0.f;
    for (int a = threadIdx.x; a < A4; a += kSA4T) {
        const float4 hv = h4[a], wv = w4[a];
        float4 x[sNS];
#pragma unroll
        for (int j = 0; j < sNS; ++j) x[j] = at4[(size_t)j * A4 + a];
#pragma unroll
        for (int j = 0; j < sNS; ++j)
            part[j] += tanhf(x[j].x + hv.x) * wv.x + tanhf(x[j].y + hv.y) * wv.y + tanhf(x[j].z + hv.z) * wv.z +
                       tanhf(x[j].w + hv.w) * wv.w;
    }
    block_sum16w<kSA4W>(part, red, lane, wid);
    const float* dots = red + kSA4W * sNS;
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < sNS; ++j) mx = fmaxf(mx, dots[j] + ab[0]);
    float p[sNS], sum = 0.f;
#pragma unroll
    for (int j = 0; j < sNS; ++j) {
        p[j] = expf(dots[j] + ab[0] - mx);
        sum += p[j];
    }
    const float inv = 1.f / sum;
#pragma unroll
    for (int j = 0; j < sNS; ++j) p[j] = p[j] * inv;
    if (threadIdx.x < sNS) {
        float pj = 0.f;
#pragma unroll
        for (int j = 0; j < sNS; ++j) pj = (j == (int)threadIdx.x) ? p[j] : pj;
        probs[(size_t)wg * sNS + threadIdx.x] = pj;
    }
    const float4* c4 = reinterpret_cast<const float4*>(clip + (size_t)wg * sNS * D);
    float4* r4 = reinterpret_cast<float4*>(res + (size_t)wg * D);
    for (int d = threadIdx.x; d < D4; d += kSA4T) {
        float4 x[sNS];
#pragma unroll
        for (int j = 0; j < sNS; ++j) x[j] = c4[(size_t)j * D4 + d];
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < sNS; ++j) {
            o.x += p[j] * x[j].x;
            o.y += p[j] * x[j].y;
            o.z += p[j] * x[j].z;
            o.w += p[j] * x[j].w;
        }
        r4[d] = o;
    }
}

__global__ __launch_bounds__(kSA4T) void softattn_bwd4_kernel(const float* __restrict__ att,
                                                              const float* __restrict__ att_h, int ldh,
                                                              const float* __restrict__ aw,
                                                              const float* __restrict__ clip,
                                                              const float* __restrict__ probs,
                                                              const float* __restrict__ gres, int R, int M, int A,
                                                              int D, float* __restrict__ gatt,
                                                              float* __restrict__ gatt_h, int ldgh,
                                                              float* __restrict__ gclip, float* __restrict__ gaw_part,
                                                              float* __restrict__ gab_part) {
    __shared__ float red[(kSA4W + 1) * sNS];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wg = blockIdx.x;
    const int r = wg / M;
    const int A4 = A / 4, D4 = D / 4;
    float p[sNS];
#pragma unroll
    for (int j = 0; j < sNS; ++j) p[j] = probs[(size_t)wg * sNS + j];
    const float4* c4 = reinterpret_cast<const float4*>(clip + (size_t)wg * sNS * D);
    float4* gc4 = reinterpret_cast<float4*>(gclip + (size_t)wg * sNS * D);
    const float4* g4 = reinterpret_cast<const float4*>(gres + (size_t)wg * D);
    float part[sNS];
#pragma unroll
    for (int j = 0; j < sNS; ++j) part[j] = 0.f;
    for (int d = threadIdx.x; d < D4; d += kSA4T) {
        const float4 g = g4[d];
        float4 x[sNS];
#pragma unroll
        for (int j = 0; j < sNS; ++j) x[j] = c4[(size_t)j * D4 + d];
#pragma unroll
        for (int j = 0; j < sNS; ++j) {
            part[j] += dot4(g, x[j]);
            gc4[(size_t)j * D4 + d] = make_float4(p[j] * g.x, p[j] * g.y, p[j] * g.z, p[j] * g.w);
        }
    }
    block_sum16w<kSA4W>(part, red, lane, wid);
    const float* dp = red + kSA4W * sNS;
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < sNS; ++j) t += p[j] * dp[j];
    float dd[sNS], sb = 0.f;
#pragma unroll
    for (int j = 0; j < sNS; ++j) {
        dd[j] = p[j] * (dp[j] - t);
        sb += dd[j];
    }
    if (threadIdx.x == 0) gab_part[wg] = sb;
    const float4* at4 = reinterpret_cast<const float4*>(att + (size_t)wg * sNS * A);
    float4* ga4 = reinterpret_cast<float4*>(gatt + (size_t)wg * sNS * A);
    const float4* h4 = reinterpret_cast<const float4*>(att_h + (size_t)r * ldh);
    const float4* w4 = reinterpret_cast<const float4*>(aw);
    float4* gh4 = reinterpret_cast<float4*>(gatt_h + (size_t)r * ldgh);
    float4* gw4 = reinterpret_cast<float4*>(gaw_part + (size_t)wg * A);
    for (int a = threadIdx.x; a < A4; a += kSA4T) {
        const float4 hv = h4[a], wv = w4[a];
        float4 x[sNS];
#pragma unroll
        for (int j = 0; j < sNS; ++j) x[j] = at4[(size_t)j * A4 + a];
        float4 gh = make_float4(0.f, 0.f, 0.f, 0.f), gw = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < sNS; ++j) {
            const float tx = tanhf(x[j].x + hv.x), ty = tanhf(x[j].y + hv.y), tz = tanhf(x[j].z + hv.z),
                        tw = tanhf(x[j].w + hv.w);
            const float4 dpre = make_float4(dd[j] * wv.x * (1.f - tx * tx), dd[j] * wv.y * (1.f - ty * ty),
                                            dd[j] * wv.z * (1.f - tz * tz), dd[j] * wv.w * (1.f - tw * tw));
            ga4[(size_t)j * A4 + a] = dpre;
            gh.x += dpre.x; gh.y += dpre.y; gh.z += dpre.z; gh.w += dpre.w;
            gw.x += dd[j] * tx; gw.y += dd[j] * ty; gw.z += dd[j] * tz; gw.w += dd[j] * tw;
        }
        if (M == 1) {
            gh4[a] = gh;
        } else {
            float* gp = gatt_h + (size_t)r * ldgh + 4 * a;
            atomicAdd(gp, gh.x); atomicAdd(gp + 1, gh.y); atomicAdd(gp + 2, gh.z); atomicAdd(gp + 3, gh.w);
        }
        gw4[a] = gw;
    }
}

// PDVC_SOFTATTN_SCALAR=1 keeps the 512-thread kernels (same-box A/B)
static bool sa_vec4(const void* const* ptrs, int n, int A, int D, int ld1, int ld2) {
    static const bool scalar = [] {
        const char* e = getenv("PDVC_SOFTATTN_SCALAR");
        return e && e[0] == '1';
    }();
    if (scalar || A % 4 || D % 4 || ld1 % 4 || ld2 % 4) return false;
    for (int i = 0; i < n; ++i)
        if (((uintptr_t)ptrs[i]) % 16) return false;
    return true;
}

// gates = a + b + c + d (each (R,4H) with its own row stride; b, c or d may be NULL); acts <- (i,f,g,o) activations
// GATHER: gates_a's row of output row r is a_rows[r] (the greedy decode's word-gate table rows, no gathered copy);
// acts may be NULL (no backward follows: greedy decoding)
template <bool GATHER>
__global__ __launch_bounds__(256) void lstm_fwd_kernel(const float* __restrict__ ga, int lda, const float* __restrict__ gb,
                                                       int ldb, const float* __restrict__ gc, int ldc,
                                                       const float* __restrict__ gd, int ldd,
                                                       const float* __restrict__ c_prev, int R, int H,
                                                       float* __restrict__ h_out, int ldho, float* __restrict__ c_out,
                                                       float* __restrict__ acts, const int64_t* __restrict__ a_rows) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)R * H) return;
    const int r = (int)(idx / H), u = (int)(idx - (long)r * H);
    const size_t ra = GATHER ? (size_t)a_rows[r] : (size_t)r;
    float z[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int col = q * H + u;
        float v = ga[ra * lda + col];
        if (gb) v += gb[(size_t)r * ldb + col];
        if (gc) v += gc[(size_t)r * ldc + col];
        if (gd) v += gd[(size_t)r * ldd + col];
        z[q] = v;
    }
    const float i = sigm(z[0]), f = sigm(z[1]), g = tanhf(z[2]), o = sigm(z[3]);
    const float c = f * c_prev[idx] + i * g;
    const float h = o * tanhf(c);
    c_out[idx] = c;
    h_out[(size_t)r * ldho + u] = h;
    if (acts) {
        float* a = acts + (size_t)r * 4 * H;
        a[u] = i;
        a[H + u] = f;
        a[2 * H + u] = g;
        a[3 * H + u] = o;
    }
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

extern "C" int pdvc_softattn_forward_f32(const float* att, const float* att_h, int ld_att_h, const float* alpha_w,
                                         const float* alpha_b, const float* clip, int rows, int num_heads,
                                         int att_hid, int head_dim, float* att_res, float* probs, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && num_heads > 0, "invalid sizes");
    const long waves = (long)rows * num_heads;
    if (waves == 0) return PDVC_OK;
    PDVC_CHECK_ARG(att_hid > 0 && head_dim > 0 && waves < (1L << 31), "invalid sizes");
    hipStream_t s = (hipStream_t)stream;
    const void* fp[] = {att, att_h, alpha_w, clip, att_res};
    if (sa_vec4(fp, 5, att_hid, head_dim, ld_att_h, 0))
        hipLaunchKernelGGL(softattn_fwd4_kernel, dim3((unsigned)waves), dim3(kSA4T), 0, s, att, att_h, ld_att_h,
                           alpha_w, alpha_b, clip, rows, num_heads, att_hid, head_dim, att_res, probs);
    else
        hipLaunchKernelGGL(softattn_fwd_kernel, dim3((unsigned)waves), dim3(kSAT), 0, s, att, att_h, ld_att_h, alpha_w,
                           alpha_b, clip, rows, num_heads, att_hid, head_dim, att_res, probs);
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
    PDVC_CHECK_ARG(att_hid > 0 && head_dim > 0 && waves < (1L << 31), "invalid sizes");
    const void* bp[] = {att, att_h, alpha_w, clip, grad_res, grad_att, grad_att_h, grad_clip, grad_alpha_w_part};
    if (sa_vec4(bp, 9, att_hid, head_dim, ld_att_h, ld_grad_att_h))
        hipLaunchKernelGGL(softattn_bwd4_kernel, dim3((unsigned)waves), dim3(kSA4T), 0, s, att, att_h, ld_att_h,
                           alpha_w, clip, probs, grad_res, rows, num_heads, att_hid, head_dim, grad_att, grad_att_h,
                           ld_grad_att_h, grad_clip, grad_alpha_w_part, grad_alpha_b_part);
    else
        hipLaunchKernelGGL(softattn_bwd_kernel, dim3((unsigned)waves), dim3(kSAT), 0, s, att, att_h, ld_att_h, alpha_w,
                           clip, probs, grad_res, rows, num_heads, att_hid, head_dim, grad_att, grad_att_h,
                           ld_grad_att_h, grad_clip, grad_alpha_w_part, grad_alpha_b_part);
    PDVC_CHECK_LAUNCH("softattn_bwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_lstm_cell_forward_f32(const float* gates_a, int lda, const float* gates_b, int ldb,
                                          const float* gates_c, int ldc, const float* gates_d, int ldd,
                                          const float* c_prev, int rows, int hidden,
                                          float* h_out, int ld_h_out, float* c_out, float* acts, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && hidden > 0 && lda >= 4 * hidden, "invalid sizes");
    const long n = (long)rows * hidden;
    if (n == 0) return PDVC_OK;
    PDVC_CHECK_ARG(acts != nullptr, "acts (rows, 4 hidden) is required");
    hipLaunchKernelGGL(lstm_fwd_kernel<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       gates_a, lda, gates_b, ldb, gates_c, ldc, gates_d, ldd, c_prev, rows, hidden, h_out, ld_h_out,
                       c_out, acts, (const int64_t*)nullptr);
    PDVC_CHECK_LAUNCH("lstm_fwd_kernel");
    return PDVC_OK;
}

// The same with gates_a read through a row index (gates_a[a_rows[r]], e.g. a vocabulary table's rows) and acts
// optional (NULL: not written -- greedy decoding, no backward)
extern "C" int pdvc_lstm_cell_forward_gather_f32(const float* gates_a, int lda, const int64_t* a_rows,
                                                 const float* gates_b, int ldb, const float* gates_c, int ldc,
                                                 const float* gates_d, int ldd, const float* c_prev, int rows,
                                                 int hidden, float* h_out, int ld_h_out, float* c_out, float* acts,
                                                 void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && hidden > 0 && lda >= 4 * hidden, "invalid sizes");
    PDVC_CHECK_ARG(rows == 0 || (gates_a && a_rows && c_prev && h_out && c_out), "null pointer");
    const long n = (long)rows * hidden;
    if (n == 0) return PDVC_OK;
    hipLaunchKernelGGL(lstm_fwd_kernel<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       gates_a, lda, gates_b, ldb, gates_c, ldc, gates_d, ldd, c_prev, rows, hidden, h_out, ld_h_out,
                       c_out, acts, a_rows);
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
