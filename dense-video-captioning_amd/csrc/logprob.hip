// logprob.hip -- the caption head's word log-probabilities and the log-probability of the target word, both ways
// (reference: Captioner.get_logprobs_state, LSTM_DSA.py:112-116: logprobs = log_softmax(logit(dropout(h))), and
// LanguageModelCriterion / build_loss, LSTM_DSA.py:48-52: -sum_t logp[t, target_t] * mask_t / sum mask).
//
// Forward: one workgroup per (caption row, step) -- a row of V logits (V = 5748 on ActivityNet, 1609 on YouCook2).
// For V <= 8192 (V % 4 == 0) the row is held in registers: max, then sum exp(x - max), then
// logp = (x - max) - log(sum) -- torch's log_softmax arithmetic -- and the row's target entry picked = logp[target].
// Longer or unaligned rows take a streaming form: a per-lane running (max, sum of exp) pair, merged over the
// workgroup, and a second pass over the row (in L2 by then).  torch needed log_softmax, a gather, and in
// the backward a zero-fill of a (rows, V) tensor, a scatter and log_softmax_backward: ~5 full passes.
// Backward: the loss reaches the logits only through `picked`, so
//     dlogits[j] = g * ([j == target] - exp(logp[j]))
// one read of logp and one write of dlogits per element, no (rows, V) one-hot or zero fill.
// HBM-bound: forward 8 bytes per element (x read once into registers for V <= 8192, logp written), backward 8.
#include <math.h>

#include "pdvc_common.h"

namespace pdvc {

constexpr int kLpThreads = 256;

// merge two (max, sum of exp(x - max)) pairs
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
    if (m2 > m) {
        s = s * expf(m - m2) + s2;
        m = m2;
    } else if (m2 > -INFINITY) {
        s += s2 * expf(m2 - m);
    }
}

__device__ __forceinline__ void lse_add(float& m, float& s, float x) {
    if (x > m) {
        s = s * expf(m - x) + 1.f;
        m = x;
    } else {
        s += expf(x - m);
    }
}

template <bool VEC4>
__global__ __launch_bounds__(kLpThreads) void logprob_pick_fwd_kernel(const float* __restrict__ x,
                                                                     const int64_t* __restrict__ target, int V,
                                                                     float* __restrict__ logp,
                                                                     float* __restrict__ picked) {
    __shared__ float red_m[kLpThreads / PDVC_WAVE], red_s[kLpThreads / PDVC_WAVE];
    const long row = blockIdx.x;
    const float* xr = x + row * (long)V;
    float* lr = logp + row * (long)V;
    float m = -INFINITY, s = 0.f;
    if (VEC4) {
        const int v4 = V / 4;
        const float4* x4 = reinterpret_cast<const float4*>(xr);
        for (int i = threadIdx.x; i < v4; i += kLpThreads) {
            const float4 a = x4[i];
            lse_add(m, s, a.x); lse_add(m, s, a.y); lse_add(m, s, a.z); lse_add(m, s, a.w);
        }
    } else {
        for (int i = threadIdx.x; i < V; i += kLpThreads) lse_add(m, s, xr[i]);
    }
#pragma unroll
    for (int d = 1; d < PDVC_WAVE; d <<= 1) {
        const float m2 = lane_swap(m, d), s2 = lane_swap(s, d);
        lse_merge(m, s, m2, s2);
    }
    const int wave = threadIdx.x / PDVC_WAVE, lane = threadIdx.x % PDVC_WAVE;
    if (lane == 0) {
        red_m[wave] = m;
        red_s[wave] = s;
    }
    __syncthreads();
    m = red_m[0];
    s = red_s[0];
#pragma unroll
    for (int w = 1; w < kLpThreads / PDVC_WAVE; ++w) lse_merge(m, s, red_m[w], red_s[w]);
    const float ls = logf(s);
    if (VEC4) {
        const int v4 = V / 4;
        const float4* x4 = reinterpret_cast<const float4*>(xr);
        float4* l4 = reinterpret_cast<float4*>(lr);
        for (int i = threadIdx.x; i < v4; i += kLpThreads) {
            const float4 a = x4[i];
            l4[i] = make_float4((a.x - m) - ls, (a.y - m) - ls, (a.z - m) - ls, (a.w - m) - ls);
        }
    } else {
        for (int i = threadIdx.x; i < V; i += kLpThreads) lr[i] = (xr[i] - m) - ls;
    }
    if (threadIdx.x == 0) {
        const int64_t t = target[row];
        // an out-of-range target poisons the loss (torch's gather would raise a device-side assert)
        picked[row] = (t >= 0 && t < V) ? (xr[t] - m) - ls : NAN;
    }
}

template <bool VEC4>
__global__ __launch_bounds__(kLpThreads) void logprob_pick_bwd_kernel(const float* __restrict__ logp,
                                                                     const int64_t* __restrict__ target,
                                                                     const float* __restrict__ gpick, int V,
                                                                     float* __restrict__ dx, int ldo) {
    const long row = blockIdx.x;
    const float g = gpick[row];
    const int64_t t = target[row];
    const float* lr = logp + row * (long)V;
    float* dr = dx + row * (long)ldo;
    for (int j = V + threadIdx.x; j < ldo; j += kLpThreads) dr[j] = 0.f;  // a padded row's tail: zeros
    if (VEC4) {
        const int v4 = V / 4;
        const float4* l4 = reinterpret_cast<const float4*>(lr);
        float4* d4 = reinterpret_cast<float4*>(dr);
        for (int i = threadIdx.x; i < v4; i += kLpThreads) {
            const float4 a = l4[i];
            const int j = 4 * i;
            d4[i] = make_float4(g * ((j == t ? 1.f : 0.f) - expf(a.x)), g * ((j + 1 == t ? 1.f : 0.f) - expf(a.y)),
                                g * ((j + 2 == t ? 1.f : 0.f) - expf(a.z)),
                                g * ((j + 3 == t ? 1.f : 0.f) - expf(a.w)));
        }
    } else {
        for (int j = threadIdx.x; j < V; j += kLpThreads) dr[j] = g * ((j == t ? 1.f : 0.f) - expf(lr[j]));
    }
}

// Register-resident forms for V <= 4 * kLpThreads * KR (KR float4 per lane: 8192 logits at KR = 8): every load
// of the row is issued before any arithmetic, the max and then sum exp(x - max) are taken from registers (the
// order torch's log_softmax uses: no running rescale), and logp is written from the same registers -- the row
// is read once.  The streaming kernels above serialised one float4 load and four expf per loop trip.
constexpr int kLpKR = 8;

__device__ __forceinline__ float block_max(float v, float* red) {
#pragma unroll
    for (int d = 1; d < PDVC_WAVE; d <<= 1) v = fmaxf(v, lane_swap(v, d));
    const int wave = threadIdx.x / PDVC_WAVE;
    __syncthreads();
    if ((threadIdx.x % PDVC_WAVE) == 0) red[wave] = v;
    __syncthreads();
    v = red[0];
#pragma unroll
    for (int w = 1; w < kLpThreads / PDVC_WAVE; ++w) v = fmaxf(v, red[w]);
    return v;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
    for (int d = 1; d < PDVC_WAVE; d <<= 1) v += lane_swap(v, d);
    const int wave = threadIdx.x / PDVC_WAVE;
    __syncthreads();
    if ((threadIdx.x % PDVC_WAVE) == 0) red[wave] = v;
    __syncthreads();
    v = red[0];
#pragma unroll
    for (int w = 1; w < kLpThreads / PDVC_WAVE; ++w) v += red[w];
    return v;
}

__global__ __launch_bounds__(kLpThreads) void logprob_pick_fwd_reg_kernel(const float* __restrict__ x,
                                                                         const int64_t* __restrict__ target, int V,
                                                                         float* __restrict__ logp,
                                                                         float* __restrict__ picked) {
    __shared__ float red[kLpThreads / PDVC_WAVE];
    const long row = blockIdx.x;
    const int v4 = V / 4;
    const float4* x4 = reinterpret_cast<const float4*>(x + row * (long)V);
    float4 r[kLpKR];
#pragma unroll
    for (int k = 0; k < kLpKR; ++k) {
        const int i = threadIdx.x + k * kLpThreads;
        r[k] = i < v4 ? x4[i] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < kLpKR; ++k) m = fmaxf(m, fmaxf(fmaxf(r[k].x, r[k].y), fmaxf(r[k].z, r[k].w)));
    m = block_max(m, red);
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < kLpKR; ++k)
        if (threadIdx.x + k * kLpThreads < v4)
            sm += expf(r[k].x - m) + expf(r[k].y - m) + expf(r[k].z - m) + expf(r[k].w - m);
    const float ls = logf(block_sum(sm, red));
    float4* l4 = reinterpret_cast<float4*>(logp + row * (long)V);
#pragma unroll
    for (int k = 0; k < kLpKR; ++k) {
        const int i = threadIdx.x + k * kLpThreads;
        if (i < v4) l4[i] = make_float4((r[k].x - m) - ls, (r[k].y - m) - ls, (r[k].z - m) - ls, (r[k].w - m) - ls);
    }
    if (threadIdx.x == 0) {
        const int64_t t = target[row];
        picked[row] = (t >= 0 && t < V) ? (x[row * (long)V + t] - m) - ls : NAN;
    }
}

__global__ __launch_bounds__(kLpThreads) void logprob_pick_bwd_reg_kernel(const float* __restrict__ logp,
                                                                         const int64_t* __restrict__ target,
                                                                         const float* __restrict__ gpick, int V,
                                                                         float* __restrict__ dx,
                                                                         uint16_t* __restrict__ dx16, int ldo) {
    const long row = blockIdx.x;
    const int v4 = V / 4;
    const float g = gpick[row];
    const int64_t t = target[row];
    const float4* l4 = reinterpret_cast<const float4*>(logp + row * (long)V);
    float4* d4 = reinterpret_cast<float4*>(dx + row * (long)ldo);
    for (int i = v4 + threadIdx.x; i < ldo / 4; i += kLpThreads) d4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 r[kLpKR];
#pragma unroll
    for (int k = 0; k < kLpKR; ++k) {
        const int i = threadIdx.x + k * kLpThreads;
        if (i < v4) r[k] = l4[i];
    }
#pragma unroll
    for (int k = 0; k < kLpKR; ++k) {
        const int i = threadIdx.x + k * kLpThreads;
        if (i < v4) {
            const int j = 4 * i;
            const float4 o = make_float4(g * ((j == t ? 1.f : 0.f) - expf(r[k].x)),
                                         g * ((j + 1 == t ? 1.f : 0.f) - expf(r[k].y)),
                                         g * ((j + 2 == t ? 1.f : 0.f) - expf(r[k].z)),
                                         g * ((j + 3 == t ? 1.f : 0.f) - expf(r[k].w)));
            d4[i] = o;
            if (dx16) store_bf16x4(dx16 + row * (long)V + j, o.x, o.y, o.z, o.w);
        }
    }
}

// Greedy decoding's word choice (LSTM_DSA.py:149-151: sampleLogprobs, it = torch.max(logprobs, 1) over
// logprobs = log_softmax(logits)): per row the first index of the largest logit and its log-probability
// (x_max - max) - log(sum exp(x - max)) = -log(sum exp(x - max)), from ONE read of the logits -- the (rows, V)
// log_softmax is never written.  One workgroup per row; per lane a running (max, first index) and (max, sum exp)
// pair, merged over the workgroup (ties to the smaller index, as torch.max).
__global__ __launch_bounds__(kLpThreads) void logprob_argmax_kernel(const float* __restrict__ x, int V,
                                                                   int64_t* __restrict__ idx,
                                                                   float* __restrict__ lp) {
    __shared__ float red_m[kLpThreads / PDVC_WAVE], red_s[kLpThreads / PDVC_WAVE];
    __shared__ int red_i[kLpThreads / PDVC_WAVE];
    const long row = blockIdx.x;
    const float* xr = x + row * (long)V;
    float m = -INFINITY, s = 0.f;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < V; i += kLpThreads) {
        const float v = xr[i];
        if (v > m || bi == 0x7fffffff) bi = i;  // a lane's indices ascend: ties keep the first
        lse_add(m, s, v);
    }
#pragma unroll
    for (int d = 1; d < PDVC_WAVE; d <<= 1) {
        const float m2 = lane_swap(m, d), s2 = lane_swap(s, d);
        const int i2 = __shfl_xor(bi, d, PDVC_WAVE);
        if (m2 > m || (m2 == m && i2 < bi)) bi = i2;
        lse_merge(m, s, m2, s2);
    }
    const int wave = threadIdx.x / PDVC_WAVE, lane = threadIdx.x % PDVC_WAVE;
    if (lane == 0) {
        red_m[wave] = m;
        red_s[wave] = s;
        red_i[wave] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        m = red_m[0];
        s = red_s[0];
        bi = red_i[0];
#pragma unroll
        for (int w = 1; w < kLpThreads / PDVC_WAVE; ++w) {
            if (red_m[w] > m || (red_m[w] == m && red_i[w] < bi)) bi = red_i[w];
            lse_merge(m, s, red_m[w], red_s[w]);
        }
        idx[row] = bi;
        lp[row] = (xr[bi] - m) - logf(s);
    }
}

// The same from registers for V <= kLpThreads * kLpKS (the caption vocabulary, 5 749): every scalar load of the row
// issued before any arithmetic (the streaming form above waited on one load per trip: 2.4 TB/s at 25 600 x 5 749),
// the (max, first index) pair reduced first, then sum exp(x - max) without a running rescale (torch's order)
constexpr int kLpKS = 32;

__global__ __launch_bounds__(kLpThreads) void logprob_argmax_reg_kernel(const float* __restrict__ x, int V,
                                                                       int64_t* __restrict__ idx,
                                                                       float* __restrict__ lp) {
    __shared__ float red_m[kLpThreads / PDVC_WAVE], red[kLpThreads / PDVC_WAVE];
    __shared__ int red_i[kLpThreads / PDVC_WAVE];
    const long row = blockIdx.x;
    const float* xr = x + row * (long)V;
    float r[kLpKS];
#pragma unroll
    for (int k = 0; k < kLpKS; ++k) {
        const int i = threadIdx.x + k * kLpThreads;
        r[k] = i < V ? xr[i] : -INFINITY;
    }
    float m = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < kLpKS; ++k) {  // a lane's indices ascend with k: ties keep the first
        const int i = threadIdx.x + k * kLpThreads;
        if (r[k] > m || (bi == 0x7fffffff && i < V)) {
            m = r[k];
            bi = i;
        }
    }
#pragma unroll
    for (int d = 1; d < PDVC_WAVE; d <<= 1) {
        const float m2 = lane_swap(m, d);
        const int i2 = __shfl_xor(bi, d, PDVC_WAVE);
        if (m2 > m || (m2 == m && i2 < bi)) {
            m = m2;
            bi = i2;
        }
    }
    const int wave = threadIdx.x / PDVC_WAVE;
    if ((threadIdx.x % PDVC_WAVE) == 0) {
        red_m[wave] = m;
        red_i[wave] = bi;
    }
    __syncthreads();
    m = red_m[0];
    bi = red_i[0];
#pragma unroll
    for (int w = 1; w < kLpThreads / PDVC_WAVE; ++w)
        if (red_m[w] > m || (red_m[w] == m && red_i[w] < bi)) {
            m = red_m[w];
            bi = red_i[w];
        }
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < kLpKS; ++k)
        if (threadIdx.x + k * kLpThreads < V) sm += expf(r[k] - m);
    const float s = block_sum(sm, red);
    if (threadIdx.x == 0) {
        idx[row] = bi;
        lp[row] = (xr[bi] - m) - logf(s);
    }
}

}  // namespace pdvc

using namespace pdvc;

extern "C" int pdvc_logprob_argmax_f32(const float* logits, int rows, int V, int64_t* index, float* logp_max,
                                       void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && V > 0, "invalid sizes (rows >= 0, V > 0)");
    PDVC_CHECK_ARG(rows == 0 || (logits && index && logp_max), "null pointer");
    if (rows == 0) return PDVC_OK;
    if (V <= kLpThreads * kLpKS)
        hipLaunchKernelGGL(logprob_argmax_reg_kernel, dim3((unsigned)rows), dim3(kLpThreads), 0, (hipStream_t)stream,
                           logits, V, index, logp_max);
    else
        hipLaunchKernelGGL(logprob_argmax_kernel, dim3((unsigned)rows), dim3(kLpThreads), 0, (hipStream_t)stream,
                           logits, V, index, logp_max);
    PDVC_CHECK_LAUNCH("logprob_argmax_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_logprob_pick_forward_f32(const float* logits, const int64_t* target, int rows, int V,
                                             float* logp, float* picked, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && V > 0, "invalid sizes (rows >= 0, V > 0)");
    PDVC_CHECK_ARG(rows == 0 || (logits && target && logp && picked), "null pointer");
    if (rows == 0) return PDVC_OK;
    const bool vec4 = (V % 4) == 0 && ((uintptr_t)logits % 16) == 0 && ((uintptr_t)logp % 16) == 0;
    hipStream_t s = (hipStream_t)stream;
    if (vec4 && V / 4 <= kLpThreads * kLpKR)
        hipLaunchKernelGGL(logprob_pick_fwd_reg_kernel, dim3((unsigned)rows), dim3(kLpThreads), 0, s, logits, target, V,
                           logp, picked);
    else if (vec4)
        hipLaunchKernelGGL(logprob_pick_fwd_kernel<true>, dim3((unsigned)rows), dim3(kLpThreads), 0, s, logits,
                           target, V, logp, picked);
    else
        hipLaunchKernelGGL(logprob_pick_fwd_kernel<false>, dim3((unsigned)rows), dim3(kLpThreads), 0, s, logits,
                           target, V, logp, picked);
    PDVC_CHECK_LAUNCH("logprob_pick_fwd_kernel");
    return PDVC_OK;
}

static int logprob_pick_backward_impl(const float* logp, const int64_t* target, const float* grad_picked, int rows,
                                      int V, int ldo, float* grad_logits, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && V > 0 && ldo >= V, "invalid sizes (rows >= 0, V > 0, ld >= V)");
    PDVC_CHECK_ARG(rows == 0 || (logp && target && grad_picked && grad_logits), "null pointer");
    if (rows == 0) return PDVC_OK;
    const bool vec4 = (V % 4) == 0 && (ldo % 4) == 0 && ((uintptr_t)logp % 16) == 0 &&
                      ((uintptr_t)grad_logits % 16) == 0;
    hipStream_t s = (hipStream_t)stream;
    if (vec4 && V / 4 <= kLpThreads * kLpKR)
        hipLaunchKernelGGL(logprob_pick_bwd_reg_kernel, dim3((unsigned)rows), dim3(kLpThreads), 0, s, logp, target,
                           grad_picked, V, grad_logits, (uint16_t*)nullptr, ldo);
    else if (vec4)
        hipLaunchKernelGGL(logprob_pick_bwd_kernel<true>, dim3((unsigned)rows), dim3(kLpThreads), 0, s, logp,
                           target, grad_picked, V, grad_logits, ldo);
    else
        hipLaunchKernelGGL(logprob_pick_bwd_kernel<false>, dim3((unsigned)rows), dim3(kLpThreads), 0, s, logp,
                           target, grad_picked, V, grad_logits, ldo);
    PDVC_CHECK_LAUNCH("logprob_pick_bwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_logprob_pick_backward_f32(const float* logp, const int64_t* target, const float* grad_picked,
                                              int rows, int V, float* grad_logits, void* stream) {
    return logprob_pick_backward_impl(logp, target, grad_picked, rows, V, V, grad_logits, stream);
}

// The same into rows of stride ld >= V whose columns [V, ld) are written as zeros: a K-padded operand for the logit
// layer's input-gradient GEMM (pdvc/ops/functions/logprob.py LogitPickFunction)
extern "C" int pdvc_logprob_pick_backward_ld_f32(const float* logp, const int64_t* target, const float* grad_picked,
                                                 int rows, int V, int ld, float* grad_logits, void* stream) {
    return logprob_pick_backward_impl(logp, target, grad_picked, rows, V, ld, grad_logits, stream);
}

// The bf16 mode's form (pdvc/precision.py): also writes grad_logits' bf16 rounding into grad16 -- the operand of
// the logit layer's two gradient GEMMs.  Only the register-resident form (V % 4 == 0, V / 4 <= 2048 float4s per
// row, 16-byte aligned rows): otherwise PDVC_ERR_UNSUPPORTED and nothing is launched (the caller casts instead).
extern "C" int pdvc_logprob_pick_backward_f32_bf16out(const float* logp, const int64_t* target,
                                                      const float* grad_picked, int rows, int V, float* grad_logits,
                                                      uint16_t* grad16, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && V > 0, "invalid sizes (rows >= 0, V > 0)");
    PDVC_CHECK_ARG(rows == 0 || (logp && target && grad_picked && grad_logits && grad16), "null pointer");
    const bool reg = (V % 4) == 0 && ((uintptr_t)logp % 16) == 0 && ((uintptr_t)grad_logits % 16) == 0 &&
                     ((uintptr_t)grad16 % 8) == 0 && V / 4 <= kLpThreads * kLpKR;
    if (!reg) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "bf16 shadow needs the register-resident row form");
    if (rows == 0) return PDVC_OK;
    hipLaunchKernelGGL(logprob_pick_bwd_reg_kernel, dim3((unsigned)rows), dim3(kLpThreads), 0, (hipStream_t)stream,
                       logp, target, grad_picked, V, grad_logits, grad16, V);
    PDVC_CHECK_LAUNCH("logprob_pick_bwd_reg_kernel");
    return PDVC_OK;
}
