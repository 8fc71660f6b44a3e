// mha.hip -- decoder query self-attention core for MI355X (gfx950).
//
// Replaces the attention core of nn.MultiheadAttention as DeformableTransformerDecoderLayer uses it
// (pdvc/deformable_transformer.py:231,256-258; torch's multi_head_attention_forward with need_weights):
//   P = softmax(q * sqrt(1/D) . k^T  [+ -inf at padded keys]),  P_d = dropout(P),  O = P_d . v
// The in/out projections stay GEMMs (hipBLASLt through torch).  PDVC's decoder (D = 64, Q = 100) takes the
// matrix-core kernels below (mha_*_mfma_kernel: one workgroup per (video, head), 32x32 fp32 MFMA tiles, the
// backward in one launch).  The scalar kernels serve any other shape (Q <= 300, D <= 64): a workgroup owns 16
// queries of one (video, head), K and V staged in LDS (rows padded to D+1 floats), a lane owns one key for the
// scores (exact softmax over <= 5 keys per lane + wave reductions) and one channel for P.V.  The dropout seed
// may come from device memory (seed_dev), so a captured hipGraph replays with a fresh seed drawn by the graph.
// Backward: phase A (query-major) recomputes P from the saved log-sum-exp, forms dS = P (dP - delta) with
// delta = dO . O, writes dq, and stages P_d and dS rows in a global workspace; phase B (key-major) forms
// dK = dS^T q_scaled and dV = P_d^T dO.
// Dropout keeps a counter-hash mask of (seed, video, head, query, key) -- regenerated in the backward.
#include "pdvc_common.h"
#include "seqattn.h"

#include <cstdlib>

namespace pdvc {

constexpr int kHD = 64;      // max head dim (PDVC: 512 / 8 = 64); lanes >= D idle in channel phases
constexpr int kMaxQ = 300;   // LDS budget: 2 * Q * (D+1) floats + row buffers <= 160 KiB

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = fmaxf(v, lane_swap(v, d));
    return v;
}
__device__ __forceinline__ float wave_add(float v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += lane_swap(v, d);
    return v;
}

constexpr int kKPL = (kMaxQ + 63) / 64;  // keys per lane

constexpr int kQB = 16;  // queries (forward / backward phase A) or keys (phase B) per workgroup

__global__ __launch_bounds__(256) void mha_fwd_kernel(const float* __restrict__ qk, const float* __restrict__ v,
                                                      const uint8_t* __restrict__ kpm, int Q, int M, int D, float scaling,
                                                      float p_drop, uint32_t thresh, uint64_t seed0,
                                                      const uint64_t* __restrict__ seed_dev, int qchunks,
                                                      float* __restrict__ out, float* __restrict__ lse) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int E = M * D;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);  // the chunks of one (video, head) share an XCD
    const int nm = lb / qchunks;
    const int q0 = (lb - nm * qchunks) * kQB, q1 = min(Q, q0 + kQB);
    const int n = nm / M, m = nm - n * M;
    const uint64_t seed = load_seed(seed0, seed_dev);
    float* Ks = smem;                      // [Q][D+1]
    float* Vs = Ks + Q * (D + 1);          // [Q][D]
    float* Ps = Vs + Q * D;                // [4][Q]
    float* Qrow = Ps + 4 * Q;              // [4][64]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int i = tid; i < Q * D; i += 256) {
        const int r = i / D, c = i - r * D;
        Ks[r * (D + 1) + c] = qk[((size_t)n * Q + r) * 2 * E + E + m * D + c];
        Vs[r * D + c] = v[((size_t)n * Q + r) * E + m * D + c];
    }
    __syncthreads();
    const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    float* prow = Ps + w * Q;
    float* qrow = Qrow + w * kHD;
    for (int q = q0 + w; q < q1; q += 4) {
        if (lane < D) qrow[lane] = qk[((size_t)n * Q + q) * 2 * E + m * D + lane] * scaling;
        __builtin_amdgcn_wave_barrier();
        float s[kKPL];
        float mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < kKPL; ++i) {
            const int k = lane + 64 * i;
            s[i] = -INFINITY;
            if (k < Q) {
                float acc = 0.f;
                const float* kr = Ks + k * (D + 1);
#pragma unroll 16
                for (int d = 0; d < D; ++d) acc += qrow[d] * kr[d];
                s[i] = (kpm && kpm[(size_t)n * Q + k]) ? -INFINITY : acc;
            }
            mx = fmaxf(mx, s[i]);
        }
        mx = wave_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < kKPL; ++i) {
            s[i] = (lane + 64 * i < Q) ? expf(s[i] - mx) : 0.f;
            sum += s[i];
        }
        sum = wave_add(sum);
        const float inv = 1.f / sum;
#pragma unroll
        for (int i = 0; i < kKPL; ++i) {
            const int k = lane + 64 * i;
            if (k < Q) {
                float p = s[i] * inv;
                if (p_drop > 0.f) p = keep_elem(seed, (uint32_t)nm, q, k, Q, thresh) ? p * keep_scale : 0.f;
                prow[k] = p;
            }
        }
        if (lane == 0) lse[(size_t)nm * Q + q] = mx + logf(sum);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (lane < D) {
            float o = 0.f;
            for (int k = 0; k < Q; ++k) o += prow[k] * Vs[k * D + lane];
            out[((size_t)n * Q + q) * E + m * D + lane] = o;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// backward phase A: one workgroup per (video, head, chunk of kQB queries)
__global__ __launch_bounds__(256) void mha_bwd_q_kernel(const float* __restrict__ qk, const float* __restrict__ v,
                                                        const uint8_t* __restrict__ kpm, const float* __restrict__ out,
                                                        const float* __restrict__ gout, const float* __restrict__ lse,
                                                        int Q, int M, int D, float scaling, float p_drop, uint32_t thresh,
                                                        uint64_t seed0, const uint64_t* __restrict__ seed_dev,
                                                        int qchunks, float* __restrict__ ws_p,
                                                        float* __restrict__ ws_ds, float* __restrict__ dqk) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int E = M * D;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int nm = lb / qchunks;
    const int q0 = (lb - nm * qchunks) * kQB, q1 = min(Q, q0 + kQB);
    const int n = nm / M, m = nm - n * M;
    const uint64_t seed = load_seed(seed0, seed_dev);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float* A = smem;                   // K [Q][D+1]
    float* B = A + Q * (D + 1);        // V [Q][D+1]
    float* R = B + Q * (D + 1);        // [4][Q] per-wave row buffer (dS row)
    float* Rv = R + 4 * Q;             // [4][64] per-wave q rows
    float* Ro = Rv + 4 * kHD;          // [4][64] per-wave dO rows
    for (int i = tid; i < Q * D; i += 256) {
        const int r = i / D, c = i - r * D;
        A[r * (D + 1) + c] = qk[((size_t)n * Q + r) * 2 * E + E + m * D + c];
        B[r * (D + 1) + c] = v[((size_t)n * Q + r) * E + m * D + c];
    }
    __syncthreads();
    const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    float* dsrow = R + w * Q;
    float* qrow = Rv + w * kHD;
    float* dorow = Ro + w * kHD;
    float* wsp = ws_p + (size_t)nm * Q * Q;
    float* wsd = ws_ds + (size_t)nm * Q * Q;
    for (int q = q0 + w; q < q1; q += 4) {
        const size_t orow = ((size_t)n * Q + q) * E + m * D;
        const float go = lane < D ? gout[orow + lane] : 0.f;
        if (lane < D) {
            qrow[lane] = qk[((size_t)n * Q + q) * 2 * E + m * D + lane] * scaling;
            dorow[lane] = go;
        }
        const float delta = wave_add(lane < D ? go * out[orow + lane] : 0.f);
        const float l = lse[(size_t)nm * Q + q];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < kKPL; ++i) {
            const int k = lane + 64 * i;
            if (k < Q) {
                float s = 0.f, dp = 0.f;
                const float* kr = A + k * (D + 1);
                const float* vr = B + k * (D + 1);
#pragma unroll 16
                for (int d = 0; d < D; ++d) {
                    s += qrow[d] * kr[d];
                    dp += dorow[d] * vr[d];
                }
                const bool masked = kpm && kpm[(size_t)n * Q + k];
                const float p = masked ? 0.f : expf(s - l);
                float z = 1.f;
                if (p_drop > 0.f) z = keep_elem(seed, (uint32_t)nm, q, k, Q, thresh) ? keep_scale : 0.f;
                const float ds = p * (dp * z - delta);
                dsrow[k] = ds;
                wsp[(size_t)q * Q + k] = p * z;
                wsd[(size_t)q * Q + k] = ds;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (lane < D) {
            float dq = 0.f;
            for (int k = 0; k < Q; ++k) dq += dsrow[k] * A[k * (D + 1) + lane];
            dqk[((size_t)n * Q + q) * 2 * E + m * D + lane] = dq * scaling;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// backward phase B: one workgroup per (video, head, chunk of kQB keys); dK = dS^T q_scaled, dV = P_d^T dO.
// The chunk's P_d / dS columns stay in LDS; dO and q_scaled stream through in 64-query slabs, each wave
// accumulating its kQB/4 keys with lanes over channels.
constexpr int kQS = 64;  // query slab
__global__ __launch_bounds__(256) void mha_bwd_k_kernel(const float* __restrict__ qk, const float* __restrict__ gout,
                                                        int Q, int M, int D, float scaling, int kchunks,
                                                        const float* __restrict__ ws_p, const float* __restrict__ ws_ds,
                                                        float* __restrict__ dqk, float* __restrict__ dv) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int KPW = kQB / 4;  // keys per wave
    const int E = M * D;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int nm = lb / kchunks;
    const int k0 = (lb - nm * kchunks) * kQB, k1 = min(Q, k0 + kQB);
    const int n = nm / M, m = nm - n * M;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float* Pc = smem;             // P_d columns of the chunk [kQB][Q]
    float* Dc = Pc + kQB * Q;     // dS columns [kQB][Q]
    float* A = Dc + kQB * Q;      // dO slab [kQS][D]
    float* B = A + kQS * D;       // q_scaled slab [kQS][D]
    const float* wsp = ws_p + (size_t)nm * Q * Q;
    const float* wsd = ws_ds + (size_t)nm * Q * Q;
    const int nk = k1 - k0;
    for (int i = tid; i < Q * nk; i += 256) {  // coalesced along keys within each query row
        const int q = i / nk, kk = i - q * nk;
        Pc[kk * Q + q] = wsp[(size_t)q * Q + k0 + kk];
        Dc[kk * Q + q] = wsd[(size_t)q * Q + k0 + kk];
    }
    float gk[KPW], gv[KPW];
#pragma unroll
    for (int j = 0; j < KPW; ++j) gk[j] = gv[j] = 0.f;
    for (int qs = 0; qs < Q; qs += kQS) {
        const int nq = min(kQS, Q - qs);
        __syncthreads();
        for (int i = tid; i < nq * D; i += 256) {
            const int r = i / D, c = i - r * D;
            A[r * D + c] = gout[((size_t)n * Q + qs + r) * E + m * D + c];
            B[r * D + c] = qk[((size_t)n * Q + qs + r) * 2 * E + m * D + c] * scaling;
        }
        __syncthreads();
        if (lane < D) {
#pragma unroll
            for (int j = 0; j < KPW; ++j) {
                const int kk = w * KPW + j;
                if (k0 + kk < k1) {
                    const float* pc = Pc + kk * Q + qs;
                    const float* dc = Dc + kk * Q + qs;
                    float a = 0.f, bsum = 0.f;
#pragma unroll 8
                    for (int q = 0; q < nq; ++q) {
                        a += pc[q] * A[q * D + lane];
                        bsum += dc[q] * B[q * D + lane];
                    }
                    gv[j] += a;
                    gk[j] += bsum;
                }
            }
        }
    }
    if (lane >= D) return;
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
        const int k = k0 + w * KPW + j;
        if (k < k1) {
            dqk[((size_t)n * Q + k) * 2 * E + E + m * D + lane] = gk[j];
            dv[((size_t)n * Q + k) * E + m * D + lane] = gv[j];
        }
    }
}

// ---------------------------------------------------------------------------------------------------------
// Matrix-core path (D == 64, Q <= 128: PDVC's decoder).  One 256-thread workgroup per (video, head) with the
// queries padded to 128 (zero rows / masked keys): wave w owns query rows 32w..32w+31.  Scores, P.V, dP, dq, dk
// and dv are 32x32 tiles of v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulation).  Operand layout
// of one MFMA step kk: lane l supplies A[l%32][2kk + l/32] and B[2kk + l/32][l%32]; accumulator register r of
// lane l holds C[(r&3) + 8(r>>2) + 4(l/32)][l%32].  Rows of the C tile are spread over 32-lane halves, so a row
// softmax is a 5-step butterfly inside each half.
typedef float mha_f32x16 __attribute__((ext_vector_type(16)));
constexpr int kMQ = 128;   // padded queries / keys
constexpr int kMLD = 65;   // LDS row stride of [row][channel] images (conflict-free column walks)

__device__ __forceinline__ int crow(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }

__device__ __forceinline__ mha_f32x16 mfma32(float a, float b, mha_f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// rows [0, Q) of one head's 64 channels (row stride `ld` floats, x `mul`) -> LDS [128][stride]; rows >= Q zero
__device__ __forceinline__ void mha_stage(const float* __restrict__ src, size_t ld, int Q, float mul, float* dst,
                                          int stride, int tid) {
    for (int i = tid; i < kMQ * 16; i += 256) {
        const int r = i >> 4, c = (i & 15) * 4;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < Q) x = *reinterpret_cast<const float4*>(src + (size_t)r * ld + c);
        float* d = dst + r * stride + c;
        d[0] = x.x * mul;
        d[1] = x.y * mul;
        d[2] = x.z * mul;
        d[3] = x.w * mul;
    }
}

__global__ __launch_bounds__(256) void mha_fwd_mfma_kernel(const float* __restrict__ qk, const float* __restrict__ v,
                                                           const uint8_t* __restrict__ kpm, int Q, int M,
                                                           float scaling, float p_drop, uint32_t thresh, uint64_t seed0,
                                                           const uint64_t* __restrict__ seed_dev,
                                                           float* __restrict__ out, float* __restrict__ lse) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int D = 64;
    constexpr int kPLD = kMQ + 1;               // P tile row stride
    float* Ks = smem;                           // [128][65]
    float* Qs = Ks + kMQ * kMLD;                // [128][65] q * scaling
    float* Vs = Qs + kMQ * kMLD;                // [128][64]
    const int E = M * D;
    const int nm = xcd_remap(blockIdx.x, gridDim.x);
    const int n = nm / M, m = nm - n * M;
    const uint64_t seed = load_seed(seed0, seed_dev);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hi = lane >> 5;
    const float* qbase = qk + (size_t)n * Q * 2 * E + m * D;
    mha_stage(qbase + E, 2 * (size_t)E, Q, 1.f, Ks, kMLD, tid);
    mha_stage(qbase, 2 * (size_t)E, Q, scaling, Qs, kMLD, tid);
    mha_stage(v + (size_t)n * Q * E + m * D, (size_t)E, Q, 1.f, Vs, D, tid);
    __syncthreads();
    const int row0 = w * 32;
    mha_f32x16 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) s[kb] = mha_f32x16{};
    {
        const float* qa = Qs + (row0 + l32) * kMLD + hi;
        const float* kbp = Ks + l32 * kMLD + hi;
#pragma unroll 8
        for (int kk = 0; kk < D / 2; ++kk) {
            const float a = qa[2 * kk];
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) s[kb] = mfma32(a, kbp[kb * 32 * kMLD + 2 * kk], s[kb]);
        }
    }
    bool kval[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        const int k = kb * 32 + l32;
        kval[kb] = k < Q && !(kpm && kpm[(size_t)n * Q + k]);
    }
    __syncthreads();  // every wave is done with Ks / Qs: the P tiles reuse that space
    float* Pw = smem + w * 32 * kPLD;  // [32][129] this wave's P_d rows
    const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rl = crow(r, hi), q = row0 + rl;
        float mx = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) mx = fmaxf(mx, kval[kb] ? s[kb][r] : -INFINITY);
#pragma unroll
        for (int d = 16; d > 0; d >>= 1) mx = fmaxf(mx, lane_swap(mx, d));
        float e[4], sum = 0.f;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            e[kb] = kval[kb] ? expf(s[kb][r] - mx) : 0.f;
            sum += e[kb];
        }
#pragma unroll
        for (int d = 16; d > 0; d >>= 1) sum += lane_swap(sum, d);
        const float inv = 1.f / sum;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            const int k = kb * 32 + l32;
            float p = e[kb] * inv;
            if (p_drop > 0.f && q < Q && k < Q)
                p = keep_elem(seed, (uint32_t)nm, (uint32_t)q, (uint32_t)k, (uint32_t)Q, thresh) ? p * keep_scale : 0.f;
            Pw[rl * kPLD + k] = p;
        }
        if (l32 == 0 && q < Q) lse[(size_t)nm * Q + q] = mx + logf(sum);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    mha_f32x16 o[2] = {mha_f32x16{}, mha_f32x16{}};
    {
        const float* pa = Pw + l32 * kPLD + hi;
        const float* vb = Vs + hi * D + l32;
#pragma unroll 8
        for (int kk = 0; kk < kMQ / 2; ++kk) {
            const float a = pa[2 * kk];
            o[0] = mfma32(a, vb[2 * kk * D], o[0]);
            o[1] = mfma32(a, vb[2 * kk * D + 32], o[1]);
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int q = row0 + crow(r, hi);
        if (q < Q) {
            float* orow = out + ((size_t)n * Q + q) * E + m * D + l32;
            orow[0] = o[0][r];
            orow[32] = o[1][r];
        }
    }
}

// The same forward in 66 KiB of LDS (two workgroups per CU instead of one: mha_fwd_mfma_kernel's K, Q and V images
// take 99 KiB).  A wave's query rows are its own MFMA A operand, so they are loaded straight into registers:
// k-step kk of lane half hi takes channel 32*hi + kk (a permutation of the contraction index, applied to the K
// image reads as well), i.e. each lane reads 32 contiguous channels of its query row.  P_d is written in two
// 64-key halves into the K image (no longer needed once every wave has its scores), each half consumed by the
// P.V MFMAs before the next is written.  Same softmax, dropout mask and log-sum-exp as mha_fwd_mfma_kernel.
static constexpr int kPHLD = 65;  // P half-tile row stride (64 keys + 1)

__global__ __launch_bounds__(256) void mha_fwd_mfma2_kernel(const float* __restrict__ qk, const float* __restrict__ v,
                                                            const uint8_t* __restrict__ kpm, int Q, int M,
                                                            float scaling, float p_drop, uint32_t thresh,
                                                            uint64_t seed0, const uint64_t* __restrict__ seed_dev,
                                                            float* __restrict__ out, float* __restrict__ lse) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int D = 64;
    float* Ks = smem;                // [128][65]
    float* Vs = Ks + kMQ * kMLD;     // [128][64]
    const int E = M * D;
    const int nm = xcd_remap(blockIdx.x, gridDim.x);
    const int n = nm / M, m = nm - n * M;
    const uint64_t seed = load_seed(seed0, seed_dev);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hi = lane >> 5;
    const float* qbase = qk + (size_t)n * Q * 2 * E + m * D;
    const int row0 = w * 32;
    float qa[32];  // q[row0 + l32][32*hi + kk] * scaling (zeros past Q)
    {
        const int q = row0 + l32;
        const float4* src = reinterpret_cast<const float4*>(qbase + (size_t)q * 2 * E + 32 * hi);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 x = q < Q ? src[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            qa[4 * i] = x.x * scaling;
            qa[4 * i + 1] = x.y * scaling;
            qa[4 * i + 2] = x.z * scaling;
            qa[4 * i + 3] = x.w * scaling;
        }
    }
    mha_stage(qbase + E, 2 * (size_t)E, Q, 1.f, Ks, kMLD, tid);
    mha_stage(v + (size_t)n * Q * E + m * D, (size_t)E, Q, 1.f, Vs, D, tid);
    __syncthreads();
    mha_f32x16 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) s[kb] = mha_f32x16{};
    {
        const float* kbp = Ks + l32 * kMLD + 32 * hi;
#pragma unroll
        for (int kk = 0; kk < D / 2; ++kk) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) s[kb] = mfma32(qa[kk], kbp[kb * 32 * kMLD + kk], s[kb]);
        }
    }
    bool kval[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        const int k = kb * 32 + l32;
        kval[kb] = k < Q && !(kpm && kpm[(size_t)n * Q + k]);
    }
    // softmax rows in registers: s[kb][r] becomes P_d
    const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rl = crow(r, hi), q = row0 + rl;
        float mx = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) mx = fmaxf(mx, kval[kb] ? s[kb][r] : -INFINITY);
#pragma unroll
        for (int d = 16; d > 0; d >>= 1) mx = fmaxf(mx, lane_swap(mx, d));
        float e[4], sum = 0.f;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            e[kb] = kval[kb] ? expf(s[kb][r] - mx) : 0.f;
            sum += e[kb];
        }
#pragma unroll
        for (int d = 16; d > 0; d >>= 1) sum += lane_swap(sum, d);
        const float inv = 1.f / sum;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            const int k = kb * 32 + l32;
            float p = e[kb] * inv;
            if (p_drop > 0.f && q < Q && k < Q)
                p = keep_elem(seed, (uint32_t)nm, (uint32_t)q, (uint32_t)k, (uint32_t)Q, thresh) ? p * keep_scale : 0.f;
            s[kb][r] = p;
        }
        if (l32 == 0 && q < Q) lse[(size_t)nm * Q + q] = mx + logf(sum);
    }
    __syncthreads();  // every wave is done with the K image: the P halves reuse it
    float* Pw = smem + w * 32 * kPHLD;  // [32][65] this wave's P_d rows, one 64-key half at a time
    mha_f32x16 o[2] = {mha_f32x16{}, mha_f32x16{}};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rl = crow(r, hi);
            Pw[rl * kPHLD + l32] = s[2 * h][r];
            Pw[rl * kPHLD + 32 + l32] = s[2 * h + 1][r];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float* pa = Pw + l32 * kPHLD + hi;
        const float* vb = Vs + (64 * h + hi) * D + l32;
#pragma unroll 8
        for (int kk = 0; kk < 32; ++kk) {
            const float a = pa[2 * kk];
            o[0] = mfma32(a, vb[2 * kk * D], o[0]);
            o[1] = mfma32(a, vb[2 * kk * D + 32], o[1]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int q = row0 + crow(r, hi);
        if (q < Q) {
            float* orow = out + ((size_t)n * Q + q) * E + m * D + l32;
            orow[0] = o[0][r];
            orow[32] = o[1][r];
        }
    }
}

// Backward, one workgroup per (video, head).  Phase A (wave w = query rows 32w..): recompute P from the saved
// log-sum-exp, dP_d = dO . V^T, dS = P (dP_d z - delta), dq = dS . K; P_d and dS go to the global workspace
// (stays in L2: this workgroup reads it back).  Phase B (wave w = key rows 32w..): dk = dS^T . q_scaled,
// dv = P_d^T . dO, A operands read from the workspace, B operands from the LDS images of phase A.
__global__ __launch_bounds__(256) void mha_bwd_mfma_kernel(const float* __restrict__ qk, const float* __restrict__ v,
                                                           const uint8_t* __restrict__ kpm,
                                                           const float* __restrict__ out,
                                                           const float* __restrict__ gout,
                                                           const float* __restrict__ lse, int Q, int M, float scaling,
                                                           float p_drop, uint32_t thresh, uint64_t seed0,
                                                           const uint64_t* __restrict__ seed_dev,
                                                           float* __restrict__ ws_p, float* __restrict__ ws_ds,
                                                           float* __restrict__ dqk, float* __restrict__ dv) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int D = 64;
    constexpr int kDLD = 33;
    float* Ks = smem;                     // [128][65]
    float* Vs = Ks + kMQ * kMLD;          // [128][65]
    float* Qs = Vs + kMQ * kMLD;          // [128][65] q * scaling
    float* Os = Qs + kMQ * kMLD;          // [128][65] dO
    float* Ds = Os + kMQ * kMLD;          // [4][32][33] per-wave dS block
    float* rowl = Ds + 4 * 32 * kDLD;     // [128] lse
    float* rowd = rowl + kMQ;             // [128] delta = dO . O
    const int E = M * D;
    const int nm = xcd_remap(blockIdx.x, gridDim.x);
    const int n = nm / M, m = nm - n * M;
    const uint64_t seed = load_seed(seed0, seed_dev);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hi = lane >> 5;
    const float* qbase = qk + (size_t)n * Q * 2 * E + m * D;
    const size_t hbase = (size_t)n * Q * E + m * D;
    mha_stage(qbase + E, 2 * (size_t)E, Q, 1.f, Ks, kMLD, tid);
    mha_stage(v + hbase, (size_t)E, Q, 1.f, Vs, kMLD, tid);
    mha_stage(qbase, 2 * (size_t)E, Q, scaling, Qs, kMLD, tid);
    mha_stage(gout + hbase, (size_t)E, Q, 1.f, Os, kMLD, tid);
    if (tid < kMQ) {
        float dl = 0.f, l = 0.f;
        if (tid < Q) {
            const float4* orow = reinterpret_cast<const float4*>(out + hbase + (size_t)tid * E);
            const float4* grow = reinterpret_cast<const float4*>(gout + hbase + (size_t)tid * E);
#pragma unroll 4
            for (int c = 0; c < D / 4; ++c) {
                const float4 a = orow[c], b = grow[c];
                dl += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
            }
            l = lse[(size_t)nm * Q + tid];
        }
        rowd[tid] = dl;
        rowl[tid] = l;
    }
    __syncthreads();
    const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    float* wsp = ws_p + (size_t)nm * Q * Q;
    float* wsd = ws_ds + (size_t)nm * Q * Q;
    const int row0 = w * 32;
    float* Dw = Ds + w * 32 * kDLD;
    mha_f32x16 dq[2] = {mha_f32x16{}, mha_f32x16{}};
#pragma unroll 1
    for (int kb = 0; kb < 4; ++kb) {
        const int k = kb * 32 + l32;
        const bool kv = k < Q && !(kpm && kpm[(size_t)n * Q + k]);
        mha_f32x16 s = mha_f32x16{}, dp = mha_f32x16{};
        {
            const float* qa = Qs + (row0 + l32) * kMLD + hi;
            const float* oa = Os + (row0 + l32) * kMLD + hi;
            const float* kbp = Ks + k * kMLD + hi;
            const float* vbp = Vs + k * kMLD + hi;
#pragma unroll 8
            for (int kk = 0; kk < D / 2; ++kk) {
                s = mfma32(qa[2 * kk], kbp[2 * kk], s);
                dp = mfma32(oa[2 * kk], vbp[2 * kk], dp);
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rl = crow(r, hi), q = row0 + rl;
            float ds = 0.f;
            if (q < Q) {
                const float p = kv ? expf(s[r] - rowl[q]) : 0.f;
                float z = 1.f;
                if (p_drop > 0.f && k < Q)
                    z = keep_elem(seed, (uint32_t)nm, (uint32_t)q, (uint32_t)k, (uint32_t)Q, thresh) ? keep_scale : 0.f;
                ds = p * (dp[r] * z - rowd[q]);
                if (k < Q) {
                    wsp[(size_t)q * Q + k] = p * z;
                    wsd[(size_t)q * Q + k] = ds;
                }
            }
            Dw[rl * kDLD + l32] = ds;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        {
            const float* da = Dw + l32 * kDLD + hi;
            const float* kb0 = Ks + (kb * 32 + hi) * kMLD + l32;
#pragma unroll 8
            for (int kk = 0; kk < 16; ++kk) {
                const float a = da[2 * kk];
                dq[0] = mfma32(a, kb0[2 * kk * kMLD], dq[0]);
                dq[1] = mfma32(a, kb0[2 * kk * kMLD + 32], dq[1]);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int q = row0 + crow(r, hi);
        if (q < Q) {
            float* drow = dqk + ((size_t)n * Q + q) * 2 * E + m * D + l32;
            drow[0] = dq[0][r] * scaling;
            drow[32] = dq[1][r] * scaling;
        }
    }
    __syncthreads();  // the workspace rows of every wave are written (global writes visible to the workgroup)
    // phase B: wave w owns keys key0..key0+31
    const int key0 = w * 32, kl = key0 + l32;
    mha_f32x16 gk[2] = {mha_f32x16{}, mha_f32x16{}}, gv[2] = {mha_f32x16{}, mha_f32x16{}};
    if (key0 < Q) {
        const int half = (Q + 1) >> 1;
        const bool kin = kl < Q;
        for (int kk0 = 0; kk0 < half; kk0 += 4) {  // q <= 2 * (half + 3) + 1 < 128: padded LDS rows are zero
            float ad[4], ap[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int q = 2 * (kk0 + j) + hi;
                const bool in = kin && q < Q;
                ad[j] = in ? wsd[(size_t)q * Q + kl] : 0.f;
                ap[j] = in ? wsp[(size_t)q * Q + kl] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int q = 2 * (kk0 + j) + hi;
                const float* qb = Qs + q * kMLD + l32;
                const float* ob = Os + q * kMLD + l32;
                gk[0] = mfma32(ad[j], qb[0], gk[0]);
                gk[1] = mfma32(ad[j], qb[32], gk[1]);
                gv[0] = mfma32(ap[j], ob[0], gv[0]);
                gv[1] = mfma32(ap[j], ob[32], gv[1]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int k = key0 + crow(r, hi);
        if (k < Q) {
            float* krow = dqk + ((size_t)n * Q + k) * 2 * E + E + m * D + l32;
            float* vrow = dv + ((size_t)n * Q + k) * E + m * D + l32;
            krow[0] = gk[0][r];
            krow[32] = gk[1][r];
            vrow[0] = gv[0][r];
            vrow[32] = gv[1][r];
        }
    }
}


// Backward in 51 KiB of LDS (mha_bwd_mfma_kernel's four 33-KiB row images held one workgroup per CU; this one is held
// at two by its 248 registers -- the own-row A operands take 64): the K / V rows (phase A) and the q / dO rows
// (phase B) stream through two 32-row block buffers, the next block staged after the current one's MFMAs (a register
// prefetch under them took the kernel to 264 registers, one workgroup per CU).  Phase A (wave w = query rows 32w..32w+31) takes its
// own q (scaled) and dO rows as register A operands with mha_fwd_mfma2_kernel's permuted contraction index (k-step kk
// of lane half hi = channel 32*hi + kk, the same for the B reads of the K / V block), so no q / dO image is staged
// for it.  Per key block: S, dP_d, P = exp(S - lse), dS = P (dP_d z - delta), P_d and dS to the workspace, dq += dS.K
// through the wave's 32x33 dS block.  Phase B (wave w = keys 32w..32w+31): dk = dS^T.q_scaled, dv = P_d^T.dO, A
// operands from the workspace, B operands from the q / dO block.  Same arithmetic as mha_bwd_mfma_kernel per element
// and the same summation order over keys (dq) and queries (dk, dv).
static constexpr int kBlkLd = 65;                       // block row stride (conflict-free column walks)
static constexpr int kBlkF = 32 * kBlkLd;               // floats per 32-row block image
static constexpr size_t kBwdMfma2Lds = sizeof(float) * (4 * kBlkF + 4 * 32 * 33 + 2 * kMQ);

// rows [r0, r0 + 32) of one head's 64 channels (row stride ld, x mul; rows >= Q zero) into two float4 registers per
// thread, then into a 32-row block image
struct BlkRegs {
    float4 x[2];
};
__device__ __forceinline__ BlkRegs blk_load(const float* __restrict__ src, size_t ld, int r0, int Q, float mul,
                                            int tid) {
    BlkRegs b;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int idx = tid + 256 * i, r = idx >> 4, c = (idx & 15) * 4;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r0 + r < Q) x = *reinterpret_cast<const float4*>(src + (size_t)(r0 + r) * ld + c);
        b.x[i] = make_float4(x.x * mul, x.y * mul, x.z * mul, x.w * mul);
    }
    return b;
}
__device__ __forceinline__ void blk_store(const BlkRegs& b, float* dst, int tid) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int idx = tid + 256 * i, r = idx >> 4, c = (idx & 15) * 4;
        float* d = dst + r * kBlkLd + c;
        d[0] = b.x[i].x;
        d[1] = b.x[i].y;
        d[2] = b.x[i].z;
        d[3] = b.x[i].w;
    }
}

__global__ __launch_bounds__(256) void mha_bwd_mfma2_kernel(const float* __restrict__ qk, const float* __restrict__ v,
                                                            const uint8_t* __restrict__ kpm,
                                                            const float* __restrict__ out,
                                                            const float* __restrict__ gout,
                                                            const float* __restrict__ lse, int Q, int M, float scaling,
                                                            float p_drop, uint32_t thresh, uint64_t seed0,
                                                            const uint64_t* __restrict__ seed_dev,
                                                            float* __restrict__ ws_p, float* __restrict__ ws_ds,
                                                            float* __restrict__ dqk, float* __restrict__ dv) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int D = 64;
    constexpr int kDLD = 33;
    float* blk = smem;                    // [2 buffers][2 images][32][65]
    float* Ds = blk + 4 * kBlkF;          // [4][32][33] per-wave dS block
    float* rowl = Ds + 4 * 32 * kDLD;     // [128] lse
    float* rowd = rowl + kMQ;             // [128] delta = dO . O
    const int E = M * D;
    const int nm = xcd_remap(blockIdx.x, gridDim.x);
    const int n = nm / M, m = nm - n * M;
    const uint64_t seed = load_seed(seed0, seed_dev);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hi = lane >> 5;
    const float* qbase = qk + (size_t)n * Q * 2 * E + m * D;
    const size_t hbase = (size_t)n * Q * E + m * D;
    const int nblk = (Q + 31) >> 5;
    // block 0 of K and V first (their loads in flight while the own rows and the row statistics load)
    BlkRegs pk = blk_load(qbase + E, 2 * (size_t)E, 0, Q, 1.f, tid);
    BlkRegs pv = blk_load(v + hbase, (size_t)E, 0, Q, 1.f, tid);
    const int row0 = w * 32;
    float qa[32], oa[32];  // q[row0 + l32][32*hi + kk] * scaling and dO[row0 + l32][32*hi + kk] (zeros past Q)
    {
        const int q = row0 + l32;
        const float4* qs = reinterpret_cast<const float4*>(qbase + (size_t)q * 2 * E + 32 * hi);
        const float4* os = reinterpret_cast<const float4*>(gout + hbase + (size_t)q * E + 32 * hi);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 x = q < Q ? qs[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 y = q < Q ? os[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            qa[4 * i] = x.x * scaling;
            qa[4 * i + 1] = x.y * scaling;
            qa[4 * i + 2] = x.z * scaling;
            qa[4 * i + 3] = x.w * scaling;
            oa[4 * i] = y.x;
            oa[4 * i + 1] = y.y;
            oa[4 * i + 2] = y.z;
            oa[4 * i + 3] = y.w;
        }
    }
    if (tid < kMQ) {
        float dl = 0.f, l = 0.f;
        if (tid < Q) {
            const float4* orow = reinterpret_cast<const float4*>(out + hbase + (size_t)tid * E);
            const float4* grow = reinterpret_cast<const float4*>(gout + hbase + (size_t)tid * E);
#pragma unroll 4
            for (int c = 0; c < D / 4; ++c) {
                const float4 a = orow[c], b = grow[c];
                dl += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
            }
            l = lse[(size_t)nm * Q + tid];
        }
        rowd[tid] = dl;
        rowl[tid] = l;
    }
    blk_store(pk, blk, tid);
    blk_store(pv, blk + kBlkF, tid);
    __syncthreads();
    const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    float* wsp = ws_p + (size_t)nm * Q * Q;
    float* wsd = ws_ds + (size_t)nm * Q * Q;
    float* Dw = Ds + w * 32 * kDLD;
    mha_f32x16 dq[2] = {mha_f32x16{}, mha_f32x16{}};
    // phase A: key blocks
#pragma unroll 1
    for (int kb = 0; kb < nblk; ++kb) {
        const float* Kb = blk + (kb & 1) * 2 * kBlkF;
        const float* Vb = Kb + kBlkF;
        const bool more = kb + 1 < nblk;
        const int k = kb * 32 + l32;
        const bool kv = k < Q && !(kpm && kpm[(size_t)n * Q + k]);
        mha_f32x16 s = mha_f32x16{}, dp = mha_f32x16{};
        {
            const float* kbp = Kb + l32 * kBlkLd + 32 * hi;
            const float* vbp = Vb + l32 * kBlkLd + 32 * hi;
            // in chunks of 8 k-steps: the compiler would otherwise hoist all 64 operand reads of the block (64 VGPRs)
#pragma unroll
            for (int c = 0; c < D / 2; c += 8) {
#pragma unroll
                for (int kk = c; kk < c + 8; ++kk) {
                    s = mfma32(qa[kk], kbp[kk], s);
                    dp = mfma32(oa[kk], vbp[kk], dp);
                }
                __asm__ volatile("" ::: "memory");
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rl = crow(r, hi), q = row0 + rl;
            float ds = 0.f;
            if (q < Q) {
                const float p = kv ? expf(s[r] - rowl[q]) : 0.f;
                float z = 1.f;
                if (p_drop > 0.f && k < Q)
                    z = keep_elem(seed, (uint32_t)nm, (uint32_t)q, (uint32_t)k, (uint32_t)Q, thresh) ? keep_scale : 0.f;
                ds = p * (dp[r] * z - rowd[q]);
                if (k < Q) {
                    wsp[(size_t)q * Q + k] = p * z;
                    wsd[(size_t)q * Q + k] = ds;
                }
            }
            Dw[rl * kDLD + l32] = ds;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        {
            const float* da = Dw + l32 * kDLD + hi;
            const float* kb0 = Kb + hi * kBlkLd + l32;
#pragma unroll 8
            for (int kk = 0; kk < 16; ++kk) {
                const float a = da[2 * kk];
                dq[0] = mfma32(a, kb0[2 * kk * kBlkLd], dq[0]);
                dq[1] = mfma32(a, kb0[2 * kk * kBlkLd + 32], dq[1]);
            }
        }
        if (more) {  // the next block into the other buffer (every wave finished reading it before the last barrier)
            pk = blk_load(qbase + E, 2 * (size_t)E, (kb + 1) * 32, Q, 1.f, tid);
            pv = blk_load(v + hbase, (size_t)E, (kb + 1) * 32, Q, 1.f, tid);
            float* nb = blk + ((kb + 1) & 1) * 2 * kBlkF;
            blk_store(pk, nb, tid);
            blk_store(pv, nb + kBlkF, tid);
        }
        __syncthreads();  // the next block is staged; this wave's dS block may be rewritten
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int q = row0 + crow(r, hi);
        if (q < Q) {
            float* drow = dqk + ((size_t)n * Q + q) * 2 * E + m * D + l32;
            drow[0] = dq[0][r] * scaling;
            drow[32] = dq[1][r] * scaling;
        }
    }
    // phase B: wave w owns keys key0..key0+31; query blocks of q (scaled) and dO stream through the block buffers.
    // The workspace rows of every wave were written before the last barrier of phase A (visible to the workgroup).
    const int key0 = w * 32, kl = key0 + l32;
    const bool kin = kl < Q;
    mha_f32x16 gk[2] = {mha_f32x16{}, mha_f32x16{}}, gv[2] = {mha_f32x16{}, mha_f32x16{}};
    pk = blk_load(qbase, 2 * (size_t)E, 0, Q, scaling, tid);
    pv = blk_load(gout + hbase, (size_t)E, 0, Q, 1.f, tid);
    blk_store(pk, blk, tid);
    blk_store(pv, blk + kBlkF, tid);
    __syncthreads();
#pragma unroll 1
    for (int qb = 0; qb < nblk; ++qb) {
        const float* Qb = blk + (qb & 1) * 2 * kBlkF;
        const float* Ob = Qb + kBlkF;
        const bool more = qb + 1 < nblk;
        if (key0 < Q) {
#pragma unroll 4
            for (int kk = 0; kk < 16; ++kk) {
                const int ql = 2 * kk + hi, q = qb * 32 + ql;
                const bool in = kin && q < Q;
                const float ad = in ? wsd[(size_t)q * Q + kl] : 0.f;
                const float ap = in ? wsp[(size_t)q * Q + kl] : 0.f;
                const float* qr = Qb + ql * kBlkLd + l32;
                const float* orr = Ob + ql * kBlkLd + l32;
                gk[0] = mfma32(ad, qr[0], gk[0]);
                gk[1] = mfma32(ad, qr[32], gk[1]);
                gv[0] = mfma32(ap, orr[0], gv[0]);
                gv[1] = mfma32(ap, orr[32], gv[1]);
            }
        }
        if (more) {
            pk = blk_load(qbase, 2 * (size_t)E, (qb + 1) * 32, Q, scaling, tid);
            pv = blk_load(gout + hbase, (size_t)E, (qb + 1) * 32, Q, 1.f, tid);
            float* nb = blk + ((qb + 1) & 1) * 2 * kBlkF;
            blk_store(pk, nb, tid);
            blk_store(pv, nb + kBlkF, tid);
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int k = key0 + crow(r, hi);
        if (k < Q) {
            float* krow = dqk + ((size_t)n * Q + k) * 2 * E + E + m * D + l32;
            float* vrow = dv + ((size_t)n * Q + k) * E + m * D + l32;
            krow[0] = gk[0][r];
            krow[32] = gk[1][r];
            vrow[0] = gv[0][r];
            vrow[32] = gv[1][r];
        }
    }
}


}  // namespace pdvc

using namespace pdvc;

static size_t fwd_lds(int Q, int D) { return sizeof(float) * ((size_t)Q * (D + 1) + (size_t)Q * D + 4 * Q + 4 * kHD); }
static size_t bwdq_lds(int Q, int D) { return sizeof(float) * (2 * (size_t)Q * (D + 1) + 4 * Q + 8 * kHD); }
static size_t bwdk_lds(int Q, int D) { return sizeof(float) * (2 * (size_t)kQB * Q + 2 * (size_t)kQS * D); }
static constexpr size_t kFwdMfmaLds = sizeof(float) * (2 * kMQ * kMLD + kMQ * 64);
static constexpr size_t kFwdMfma2Lds = sizeof(float) * (kMQ * kMLD + kMQ * 64);
static_assert(sizeof(float) * 4 * 32 * kPHLD <= sizeof(float) * kMQ * kMLD, "P half tiles must fit in the K image");
static constexpr size_t kBwdMfmaLds = sizeof(float) * (4 * kMQ * kMLD + 4 * 32 * 33 + 2 * kMQ);
static_assert(sizeof(float) * 4 * 32 * (kMQ + 1) <= sizeof(float) * 2 * kMQ * kMLD, "P tiles must fit in K/Q images");
static_assert(kBwdMfmaLds <= 160 * 1024, "backward LDS budget");

// matrix-core kernels for D == 64, Q <= 128 (PDVC_MHA_MFMA=0 selects the scalar kernels, for tests)
static bool use_mfma(int Q, int D) {
    if (D != 64 || Q > kMQ) return false;
    const char* e = getenv("PDVC_MHA_MFMA");
    return !(e && e[0] == '0');
}

// the 66-KiB forward (two workgroups per CU); PDVC_MHA_FWD2=0 keeps the 99-KiB one (A/B)
static bool fwd_lean() {
    static const bool on = [] {
        const char* e = getenv("PDVC_MHA_FWD2");
        return !(e && e[0] == '0');
    }();
    return on;
}

// the 51-KiB backward (three workgroups per CU); PDVC_MHA_BWD2=0 keeps the 133-KiB one (A/B, tests)
static bool bwd_lean() {
    const char* e = getenv("PDVC_MHA_BWD2");
    return !(e && e[0] == '0');
}

// longer query sets (anet_c3d: Q = 300): the flash-style MFMA kernels of seqattn.hip with this op's key padding
// mask, dropout mask and scaling (PDVC_MHA_MFMA=0 selects the scalar kernels here too)
static bool use_flash(int Q, int D) {
    static const int force = [] {  // PDVC_MHA_FLASH=1: the flash route for every Q (A/B against the single-workgroup kernels)
        const char* e = getenv("PDVC_MHA_FLASH");
        return (e && e[0] == '1') ? 1 : 0;
    }();
    if ((Q <= kMQ && !force) || !sq_head_dim_ok(D)) return false;
    const char* e = getenv("PDVC_MHA_MFMA");
    return !(e && e[0] == '0');
}

static int mha_attrs() {
    static std::atomic<int> done[kMaxDevices];
    const int b = 160 * 1024;
    return lds_optin(done, {{(const void*)mha_fwd_kernel, b}, {(const void*)mha_bwd_q_kernel, b},
                            {(const void*)mha_bwd_k_kernel, b}, {(const void*)mha_fwd_mfma_kernel, b},
                            {(const void*)mha_bwd_mfma_kernel, b}, {(const void*)mha_fwd_mfma2_kernel, b},
                            {(const void*)mha_bwd_mfma2_kernel, b}},
                     "mha");
}

extern "C" int pdvc_mha_forward_f32(const float* qk, const float* v, const uint8_t* key_padding_mask, int batch,
                                    int num_query, int num_heads, int head_dim, float dropout_p, uint64_t seed,
                                    const uint64_t* seed_dev, float* out, float* lse, void* stream) {
    PDVC_CHECK_ARG(head_dim > 0 && head_dim <= kHD, "query self-attention kernel needs head_dim <= %d, got %d", kHD,
                   head_dim);
    PDVC_CHECK_ARG(num_query > 0 && num_query <= kMaxQ, "num_query must be in [1,%d], got %d", kMaxQ, num_query);
    PDVC_CHECK_ARG(batch >= 0 && num_heads > 0, "invalid sizes");
    PDVC_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f, "dropout_p must be in [0,1)");
    const int qchunks = (num_query + kQB - 1) / kQB;
    const long blocks = (long)batch * num_heads * qchunks;
    if (blocks == 0) return PDVC_OK;
    int rc = mha_attrs();
    if (rc) return rc;
    const float scaling = sqrtf(1.0f / (float)head_dim);
    if (use_flash(num_query, head_dim)) {
        const long E = (long)num_heads * head_dim;
        return sq_forward(qk, 2 * E, qk + E, 2 * E, v, E, batch, num_query, num_query, num_heads, head_dim, scaling,
                          key_padding_mask, dropout_p, seed, seed_dev, out, lse, (hipStream_t)stream);
    }
    if (use_mfma(num_query, head_dim) && fwd_lean()) {
        hipLaunchKernelGGL(mha_fwd_mfma2_kernel, dim3((unsigned)((long)batch * num_heads)), dim3(256), kFwdMfma2Lds,
                           (hipStream_t)stream, qk, v, key_padding_mask, num_query, num_heads, scaling, dropout_p,
                           drop_threshold(dropout_p), seed, seed_dev, out, lse);
        PDVC_CHECK_LAUNCH("mha_fwd_mfma2_kernel");
        return PDVC_OK;
    }
    if (use_mfma(num_query, head_dim)) {
        hipLaunchKernelGGL(mha_fwd_mfma_kernel, dim3((unsigned)((long)batch * num_heads)), dim3(256), kFwdMfmaLds,
                           (hipStream_t)stream, qk, v, key_padding_mask, num_query, num_heads, scaling, dropout_p,
                           drop_threshold(dropout_p), seed, seed_dev, out, lse);
        PDVC_CHECK_LAUNCH("mha_fwd_mfma_kernel");
        return PDVC_OK;
    }
    hipLaunchKernelGGL(mha_fwd_kernel, dim3((unsigned)blocks), dim3(256), fwd_lds(num_query, head_dim),
                       (hipStream_t)stream, qk, v, key_padding_mask, num_query, num_heads, head_dim, scaling, dropout_p,
                       drop_threshold(dropout_p), seed, seed_dev, qchunks, out, lse);
    PDVC_CHECK_LAUNCH("mha_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_mha_backward_f32(const float* qk, const float* v, const uint8_t* key_padding_mask,
                                     const float* out, const float* grad_out, const float* lse, int batch,
                                     int num_query, int num_heads, int head_dim, float dropout_p, uint64_t seed,
                                     const uint64_t* seed_dev, float* workspace, float* grad_qk, float* grad_v,
                                     void* stream) {
    PDVC_CHECK_ARG(head_dim > 0 && head_dim <= kHD, "query self-attention kernel needs head_dim <= %d, got %d", kHD,
                   head_dim);
    PDVC_CHECK_ARG(num_query > 0 && num_query <= kMaxQ, "num_query must be in [1,%d], got %d", kMaxQ, num_query);
    PDVC_CHECK_ARG(workspace != nullptr, "workspace (pdvc_mha_workspace_floats) is required");
    const int chunks = (num_query + kQB - 1) / kQB;
    const long nm = (long)batch * num_heads;
    if (nm == 0) return PDVC_OK;
    int rc = mha_attrs();
    if (rc) return rc;
    const float scaling = sqrtf(1.0f / (float)head_dim);
    if (use_flash(num_query, head_dim)) {
        const long E = (long)num_heads * head_dim;
        return sq_backward(qk, 2 * E, qk + E, 2 * E, v, E, out, grad_out, lse, batch, num_query, num_query, num_heads,
                           head_dim, scaling, key_padding_mask, dropout_p, seed, seed_dev, workspace, grad_qk, 2 * E,
                           grad_qk + E, 2 * E, grad_v, E, (hipStream_t)stream);
    }
    float* ws_p = workspace;
    float* ws_ds = workspace + (size_t)nm * num_query * num_query;
    hipStream_t s = (hipStream_t)stream;
    if (use_mfma(num_query, head_dim) && bwd_lean()) {
        hipLaunchKernelGGL(mha_bwd_mfma2_kernel, dim3((unsigned)nm), dim3(256), kBwdMfma2Lds, s, qk, v,
                           key_padding_mask, out, grad_out, lse, num_query, num_heads, scaling, dropout_p,
                           drop_threshold(dropout_p), seed, seed_dev, ws_p, ws_ds, grad_qk, grad_v);
        PDVC_CHECK_LAUNCH("mha_bwd_mfma2_kernel");
        return PDVC_OK;
    }
    if (use_mfma(num_query, head_dim)) {
        hipLaunchKernelGGL(mha_bwd_mfma_kernel, dim3((unsigned)nm), dim3(256), kBwdMfmaLds, s, qk, v,
                           key_padding_mask, out, grad_out, lse, num_query, num_heads, scaling, dropout_p,
                           drop_threshold(dropout_p), seed, seed_dev, ws_p, ws_ds, grad_qk, grad_v);
        PDVC_CHECK_LAUNCH("mha_bwd_mfma_kernel");
        return PDVC_OK;
    }
    hipLaunchKernelGGL(mha_bwd_q_kernel, dim3((unsigned)(nm * chunks)), dim3(256), bwdq_lds(num_query, head_dim), s,
                       qk, v, key_padding_mask, out, grad_out, lse, num_query, num_heads, head_dim, scaling, dropout_p,
                       drop_threshold(dropout_p), seed, seed_dev, chunks, ws_p, ws_ds, grad_qk);
    PDVC_CHECK_LAUNCH("mha_bwd_q_kernel");
    hipLaunchKernelGGL(mha_bwd_k_kernel, dim3((unsigned)(nm * chunks)), dim3(256), bwdk_lds(num_query, head_dim), s,
                       qk, grad_out, num_query, num_heads, head_dim, scaling, chunks, ws_p, ws_ds, grad_qk, grad_v);
    PDVC_CHECK_LAUNCH("mha_bwd_k_kernel");
    return PDVC_OK;
}

extern "C" long pdvc_mha_workspace_floats(int batch, int num_query, int num_heads, int head_dim) {
    const long nmq = (long)batch * num_heads * num_query;
    if (use_flash(num_query, head_dim)) return nmq;  // delta rows only
    return 2 * nmq * num_query;                      // P_d and dS tiles of the scalar / single-workgroup kernels
}
