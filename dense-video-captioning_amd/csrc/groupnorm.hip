// groupnorm.hip -- GroupNorm over (video, time, channel) rows for the PDVC base encoder on MI355X.
//
// Replaces nn.GroupNorm(32, d) after each Conv1d of the temporal pyramid (pdvc/base_encoder.py:32-41, applied
// at :63-76), computed on the channels-last layout the transformer consumes, x (N, T, C) row-major: group g is
// the C/G contiguous channels [g*C/G, (g+1)*C/G) of every row of a video, statistics over T*C/G values.  The
// reference layout (N, C, T) cost a transpose copy on both sides of every level.
//
//   stats: per (video, row chunk) a workgroup accumulates (count, mean, M2) per group with Welford updates and
//          Chan merges (lane: one float4 of channels; lanes of one group merge by shuffles, rows through LDS);
//   finalize: per (video, group) merge the chunks -> mean, rstd = 1/sqrt(var + eps) (biased var, as torch);
//   apply: y = (x - mean) * rstd * gamma + beta (float4 streaming).
// backward: dxhat = dy*gamma; per (video, group) s1 = sum dxhat, s2 = sum dxhat*xhat (chunk partials, merged
// like the stats); dx = rstd*(dxhat - (s1 + xhat*s2)/n); dgamma/dbeta column partials per chunk, summed by the
// caller (pdvc_colsum_f32).  All HBM-bound streaming passes.
#include "pdvc_common.h"

namespace pdvc {

constexpr int kGnRows = 64;  // rows per stats chunk

struct Wf {
    float n, mean, m2;
};
__device__ __forceinline__ Wf wf_merge(Wf a, Wf b) {
    const float n = a.n + b.n;
    if (n == 0.f) return a;
    const float d = b.mean - a.mean;
    const float fb = b.n / n;
    Wf r;
    r.n = n;
    r.mean = a.mean + d * fb;
    r.m2 = a.m2 + b.m2 + d * d * a.n * fb;
    return r;
}
__device__ __forceinline__ Wf wf_shfl_xor(Wf a, int d) {
    Wf b;
    b.n = __shfl_xor(a.n, d, PDVC_WAVE);
    b.mean = __shfl_xor(a.mean, d, PDVC_WAVE);
    b.m2 = __shfl_xor(a.m2, d, PDVC_WAVE);
    return b;
}

// grid (N, chunks); block 256 = rpi rows x c4 float4 lanes (c4 = C/4 divides 256).  out: (N, chunks, G) x 3
__global__ __launch_bounds__(256) void gn_stats_kernel(const float* __restrict__ x, int T, int C, int G, int chunks,
                                                       float* __restrict__ part) {
    __shared__ Wf red[256];
    const int c4 = C / 4, rpi = 256 / c4;
    const int cg = threadIdx.x % c4, rr = threadIdx.x / c4;
    const int n = blockIdx.x, ch = blockIdx.y;
    const int r0 = ch * kGnRows, r1 = min(T, r0 + kGnRows);
    Wf w = {0.f, 0.f, 0.f};
    const float4* src = reinterpret_cast<const float4*>(x + (size_t)n * T * C) + cg;
    for (int r = r0 + rr; r < r1; r += rpi) {
        const float4 v = src[(size_t)r * c4];
        const float vals[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // Welford update
            w.n += 1.f;
            const float d = vals[k] - w.mean;
            w.mean += d / w.n;
            w.m2 += d * (vals[k] - w.mean);
        }
    }
    // lanes of one group: cpg4 = (C/G)/4 consecutive float4 lanes (power of two)
    const int cpg4 = (C / G) / 4;
    for (int d = 1; d < cpg4; d <<= 1) w = wf_merge(w, wf_shfl_xor(w, d));
    red[threadIdx.x] = w;
    __syncthreads();
    if (rr == 0 && (cg % cpg4) == 0) {
        for (int k = 1; k < rpi; ++k) w = wf_merge(w, red[k * c4 + cg]);
        const int g = cg / cpg4;
        float* o = part + (((size_t)n * chunks + ch) * G + g) * 3;
        o[0] = w.n;
        o[1] = w.mean;
        o[2] = w.m2;
    }
}

// one thread per (video, group): merge the chunk partials -> mean, rstd
__global__ void gn_finalize_kernel(const float* __restrict__ part, int N, int G, int chunks, float eps,
                                   float* __restrict__ mean, float* __restrict__ rstd) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * G) return;
    const int n = i / G, g = i - n * G;
    Wf w = {0.f, 0.f, 0.f};
    for (int ch = 0; ch < chunks; ++ch) {
        const float* p = part + (((size_t)n * chunks + ch) * G + g) * 3;
        w = wf_merge(w, Wf{p[0], p[1], p[2]});
    }
    mean[i] = w.mean;
    rstd[i] = rsqrtf(w.m2 / w.n + eps);
}

__global__ __launch_bounds__(256) void gn_apply_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int T, int C, int G, int total4,
                                                       float* __restrict__ y, long ys, float* __restrict__ y2) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total4) return;
    const int c4 = C / 4;
    const int row = i / c4;
    const int cg = i - row * c4;
    const int n = row / T;
    const int c = cg * 4;
    const int g = c / (C / G);
    const float mu = mean[n * G + g], rs = rstd[n * G + g];
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    const float4 ga = reinterpret_cast<const float4*>(gamma)[cg], be = reinterpret_cast<const float4*>(beta)[cg];
    float4 o;
    o.x = (v.x - mu) * rs * ga.x + be.x;
    o.y = (v.y - mu) * rs * ga.y + be.y;
    o.z = (v.z - mu) * rs * ga.z + be.z;
    o.w = (v.w - mu) * rs * ga.w + be.w;
    reinterpret_cast<float4*>(y + (size_t)n * ys + (size_t)(row - n * T) * C)[cg] = o;
    if (y2) reinterpret_cast<float4*>(y2)[i] = o;
}

// backward pass 1: per (video, chunk) group sums s1 = sum dy*gamma, s2 = sum dy*gamma*xhat, and per-column
// partials dgamma = sum dy*xhat, dbeta = sum dy over the chunk's rows -> cpart (N*chunks, 2, C)
__global__ __launch_bounds__(256) void gn_bwd_sums_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                          const float* __restrict__ mean, const float* __restrict__ rstd,
                                                          const float* __restrict__ gamma, int T, int C, int G,
                                                          int chunks, long dys, const float* __restrict__ dy2,
                                                          float* __restrict__ gpart,
                                                          float* __restrict__ cpart) {
    __shared__ float4 red_s[256];
    __shared__ float4 red_c[2][256];
    const int c4 = C / 4, rpi = 256 / c4;
    const int cg = threadIdx.x % c4, rr = threadIdx.x / c4;
    const int n = blockIdx.x, ch = blockIdx.y;
    const int r0 = ch * kGnRows, r1 = min(T, r0 + kGnRows);
    const int g = (cg * 4) / (C / G);
    const float mu = mean[n * G + g], rs = rstd[n * G + g];
    const float4 ga = reinterpret_cast<const float4*>(gamma)[cg];
    const float4* xs = reinterpret_cast<const float4*>(x + (size_t)n * T * C) + cg;
    const float4* ds = reinterpret_cast<const float4*>(dy + (size_t)n * dys) + cg;
    const float4* ds2 = dy2 ? reinterpret_cast<const float4*>(dy2 + (size_t)n * T * C) + cg : nullptr;
    float s1 = 0.f, s2 = 0.f;
    float4 dg = make_float4(0.f, 0.f, 0.f, 0.f), db = dg;
    for (int r = r0 + rr; r < r1; r += rpi) {
        const float4 v = xs[(size_t)r * c4];
        float4 d = ds[(size_t)r * c4];
        if (ds2) {
            const float4 e = ds2[(size_t)r * c4];
            d.x += e.x; d.y += e.y; d.z += e.z; d.w += e.w;
        }
        const float h0 = (v.x - mu) * rs, h1 = (v.y - mu) * rs, h2 = (v.z - mu) * rs, h3 = (v.w - mu) * rs;
        s1 += d.x * ga.x + d.y * ga.y + d.z * ga.z + d.w * ga.w;
        s2 += d.x * ga.x * h0 + d.y * ga.y * h1 + d.z * ga.z * h2 + d.w * ga.w * h3;
        dg.x += d.x * h0; dg.y += d.y * h1; dg.z += d.z * h2; dg.w += d.w * h3;
        db.x += d.x; db.y += d.y; db.z += d.z; db.w += d.w;
    }
    const int cpg4 = (C / G) / 4;
    for (int d = 1; d < cpg4; d <<= 1) {
        s1 += __shfl_xor(s1, d, PDVC_WAVE);
        s2 += __shfl_xor(s2, d, PDVC_WAVE);
    }
    red_s[threadIdx.x] = make_float4(s1, s2, 0.f, 0.f);
    red_c[0][threadIdx.x] = dg;
    red_c[1][threadIdx.x] = db;
    __syncthreads();
    if (rr == 0) {
        for (int k = 1; k < rpi; ++k) {
            const float4 a = red_c[0][k * c4 + cg], b = red_c[1][k * c4 + cg];
            dg.x += a.x; dg.y += a.y; dg.z += a.z; dg.w += a.w;
            db.x += b.x; db.y += b.y; db.z += b.z; db.w += b.w;
        }
        float* cp = cpart + ((size_t)n * chunks + ch) * 2 * C;
        reinterpret_cast<float4*>(cp)[cg] = dg;
        reinterpret_cast<float4*>(cp + C)[cg] = db;
        if ((cg % cpg4) == 0) {
            for (int k = 1; k < rpi; ++k) {
                s1 += red_s[k * c4 + cg].x;
                s2 += red_s[k * c4 + cg].y;
            }
            float* o = gpart + (((size_t)n * chunks + ch) * G + g) * 2;
            o[0] = s1;
            o[1] = s2;
        }
    }
}

// backward: merge the chunk sums per (video, group) -> gsum (N, G, 2)
__global__ void gn_bwd_finalize_kernel(const float* __restrict__ gpart, int N, int G, int chunks,
                                       float* __restrict__ gsum) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * G) return;
    const int n = i / G, g = i - n * G;
    float s1 = 0.f, s2 = 0.f;
    for (int ch = 0; ch < chunks; ++ch) {
        const float* p = gpart + (((size_t)n * chunks + ch) * G + g) * 2;
        s1 += p[0];
        s2 += p[1];
    }
    gsum[2 * i] = s1;
    gsum[2 * i + 1] = s2;
}

// backward pass 2: dx = rstd * (dy*gamma - (s1 + xhat*s2) / count)
__global__ __launch_bounds__(256) void gn_bwd_dx_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                        const float* __restrict__ mean, const float* __restrict__ rstd,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ gsum, int T, int C, int G,
                                                        int total4, long dys, const float* __restrict__ dy2,
                                                        float* __restrict__ dx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total4) return;
    const int c4 = C / 4;
    const int row = i / c4;
    const int cg = i - row * c4;
    const int n = row / T;
    const int g = (cg * 4) / (C / G);
    const float s1 = gsum[2 * (n * G + g)], s2 = gsum[2 * (n * G + g) + 1];
    const float inv_n = 1.f / ((float)T * (float)(C / G));
    const float mu = mean[n * G + g], rs = rstd[n * G + g];
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    float4 d = reinterpret_cast<const float4*>(dy + (size_t)n * dys + (size_t)(row - n * T) * C)[cg];
    if (dy2) {
        const float4 e = reinterpret_cast<const float4*>(dy2)[i];
        d.x += e.x; d.y += e.y; d.z += e.z; d.w += e.w;
    }
    const float4 ga = reinterpret_cast<const float4*>(gamma)[cg];
    float4 o;
    o.x = rs * (d.x * ga.x - (s1 + (v.x - mu) * rs * s2) * inv_n);
    o.y = rs * (d.y * ga.y - (s1 + (v.y - mu) * rs * s2) * inv_n);
    o.z = rs * (d.z * ga.z - (s1 + (v.z - mu) * rs * s2) * inv_n);
    o.w = rs * (d.w * ga.w - (s1 + (v.w - mu) * rs * s2) * inv_n);
    reinterpret_cast<float4*>(dx)[i] = o;
}

// Single-pass forms for T <= kGnFRows: one 1024-thread workgroup per (video, 64-channel block) holds the block's
// T x 64 values in registers (64 row slots x 16 float4 lanes, up to 8 rows per thread), so the group statistics
// (forward) and the group sums s1, s2 (backward) come from registers and the pass reads x (and dy) once -- the
// chunked forms above read them twice (stats or sums pass, then the apply or dx pass).  A 64-channel block holds
// whole groups (C/G a power of two <= 64 channels).  The forward's statistics are two-pass over the registers (mean,
// then the sum of squared deviations), the backward's column partials one row per video.
constexpr int kGnFRows = 512;
constexpr int kGnFThreads = 1024;
constexpr int kGnFSlots = kGnFThreads / 16;   // row slots
constexpr int kGnFRpt = kGnFRows / kGnFSlots;  // rows per thread (8)

// sums v over the lanes of a group (cpg4 consecutive float4 lanes of a 16-lane row) and over the 64 row slots; every
// thread gets its group's total.  red: kGnFSlots * 16 floats of LDS; the caller separates two uses by a barrier.
__device__ __forceinline__ float gnf_group_sum(float v, int cpg4, float* red) {
    for (int d = 1; d < cpg4; d <<= 1) v += __shfl_xor(v, d, PDVC_WAVE);
    const int c4l = threadIdx.x & 15, rr = threadIdx.x >> 4;
    red[rr * 16 + c4l] = v;
    __syncthreads();
    if (threadIdx.x < 16) {
        float t = 0.f;
        for (int k = 0; k < kGnFSlots; ++k) t += red[k * 16 + threadIdx.x];
        red[kGnFSlots * 16 + threadIdx.x] = t;
    }
    __syncthreads();
    return red[kGnFSlots * 16 + (c4l & ~(cpg4 - 1))];
}

__global__ __launch_bounds__(kGnFThreads) void gn_fwd_fused_kernel(const float* __restrict__ x, int T, int C, int G,
                                                                    float eps, const float* __restrict__ gamma,
                                                                    const float* __restrict__ beta,
                                                                    float* __restrict__ y, long ys,
                                                                    float* __restrict__ y2, float* __restrict__ mean,
                                                                    float* __restrict__ rstd,
                                                                    uint16_t* __restrict__ y16) {
    __shared__ float red[kGnFSlots * 16 + 16];
    const int n = blockIdx.x, cb = blockIdx.y;
    const int c4l = threadIdx.x & 15, rr = threadIdx.x >> 4;
    const int c4 = C / 4, cg = cb * 16 + c4l;  // this lane's float4 column
    const int cpg4 = (C / G) / 4;
    const float4* xs = reinterpret_cast<const float4*>(x + (size_t)n * T * C) + cg;
    float4 v[kGnFRpt];
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < kGnFRpt; ++k) {
        const int r = rr + k * kGnFSlots;
        v[k] = r < T ? xs[(size_t)r * c4] : make_float4(0.f, 0.f, 0.f, 0.f);
        sm += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    }
    const float cnt = (float)T * (float)(C / G);
    const float mu = gnf_group_sum(sm, cpg4, red) / cnt;
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < kGnFRpt; ++k) {
        if (rr + k * kGnFSlots < T) {
            const float a = v[k].x - mu, b = v[k].y - mu, c = v[k].z - mu, d = v[k].w - mu;
            sq += (a * a + b * b) + (c * c + d * d);
        }
    }
    __syncthreads();  // red reused
    const float rs = rsqrtf(gnf_group_sum(sq, cpg4, red) / cnt + eps);
    if (rr == 0 && (c4l & (cpg4 - 1)) == 0) {
        const int g = (cg * 4) / (C / G);
        mean[n * G + g] = mu;
        rstd[n * G + g] = rs;
    }
    const float4 ga = reinterpret_cast<const float4*>(gamma)[cg], be = reinterpret_cast<const float4*>(beta)[cg];
#pragma unroll
    for (int k = 0; k < kGnFRpt; ++k) {
        const int r = rr + k * kGnFSlots;
        if (r < T) {
            float4 o;
            o.x = (v[k].x - mu) * rs * ga.x + be.x;
            o.y = (v[k].y - mu) * rs * ga.y + be.y;
            o.z = (v[k].z - mu) * rs * ga.z + be.z;
            o.w = (v[k].w - mu) * rs * ga.w + be.w;
            reinterpret_cast<float4*>(y + (size_t)n * ys + (size_t)r * C)[cg] = o;
            if (y2) reinterpret_cast<float4*>(y2 + ((size_t)n * T + r) * C)[cg] = o;
            if (y16) store_bf16x4(y16 + (size_t)n * ys + (size_t)r * C + cg * 4, o.x, o.y, o.z, o.w);
        }
    }
}

// backward: col_partials (N, 2, C) -- per video dgamma = sum dy*xhat, dbeta = sum dy over its rows
__global__ __launch_bounds__(kGnFThreads) void gn_bwd_fused_kernel(const float* __restrict__ x,
                                                                    const float* __restrict__ dy,
                                                                    const float* __restrict__ mean,
                                                                    const float* __restrict__ rstd,
                                                                    const float* __restrict__ gamma, int T, int C,
                                                                    int G, long dys, const float* __restrict__ dy2,
                                                                    float* __restrict__ cpart,
                                                                    float* __restrict__ dx) {
    __shared__ float red[kGnFSlots * 16 + 16];
    __shared__ float4 redc[2][kGnFSlots][16];
    const int n = blockIdx.x, cb = blockIdx.y;
    const int c4l = threadIdx.x & 15, rr = threadIdx.x >> 4;
    const int c4 = C / 4, cg = cb * 16 + c4l;
    const int cpg4 = (C / G) / 4;
    const int g = (cg * 4) / (C / G);
    const float mu = mean[n * G + g], rs = rstd[n * G + g];
    const float4 ga = reinterpret_cast<const float4*>(gamma)[cg];
    const float4* xs = reinterpret_cast<const float4*>(x + (size_t)n * T * C) + cg;
    const float4* ds = reinterpret_cast<const float4*>(dy + (size_t)n * dys) + cg;
    const float4* ds2 = dy2 ? reinterpret_cast<const float4*>(dy2 + (size_t)n * T * C) + cg : nullptr;
    float4 h[kGnFRpt], d[kGnFRpt];
    float s1 = 0.f, s2 = 0.f;
    float4 dg = make_float4(0.f, 0.f, 0.f, 0.f), db = dg;
#pragma unroll
    for (int k = 0; k < kGnFRpt; ++k) {
        const int r = rr + k * kGnFSlots;
        if (r < T) {
            const float4 v = xs[(size_t)r * c4];
            d[k] = ds[(size_t)r * c4];
            if (ds2) {
                const float4 e = ds2[(size_t)r * c4];
                d[k].x += e.x; d[k].y += e.y; d[k].z += e.z; d[k].w += e.w;
            }
            h[k] = make_float4((v.x - mu) * rs, (v.y - mu) * rs, (v.z - mu) * rs, (v.w - mu) * rs);
        } else {
            d[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            h[k] = d[k];
        }
        s1 += d[k].x * ga.x + d[k].y * ga.y + d[k].z * ga.z + d[k].w * ga.w;
        s2 += d[k].x * ga.x * h[k].x + d[k].y * ga.y * h[k].y + d[k].z * ga.z * h[k].z + d[k].w * ga.w * h[k].w;
        dg.x += d[k].x * h[k].x; dg.y += d[k].y * h[k].y; dg.z += d[k].z * h[k].z; dg.w += d[k].w * h[k].w;
        db.x += d[k].x; db.y += d[k].y; db.z += d[k].z; db.w += d[k].w;
    }
    redc[0][rr][c4l] = dg;
    redc[1][rr][c4l] = db;
    s1 = gnf_group_sum(s1, cpg4, red);  // (its barriers also publish redc)
    if (threadIdx.x < 32) {  // the column partials: 16 float4 columns x (dgamma, dbeta)
        const int which = threadIdx.x >> 4, col = threadIdx.x & 15;
        float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int k = 0; k < kGnFSlots; ++k) {
            const float4 a = redc[which][k][col];
            t.x += a.x; t.y += a.y; t.z += a.z; t.w += a.w;
        }
        reinterpret_cast<float4*>(cpart + (size_t)n * 2 * C + (size_t)which * C)[cb * 16 + col] = t;
    }
    __syncthreads();  // red reused
    s2 = gnf_group_sum(s2, cpg4, red);
    const float inv_n = 1.f / ((float)T * (float)(C / G));
#pragma unroll
    for (int k = 0; k < kGnFRpt; ++k) {
        const int r = rr + k * kGnFSlots;
        if (r < T) {
            float4 o;
            o.x = rs * (d[k].x * ga.x - (s1 + h[k].x * s2) * inv_n);
            o.y = rs * (d[k].y * ga.y - (s1 + h[k].y * s2) * inv_n);
            o.z = rs * (d[k].z * ga.z - (s1 + h[k].z * s2) * inv_n);
            o.w = rs * (d[k].w * ga.w - (s1 + h[k].w * s2) * inv_n);
            reinterpret_cast<float4*>(dx + ((size_t)n * T + r) * C)[cg] = o;
        }
    }
}

// whether the single-pass forms serve this shape
static bool gn_fused_ok(int T, int C, int G) {
    static const bool on = [] {
        const char* e = getenv("PDVC_GN_FUSED");  // A/B switch: 0 = the chunked two-pass kernels
        return !(e && e[0] == '0');
    }();
    return on && T <= kGnFRows && C % 64 == 0 && (C / G) <= 64;
}

static int gn_check(int N, int T, int C, int G) {
    PDVC_CHECK_ARG(N >= 0 && T > 0 && C > 0 && G > 0 && C % G == 0, "invalid GroupNorm sizes");
    const int cpg = C / G;
    PDVC_CHECK_ARG(cpg % 4 == 0 && ((cpg / 4) & (cpg / 4 - 1)) == 0 && cpg / 4 <= 64,
                   "channels per group must be 4 x a power of two (got %d)", cpg);
    PDVC_CHECK_ARG(C % 4 == 0 && C / 4 <= 256 && 256 % (C / 4) == 0, "C/4 must divide 256 (got C=%d)", C);
    PDVC_CHECK_ARG((long)N * T * C / 4 < (1L << 31), "tensor too large");
    return PDVC_OK;
}

}  // namespace pdvc

using namespace pdvc;

static int gn_chunks(int T) { return (T + kGnRows - 1) / kGnRows; }

extern "C" int pdvc_groupnorm_rows_forward_out_f32(const float* x, int N, int T, int C, int G, float eps,
                                                   const float* gamma, const float* beta, float* workspace, float* y,
                                                   long y_video_stride, float* y_copy, float* mean, float* rstd,
                                                   void* stream) {
    int rc = gn_check(N, T, C, G);
    if (rc) return rc;
    PDVC_CHECK_ARG(y_video_stride >= (long)T * C && y_video_stride % 4 == 0, "invalid output video stride %ld",
                   y_video_stride);
    if (N == 0) return PDVC_OK;
    hipStream_t s = (hipStream_t)stream;
    const int chunks = gn_chunks(T);
    hipLaunchKernelGGL(gn_stats_kernel, dim3((unsigned)N, (unsigned)chunks), dim3(256), 0, s, x, T, C, G, chunks,
                       workspace);
    PDVC_CHECK_LAUNCH("gn_stats_kernel");
    hipLaunchKernelGGL(gn_finalize_kernel, dim3((unsigned)((N * G + 255) / 256)), dim3(256), 0, s, workspace, N, G,
                       chunks, eps, mean, rstd);
    PDVC_CHECK_LAUNCH("gn_finalize_kernel");
    const int total4 = (int)((long)N * T * C / 4);
    hipLaunchKernelGGL(gn_apply_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, s, x, mean, rstd, gamma,
                       beta, T, C, G, total4, y, y_video_stride, y_copy);
    PDVC_CHECK_LAUNCH("gn_apply_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_groupnorm_rows_forward_f32(const float* x, int N, int T, int C, int G, float eps,
                                               const float* gamma, const float* beta, float* workspace, float* y,
                                               float* mean, float* rstd, void* stream) {
    return pdvc_groupnorm_rows_forward_out_f32(x, N, T, C, G, eps, gamma, beta, workspace, y, (long)T * C, nullptr,
                                               mean, rstd, stream);
}

extern "C" int pdvc_groupnorm_rows_backward_strided_f32(const float* x, const float* dy, long dy_video_stride,
                                                        const float* dy_add, const float* mean, const float* rstd,
                                                        const float* gamma, int N, int T, int C, int G,
                                                        float* group_ws, float* col_partials, float* dx,
                                                        void* stream) {
    int rc = gn_check(N, T, C, G);
    if (rc) return rc;
    PDVC_CHECK_ARG(dy_video_stride >= (long)T * C && dy_video_stride % 4 == 0, "invalid gradient video stride %ld",
                   dy_video_stride);
    if (N == 0) return PDVC_OK;
    hipStream_t s = (hipStream_t)stream;
    const int chunks = gn_chunks(T);
    hipLaunchKernelGGL(gn_bwd_sums_kernel, dim3((unsigned)N, (unsigned)chunks), dim3(256), 0, s, x, dy, mean, rstd,
                       gamma, T, C, G, chunks, dy_video_stride, dy_add, group_ws, col_partials);
    PDVC_CHECK_LAUNCH("gn_bwd_sums_kernel");
    float* gsum = group_ws + (size_t)N * chunks * G * 2;
    hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3((unsigned)((N * G + 255) / 256)), dim3(256), 0, s, group_ws, N, G,
                       chunks, gsum);
    PDVC_CHECK_LAUNCH("gn_bwd_finalize_kernel");
    const int total4 = (int)((long)N * T * C / 4);
    hipLaunchKernelGGL(gn_bwd_dx_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, s, x, dy, mean, rstd,
                       gamma, gsum, T, C, G, total4, dy_video_stride, dy_add, dx);
    PDVC_CHECK_LAUNCH("gn_bwd_dx_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_groupnorm_rows_backward_f32(const float* x, const float* dy, const float* mean, const float* rstd,
                                                const float* gamma, int N, int T, int C, int G, float* group_ws,
                                                float* col_partials, float* dx, void* stream) {
    return pdvc_groupnorm_rows_backward_strided_f32(x, dy, (long)T * C, nullptr, mean, rstd, gamma, N, T, C, G,
                                                    group_ws, col_partials, dx, stream);
}

// Single-pass forms (gn_fwd_fused_kernel / gn_bwd_fused_kernel): T <= 512, C a multiple of 64, C / G <= 64 channels
// per group; any other shape (or PDVC_GN_FUSED=0) returns PDVC_ERR_UNSUPPORTED before launching anything (the caller
// takes the chunked forms).  Forward: as pdvc_groupnorm_rows_forward_out_f32 without a workspace, plus y16 (NULL for
// none): y's bf16 rounding at y's offsets (the bf16 mode's operand of the encoder's first projections).  Backward: as
// pdvc_groupnorm_rows_backward_strided_f32 with col_partials (N, 2, C) -- one row of (dgamma, dbeta) partials per
// video -- and no group workspace.
extern "C" int pdvc_groupnorm_rows_forward_fused_f32(const float* x, int N, int T, int C, int G, float eps,
                                                     const float* gamma, const float* beta, float* y,
                                                     long y_video_stride, float* y_copy, float* mean, float* rstd,
                                                     uint16_t* y16, void* stream) {
    int rc = gn_check(N, T, C, G);
    if (rc) return rc;
    PDVC_CHECK_ARG(y_video_stride >= (long)T * C && y_video_stride % 4 == 0, "invalid output video stride %ld",
                   y_video_stride);
    if (!gn_fused_ok(T, C, G)) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "single-pass GroupNorm: shape not served");
    if (N == 0) return PDVC_OK;
    hipLaunchKernelGGL(gn_fwd_fused_kernel, dim3((unsigned)N, (unsigned)(C / 64)), dim3(kGnFThreads), 0,
                       (hipStream_t)stream, x, T, C, G, eps, gamma, beta, y, y_video_stride, y_copy, mean, rstd,
                       y16);
    PDVC_CHECK_LAUNCH("gn_fwd_fused_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_groupnorm_rows_backward_fused_f32(const float* x, const float* dy, long dy_video_stride,
                                                      const float* dy_add, const float* mean, const float* rstd,
                                                      const float* gamma, int N, int T, int C, int G,
                                                      float* col_partials, float* dx, void* stream) {
    int rc = gn_check(N, T, C, G);
    if (rc) return rc;
    PDVC_CHECK_ARG(dy_video_stride >= (long)T * C && dy_video_stride % 4 == 0, "invalid gradient video stride %ld",
                   dy_video_stride);
    if (!gn_fused_ok(T, C, G)) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "single-pass GroupNorm: shape not served");
    if (N == 0) return PDVC_OK;
    hipLaunchKernelGGL(gn_bwd_fused_kernel, dim3((unsigned)N, (unsigned)(C / 64)), dim3(kGnFThreads), 0,
                       (hipStream_t)stream, x, dy, mean, rstd, gamma, T, C, G, dy_video_stride, dy_add, col_partials,
                       dx);
    PDVC_CHECK_LAUNCH("gn_bwd_fused_kernel");
    return PDVC_OK;
}
