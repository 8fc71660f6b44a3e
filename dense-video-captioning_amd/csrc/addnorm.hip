// addnorm.hip -- y = LayerNorm(x + dropout(s)) fused, forward and backward, for MI355X (gfx950).
//
// The residual epilogue of every transformer sub-layer in PDVC: `norm(src + dropout(src2))`
// (pdvc/deformable_transformer.py:150-156 encoder, :253-271 decoder -- reference lines cited in DESIGN.md).
// Eager PyTorch runs it as dropout (mask + scale), add and LayerNorm forward, then LayerNorm input-grad,
// LayerNorm weight-grad and dropout backward: six passes over a (rows, d) tensor that is 63 MB at the encoder
// shape.  Here: one forward pass (reads x, s; writes y and 8 bytes of statistics per row) and one backward
// pass (reads x, s, dy; writes dx, ds), the dropout mask regenerated from a counter hash of
// (seed, row, column) instead of stored.  One wave per row (d <= 512: <= 8 columns per lane, float4 loads);
// workgroups walk rows with a grid stride so each lane keeps its columns' gamma/beta-gradient partials in
// registers, summed over the workgroup in LDS and over workgroups by a second small kernel.
// The same kernels serve NewModel's front-end (NewModel.py:41-65, `ln(h) + residual`, d = 768): no s term, the
// residual added after the affine (pdvc_layernorm_residual_*).
#include "an_hash.h"
#include "pdvc_common.h"

namespace pdvc {

constexpr int kAND = 768;              // max row width
constexpr int kANW = 4;                // waves per workgroup


__device__ __forceinline__ float an_wave_sum(float v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += lane_swap(v, d);
    return v;
}

// lane's columns: c = lane*4 + 256*k + {0..3}  (float4 chunks, k < kAPL/4)
// s == NULL: no second input (z = x); r != NULL: y = LN(z) * gamma + beta + r
// Row loads of a wave: CH float4 chunks per lane, at clamped (always valid) addresses so that they are unconditional;
// the values of columns >= d and rows >= rows are never used.
template <int CH>
__device__ __forceinline__ void an_load(float4 (&v)[CH], const float* __restrict__ t, int row, int rows, int d,
                                        int lane) {
    const size_t rw = (size_t)min(row, rows - 1);
#pragma unroll
    for (int k = 0; k < CH; ++k) v[k] = *reinterpret_cast<const float4*>(t + rw * d + min(lane * 4 + 256 * k, d - 4));
}

// PF: double-buffered rows -- the next row's loads are issued before this row's reductions, into the other register
// set (two row bodies per loop trip, so that no register copy waits for the loads); gamma and beta held across rows
template <int CH, bool PF>  // float4 chunks per lane
__global__ __launch_bounds__(kANW * 64) void addnorm_fwd_kernel(const float* __restrict__ x, const float* __restrict__ s,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, int rows, int d,
                                                                float p, uint32_t thresh, uint64_t seed0,
                                                                const uint64_t* __restrict__ seed_dev, float eps,
                                                                const float* __restrict__ r,
                                                                float* __restrict__ y, float* __restrict__ mean_out,
                                                                float* __restrict__ rstd_out,
                                                                uint16_t* __restrict__ y16) {
    const int lane = threadIdx.x & 63;
    const uint64_t seed = seed_dev ? *seed_dev : seed0;
    const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
    const float inv_d = 1.f / (float)d;
    float4 gk[CH], bk[CH];
    an_load<CH>(gk, gamma, 0, 1, d, lane);
    an_load<CH>(bk, beta, 0, 1, d, lane);
    auto body = [&](int row, const float4 (&xv4)[CH], const float4 (&sv4)[CH]) {
        float z[CH][4];
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int c = lane * 4 + 256 * k;
            if (c < d) {
                const float4 xv = xv4[k];
                const float4 sv = s ? sv4[k] : make_float4(0.f, 0.f, 0.f, 0.f);
                const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, ss[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float sd = ss[e];
                    if (p > 0.f) sd = an_keep(seed, (uint32_t)row, (uint32_t)(c + e), thresh) ? sd * scale : 0.f;
                    z[k][e] = xs[e] + sd;
                    sum += z[k][e];
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) z[k][e] = 0.f;
            }
        }
        const float mean = an_wave_sum(sum) * inv_d;
        float sq = 0.f;
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int c = lane * 4 + 256 * k;
            if (c < d) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float t = z[k][e] - mean;
                    sq += t * t;
                }
            }
        }
        const float rstd = rsqrtf(an_wave_sum(sq) * inv_d + eps);
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int c = lane * 4 + 256 * k;
            if (c < d) {
                const float4 g = gk[k], b = bk[k];
                float4 o;
                o.x = (z[k][0] - mean) * rstd * g.x + b.x;
                o.y = (z[k][1] - mean) * rstd * g.y + b.y;
                o.z = (z[k][2] - mean) * rstd * g.z + b.z;
                o.w = (z[k][3] - mean) * rstd * g.w + b.w;
                if (r) {
                    const float4 rv = *reinterpret_cast<const float4*>(r + (size_t)row * d + c);
                    o.x += rv.x;
                    o.y += rv.y;
                    o.z += rv.z;
                    o.w += rv.w;
                }
                *reinterpret_cast<float4*>(y + (size_t)row * d + c) = o;
                if (y16) store_bf16x4(y16 + (size_t)row * d + c, o.x, o.y, o.z, o.w);
            }
        }
        if (lane == 0) {
            mean_out[row] = mean;
            rstd_out[row] = rstd;
        }
    };
    const int stride = gridDim.x * kANW;
    const float* sp = s ? s : x;  // s == NULL: the loads read x again (unused), the branch stays uniform
    int row = blockIdx.x * kANW + (threadIdx.x >> 6);
    if constexpr (!PF) {
        for (; row < rows; row += stride) {
            float4 xa[CH], sa[CH];
            an_load<CH>(xa, x, row, rows, d, lane);
            if (s) an_load<CH>(sa, sp, row, rows, d, lane);
            body(row, xa, sa);
        }
    } else {
        float4 xa[CH], sa[CH], xb[CH], sb[CH];
        an_load<CH>(xa, x, row, rows, d, lane);
        if (s) an_load<CH>(sa, sp, row, rows, d, lane);
        for (; row < rows; row += 2 * stride) {
            an_load<CH>(xb, x, row + stride, rows, d, lane);
            if (s) an_load<CH>(sb, sp, row + stride, rows, d, lane);
            body(row, xa, sa);
            if (row + stride >= rows) break;
            an_load<CH>(xa, x, row + 2 * stride, rows, d, lane);
            if (s) an_load<CH>(sa, sp, row + 2 * stride, rows, d, lane);
            body(row + stride, xb, sb);
        }
    }
}

template <int CH, bool PF>
__global__ __launch_bounds__(kANW * 64) void addnorm_bwd_kernel(const float* __restrict__ x, const float* __restrict__ s,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ mean_in,
                                                                const float* __restrict__ rstd_in,
                                                                const float* __restrict__ dy, int rows, int d, float p,
                                                                uint32_t thresh, uint64_t seed0,
                                                                const uint64_t* __restrict__ seed_dev,
                                                                float* __restrict__ dx, float* __restrict__ ds,
                                                                float* __restrict__ dgamma_part,
                                                                float* __restrict__ dbeta_part,
                                                                float* __restrict__ dsum_part,
                                                                uint16_t* __restrict__ ds16) {
    __shared__ float red[3][kANW][kAND];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t seed = seed_dev ? *seed_dev : seed0;
    const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
    const float inv_d = 1.f / (float)d;
    float pg[CH][4], pb[CH][4], pd[CH][4];  // column partials of dgamma, dbeta and (optionally) ds
#pragma unroll
    for (int k = 0; k < CH; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) pg[k][e] = pb[k][e] = pd[k][e] = 0.f;
    float4 gk[CH];
    an_load<CH>(gk, gamma, 0, 1, d, lane);
    auto body = [&](int row, const float4 (&xv4)[CH], const float4 (&sv4)[CH], const float4 (&dv4)[CH], float mean,
                    float rstd) {
        float xh[CH][4], gg[CH][4];
        unsigned keep_bits[CH];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int c = lane * 4 + 256 * k;
            keep_bits[k] = 0xF;
            if (c < d) {
                const float4 xv = xv4[k];
                const float4 sv = s ? sv4[k] : make_float4(0.f, 0.f, 0.f, 0.f);
                const float4 dv = dv4[k];
                const float4 gv = gk[k];
                const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, ss[4] = {sv.x, sv.y, sv.z, sv.w};
                const float dd[4] = {dv.x, dv.y, dv.z, dv.w}, gm[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float sd = ss[e];
                    if (p > 0.f) {
                        const bool kp = an_keep(seed, (uint32_t)row, (uint32_t)(c + e), thresh);
                        if (!kp) keep_bits[k] &= ~(1u << e);
                        sd = kp ? sd * scale : 0.f;
                    }
                    xh[k][e] = (xs[e] + sd - mean) * rstd;
                    gg[k][e] = dd[e] * gm[e];
                    s1 += gg[k][e];
                    s2 += gg[k][e] * xh[k][e];
                    pg[k][e] += dd[e] * xh[k][e];
                    pb[k][e] += dd[e];
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) xh[k][e] = gg[k][e] = 0.f;
            }
        }
        const float m1 = an_wave_sum(s1) * inv_d, m2 = an_wave_sum(s2) * inv_d;
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int c = lane * 4 + 256 * k;
            if (c < d) {
                float o[4], q[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    o[e] = rstd * (gg[k][e] - m1 - xh[k][e] * m2);
                    q[e] = ((keep_bits[k] >> e) & 1u) ? o[e] * scale : 0.f;
                    pd[k][e] += q[e];
                }
                *reinterpret_cast<float4*>(dx + (size_t)row * d + c) = make_float4(o[0], o[1], o[2], o[3]);
                if (ds) *reinterpret_cast<float4*>(ds + (size_t)row * d + c) = make_float4(q[0], q[1], q[2], q[3]);
                if (ds16) store_bf16x4(ds16 + (size_t)row * d + c, q[0], q[1], q[2], q[3]);
            }
        }
    };
    const int stride = gridDim.x * kANW;
    const float* sp = s ? s : x;
    int row = blockIdx.x * kANW + wid;
    auto stats = [&](int rw, float& m, float& rs) {
        const int rc = min(rw, rows - 1);
        m = mean_in[rc];
        rs = rstd_in[rc];
    };
    if constexpr (!PF) {
        for (; row < rows; row += stride) {
            float4 xa[CH], sa[CH], da[CH];
            float ma, ra;
            stats(row, ma, ra);
            an_load<CH>(xa, x, row, rows, d, lane);
            if (s) an_load<CH>(sa, sp, row, rows, d, lane);
            an_load<CH>(da, dy, row, rows, d, lane);
            body(row, xa, sa, da, ma, ra);
        }
    } else {
        float4 xa[CH], sa[CH], da[CH], xb[CH], sb[CH], db[CH];
        float ma, ra, mb, rb;
        stats(row, ma, ra);
        an_load<CH>(xa, x, row, rows, d, lane);
        if (s) an_load<CH>(sa, sp, row, rows, d, lane);
        an_load<CH>(da, dy, row, rows, d, lane);
        for (; row < rows; row += 2 * stride) {
            stats(row + stride, mb, rb);
            an_load<CH>(xb, x, row + stride, rows, d, lane);
            if (s) an_load<CH>(sb, sp, row + stride, rows, d, lane);
            an_load<CH>(db, dy, row + stride, rows, d, lane);
            body(row, xa, sa, da, ma, ra);
            if (row + stride >= rows) break;
            stats(row + 2 * stride, ma, ra);
            an_load<CH>(xa, x, row + 2 * stride, rows, d, lane);
            if (s) an_load<CH>(sa, sp, row + 2 * stride, rows, d, lane);
            an_load<CH>(da, dy, row + 2 * stride, rows, d, lane);
            body(row + stride, xb, sb, db, mb, rb);
        }
    }
    // workgroup sum of the column partials, one row of partials per workgroup
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        const int c = lane * 4 + 256 * k;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (c + e < kAND) {
                red[0][wid][c + e] = pg[k][e];
                red[1][wid][c + e] = pb[k][e];
                red[2][wid][c + e] = pd[k][e];
            }
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < d; c += blockDim.x) {
        float a = 0.f, b = 0.f, e = 0.f;
#pragma unroll
        for (int w = 0; w < kANW; ++w) {
            a += red[0][w][c];
            b += red[1][w][c];
            e += red[2][w][c];
        }
        dgamma_part[(size_t)blockIdx.x * d + c] = a;
        dbeta_part[(size_t)blockIdx.x * d + c] = b;
        if (dsum_part) dsum_part[(size_t)blockIdx.x * d + c] = e;
    }
}

// column sums of the (parts, d) partials -> dgamma, dbeta (and dsum when given): a workgroup per 64 columns,
// 16 float4 column groups x 16 lanes over the partial rows, then a fixed-order LDS sum (bitwise reproducible)
__global__ __launch_bounds__(256) void addnorm_colsum_kernel(const float* __restrict__ gpart,
                                                             const float* __restrict__ bpart,
                                                             const float* __restrict__ spart, int parts, int d,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                             float* __restrict__ dsum) {
    __shared__ float4 red[3][16][16];
    const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int c4 = blockIdx.x * 16 + cg, cs = d / 4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, e = a;
    if (c4 < cs) {
        const float4* g4 = reinterpret_cast<const float4*>(gpart) + c4;
        const float4* b4 = reinterpret_cast<const float4*>(bpart) + c4;
        const float4* s4 = spart ? reinterpret_cast<const float4*>(spart) + c4 : nullptr;
#pragma unroll 4
        for (int i = rl; i < parts; i += 16) {
            const float4 x = g4[(size_t)i * cs], y = b4[(size_t)i * cs];
            a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
            b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
            if (s4) {
                const float4 z = s4[(size_t)i * cs];
                e.x += z.x; e.y += z.y; e.z += z.z; e.w += z.w;
            }
        }
    }
    red[0][rl][cg] = a;
    red[1][rl][cg] = b;
    red[2][rl][cg] = e;
    __syncthreads();
    if (rl < 3 && c4 < cs && (rl < 2 || dsum)) {
        float4 t = red[rl][0][cg];
#pragma unroll
        for (int k = 1; k < 16; ++k) {
            t.x += red[rl][k][cg].x;
            t.y += red[rl][k][cg].y;
            t.z += red[rl][k][cg].z;
            t.w += red[rl][k][cg].w;
        }
        float* dst = rl == 0 ? dgamma : (rl == 1 ? dbeta : dsum);
        dst[c4 * 4 + 0] = t.x;
        dst[c4 * 4 + 1] = t.y;
        dst[c4 * 4 + 2] = t.z;
        dst[c4 * 4 + 3] = t.w;
    }
}


static int an_grid(int rows, int cap) {
    const int want = (rows + kANW - 1) / kANW;
    return want < cap ? (want > 0 ? want : 1) : cap;
}
constexpr int kAnFwdBlocks = 1024;  // 4 per CU
constexpr int kAnBwdBlocks = 1024;  // 4 per CU (16 waves): enough loads in flight to stream at HBM rate

static bool an_pf() {  // PDVC_AN_PF=0: the kernels without the next-row prefetch (same-box A/B)
    static const bool on = [] {
        const char* e = getenv("PDVC_AN_PF");
        return !(e && e[0] == '0');
    }();
    return on;
}

static int an_forward(const float* x, const float* s, const float* r, const float* gamma, const float* beta, int rows,
                      int d, float p, uint64_t seed, const uint64_t* seed_dev, float eps, float* y, float* mean,
                      float* rstd, void* stream, uint16_t* y16 = nullptr) {
    const dim3 grid((unsigned)an_grid(rows, kAnFwdBlocks)), block(kANW * 64);
    hipStream_t st = (hipStream_t)stream;
    const uint32_t th = an_threshold(p);
#define AN_FWD(CH)                                                                                                  \
    do {                                                                                                            \
        auto kern = an_pf() ? addnorm_fwd_kernel<CH, true> : addnorm_fwd_kernel<CH, false>;                         \
        hipLaunchKernelGGL(kern, grid, block, 0, st, x, s, gamma, beta, rows, d, p, th, seed, seed_dev, eps, r, y,  \
                           mean, rstd, y16);                                                                        \
    } while (0)
    if (d <= 256) AN_FWD(1);
    else if (d <= 512) AN_FWD(2);
    else AN_FWD(3);
#undef AN_FWD
    PDVC_CHECK_LAUNCH("addnorm_fwd_kernel");
    return PDVC_OK;
}

static int an_backward(const float* x, const float* s, const float* gamma, const float* mean, const float* rstd,
                       const float* dy, int rows, int d, float p, uint64_t seed, const uint64_t* seed_dev, float* dx,
                       float* ds, float* dgamma, float* dbeta, float* ds_colsum, float* workspace, hipStream_t st,
                       uint16_t* ds16 = nullptr) {
    const int parts = an_grid(rows, kAnBwdBlocks);
    float* gpart = workspace;
    float* bpart = workspace + (size_t)parts * d;
    float* spart = ds_colsum ? workspace + 2 * (size_t)parts * d : nullptr;
    const dim3 grid((unsigned)parts), block(kANW * 64);
    const uint32_t th = an_threshold(p);
#define AN_BWD(CH)                                                                                                  \
    do {                                                                                                            \
        auto kern = an_pf() ? addnorm_bwd_kernel<CH, true> : addnorm_bwd_kernel<CH, false>;                         \
        hipLaunchKernelGGL(kern, grid, block, 0, st, x, s, gamma, mean, rstd, dy, rows, d, p, th, seed, seed_dev,   \
                           dx, ds, gpart, bpart, spart, ds16);                                                      \
    } while (0)
    if (d <= 256) AN_BWD(1);
    else if (d <= 512) AN_BWD(2);
    else AN_BWD(3);
#undef AN_BWD
    PDVC_CHECK_LAUNCH("addnorm_bwd_kernel");
    hipLaunchKernelGGL(addnorm_colsum_kernel, dim3((unsigned)((d / 4 + 15) / 16)), dim3(256), 0, st, gpart, bpart, spart,
                       parts, d, dgamma, dbeta, ds_colsum);
    PDVC_CHECK_LAUNCH("addnorm_colsum_kernel");
    return PDVC_OK;
}

}  // namespace pdvc

using namespace pdvc;

#define AN_CHECK()                                                                                            \
    PDVC_CHECK_ARG(rows >= 0 && d > 0 && d <= kAND && d % 4 == 0, "add-norm needs 0 < d <= %d, d %% 4 == 0", \
                   kAND);                                                                                      \
    PDVC_CHECK_ARG(p >= 0.f && p < 1.f, "dropout p must be in [0, 1)")

extern "C" int pdvc_add_dropout_layernorm_forward_f32(const float* x, const float* s, const float* gamma,
                                                      const float* beta, int rows, int d, float p, uint64_t seed,
                                                      const uint64_t* seed_dev, float eps, float* y, float* mean,
                                                      float* rstd, void* stream) {
    AN_CHECK();
    if (rows == 0) return PDVC_OK;
    return an_forward(x, s, nullptr, gamma, beta, rows, d, p, seed, seed_dev, eps, y, mean, rstd, stream);
}

extern "C" int pdvc_add_dropout_layernorm_backward_f32(const float* x, const float* s, const float* gamma,
                                                       const float* mean, const float* rstd, const float* dy, int rows,
                                                       int d, float p, uint64_t seed, const uint64_t* seed_dev,
                                                       float* dx, float* ds, float* dgamma, float* dbeta,
                                                       float* ds_colsum, float* workspace, void* stream) {
    AN_CHECK();
    PDVC_CHECK_ARG(workspace != nullptr, "workspace (3 * 1024 * d floats) is required");
    hipStream_t st = (hipStream_t)stream;
    if (rows == 0) {
        hipError_t e1 = zero_async(dgamma, d, st);
        hipError_t e2 = zero_async(dbeta, d, st);
        hipError_t e3 = ds_colsum ? zero_async(ds_colsum, d, st) : hipSuccess;
        if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess)
            return pdvc_set_error(PDVC_ERR_LAUNCH, "memset failed");
        return PDVC_OK;
    }
    return an_backward(x, s, gamma, mean, rstd, dy, rows, d, p, seed, seed_dev, dx, ds, dgamma, dbeta, ds_colsum,
                       workspace, st);
}

// The bf16 mode's forms (pdvc/precision.py): the same passes, also writing the bf16 rounding (RNE, torch's cast)
// of y / ds into y16 / ds16 -- the operand the next GEMM reads -- so no separate cast pass reads y / ds again.
extern "C" int pdvc_add_dropout_layernorm_forward_f32_bf16out(const float* x, const float* s, const float* gamma,
                                                              const float* beta, int rows, int d, float p,
                                                              uint64_t seed, const uint64_t* seed_dev, float eps,
                                                              float* y, float* mean, float* rstd, uint16_t* y16,
                                                              void* stream) {
    AN_CHECK();
    PDVC_CHECK_ARG(y16 != nullptr && ((uintptr_t)y16 % 8) == 0, "y16 must be an 8-byte aligned bf16 buffer");
    if (rows == 0) return PDVC_OK;
    return an_forward(x, s, nullptr, gamma, beta, rows, d, p, seed, seed_dev, eps, y, mean, rstd, stream, y16);
}

extern "C" int pdvc_add_dropout_layernorm_backward_f32_bf16out(const float* x, const float* s, const float* gamma,
                                                               const float* mean, const float* rstd, const float* dy,
                                                               int rows, int d, float p, uint64_t seed,
                                                               const uint64_t* seed_dev, float* dx, float* ds,
                                                               float* dgamma, float* dbeta, float* ds_colsum,
                                                               float* workspace, uint16_t* ds16, void* stream) {
    AN_CHECK();
    PDVC_CHECK_ARG(workspace != nullptr, "workspace (3 * 1024 * d floats) is required");
    PDVC_CHECK_ARG(ds != nullptr && ds16 != nullptr && ((uintptr_t)ds16 % 8) == 0,
                   "ds16 must be an 8-byte aligned bf16 buffer beside ds");
    if (rows == 0)
        return pdvc_add_dropout_layernorm_backward_f32(x, s, gamma, mean, rstd, dy, rows, d, p, seed, seed_dev, dx, ds,
                                                       dgamma, dbeta, ds_colsum, workspace, stream);
    return an_backward(x, s, gamma, mean, rstd, dy, rows, d, p, seed, seed_dev, dx, ds, dgamma, dbeta, ds_colsum,
                       workspace, (hipStream_t)stream, ds16);
}

extern "C" int pdvc_layernorm_residual_forward_f32(const float* x, const float* r, const float* gamma,
                                                   const float* beta, int rows, int d, float eps, float* y, float* mean,
                                                   float* rstd, void* stream) {
    const float p = 0.f;
    AN_CHECK();
    if (rows == 0) return PDVC_OK;
    return an_forward(x, nullptr, r, gamma, beta, rows, d, 0.f, 0, nullptr, eps, y, mean, rstd, stream);
}

extern "C" int pdvc_layernorm_backward_f32(const float* x, const float* gamma, const float* mean, const float* rstd,
                                           const float* dy, int rows, int d, float* dx, float* dgamma, float* dbeta,
                                           float* workspace, void* stream) {
    const float p = 0.f;
    AN_CHECK();
    PDVC_CHECK_ARG(workspace != nullptr, "workspace (2 * 1024 * d floats) is required");
    hipStream_t st = (hipStream_t)stream;
    if (rows == 0) {
        hipError_t e1 = zero_async(dgamma, d, st);
        hipError_t e2 = zero_async(dbeta, d, st);
        if (e1 != hipSuccess || e2 != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "memset failed");
        return PDVC_OK;
    }
    return an_backward(x, nullptr, gamma, mean, rstd, dy, rows, d, 0.f, 0, nullptr, dx, nullptr, dgamma, dbeta,
                       nullptr, workspace, st);
}
