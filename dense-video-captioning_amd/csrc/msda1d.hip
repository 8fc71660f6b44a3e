// msda1d.hip -- fused 1-D multi-scale deformable attention for PDVC on MI355X (gfx950).
//
// Replaces the body of MSDeformAttn.forward between its two projections
// (pdvc/ops/modules/ms_deform_attn.py:167-192): softmax of the attention logits, sampling-location math
// (ref dim 1: loc = ref + off / T_l; ref dim 2: loc = c + off / P * len * 0.5), the 1-D -> 2-D lift
// (y = 0.5, H = 1) and the reference CUDA op (ms_deform_im2col_cuda.cuh:238-300, zero padding).
// PDVC's pyramid is 1-D, so only the two corners on the H=0 row can be in range (for H=1 the CUDA
// kernel's h_im is exactly 0, so lh = 0 and the two lower corners carry weight 0): the kernels read
// exactly those two rows.  Results equal the reference op's float arithmetic up to FMA contraction.
//
// Layout / mapping (MI355X-first):
//   * forward and backward-query: one wave64 per (video, query, group of heads).  A lane owns CPL = 8
//     consecutive channels of one head (two float4 loads per corner: 1 KiB per wave-instruction over
//     8 heads at D = 64), LPH = D / CPL lanes per head.  A (video, query) row of M*D = 512 floats is
//     exactly one wave at PDVC's shape, so the 2 KiB output row is written by one wave.
//   * backward-value: destination-centric.  One workgroup owns a 64-row tile of one (video, head, level)
//     and accumulates its grad_value rows in LDS (ds_add_f32) from every sample whose two corners touch
//     the tile, then writes the tile once with plain stores -- no global float atomics (the reference
//     issues 2 per channel per sample, ~63 MB of atomics per video at T=512, which would cap the kernel
//     at the ~1.3 TB/s atomic rate) and every grad_value element has exactly one writer.
//   * blocks are XCD-remapped so that all blocks of one video run on one XCD and share its L2.
#include <cstdlib>

#include "pdvc_common.h"

namespace pdvc {

constexpr int kNS = 16;   // samples per (query, head) = L * P; PDVC: 4 levels x 4 points
constexpr int kP = 4;     // points per level
constexpr int kL = 4;     // levels

struct Levels1d {
    int T[kL];
    int start[kL];
};

template <int CPL>
__device__ __forceinline__ void load_row(VecF<CPL>& v, const float* __restrict__ p, bool ok) {
    if (ok) v.load(p);
    else v.zero();
}

// select a level's constant without runtime-indexing the (register-resident) struct
__device__ __forceinline__ int lvl_sel(const int (&v)[kL], int l) {
    return l == 0 ? v[0] : l == 1 ? v[1] : l == 2 ? v[2] : v[3];
}

// -------------------------------------------------------------------------------------------------
// forward
// -------------------------------------------------------------------------------------------------
template <int CPL, int LPH, int RD>
__global__ __launch_bounds__(256) void msda1d_fwd_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int D, int waves_per_row, int total_waves, float* __restrict__ out, float* __restrict__ save_attn,
    float* __restrict__ save_loc) {
    constexpr int HPW = 64 / LPH;
    const int lane = threadIdx.x & 63;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int wave = lb * 4 + (threadIdx.x >> 6);
    if (wave >= total_waves) return;
    const int row = wave / waves_per_row;
    const int hg = wave - row * waves_per_row;
    const int b = row / Lq;
    const int sub = lane % LPH;
    const int m = hg * HPW + lane / LPH;
    if (m >= M) return;
    const int c0 = sub * CPL;
    const float* logits = proj + (size_t)row * proj_stride + logit_base + m * kNS;
    const float* offs = proj + (size_t)row * proj_stride + off_base + m * kNS;

    // softmax statistics over the head's L*P logits (ms_deform_attn.py:168-169); weights formed per level
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < kNS; ++j) mx = fmaxf(mx, logits[j]);
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < kNS; ++j) sum += expf(logits[j] - mx);

    const size_t MD = (size_t)M * D;
    const float* vbase = value + (size_t)b * S * MD + (size_t)m * D + c0;
    const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
    VecF<CPL> acc;
    acc.zero();
#pragma unroll 1
    for (int l = 0; l < kL; ++l) {
        const int T = lvl_sel(lv.T, l), st = lvl_sel(lv.start, l);
        const float Tf = (float)T;
        const float r0 = ref[((size_t)row * kL + l) * RD];
        const float r1 = (RD == 2) ? ref[((size_t)row * kL + l) * RD + 1] : 0.f;
        // positions of the level's P points, then all 2*P corner rows loaded together (clamped addresses;
        // out-of-range corners are selected to 0 after the load: no data-dependent branches around loads)
        int i0[kP];
        float lw[kP], aw[kP];
        bool ok1[kP], ok2[kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const int j = l * kP + p;
            aw[p] = expf(logits[j] - mx) / sum;
            const float off = offs[j];
            // ms_deform_attn.py:171-177 (same evaluation order)
            const float loc = (RD == 1) ? r0 + off / Tf : r0 + ((off / (float)kP) * r1) * 0.5f;
            if (save_loc && sub == (j % LPH)) {
                const size_t si = ((size_t)row * M + m) * kNS + j;
                save_loc[si] = loc;
                save_attn[si] = aw[p];
            }
            const float x = loc * Tf - 0.5f;  // w_im (.cuh:284); h_im == 0 for H == 1
            const bool inside = x > -1.f && x < Tf;
            const float xf = floorf(inside ? x : 0.f);
            i0[p] = (int)xf;
            lw[p] = inside ? x - xf : 0.f;
            ok1[p] = inside && i0[p] >= 0;
            ok2[p] = inside && i0[p] + 1 <= T - 1;
        }
        VecF<CPL> v1[kP], v2[kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const int a1 = min(max(i0[p], 0), T - 1), a2 = min(max(i0[p] + 1, 0), T - 1);
            v1[p].load(vbase + (size_t)(st + a1) * MD);
            v2[p].load(vbase + (size_t)(st + a2) * MD);
            if (mbase) {
                ok1[p] = ok1[p] && !mbase[st + a1];
                ok2[p] = ok2[p] && !mbase[st + a2];
            }
        }
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const float hw = 1.f - lw[p];
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const float x1 = ok1[p] ? v1[p].v[c] : 0.f, x2 = ok2[p] ? v2[p].v[c] : 0.f;
                acc.v[c] += (hw * x1 + lw[p] * x2) * aw[p];
            }
        }
    }
    acc.store(out + (size_t)row * MD + (size_t)m * D + c0);
}

// -------------------------------------------------------------------------------------------------
// backward, query side: grad of the offset and attention logits (+ reference points)
// softmax backward uses delta = sum_j a_j dL/da_j = <dL/dout, out> (out = the forward output of this head),
// so every level's samples are finished as soon as they are reduced -- no state carried across levels.
// -------------------------------------------------------------------------------------------------
template <int CPL, int LPH, int RD>
__global__ __launch_bounds__(256) void msda1d_bwd_query_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int D, int waves_per_row, int total_waves, const float* __restrict__ gout, const float* __restrict__ fout,
    const float* __restrict__ save_attn, const float* __restrict__ save_loc, float* __restrict__ grad_proj,
    float* __restrict__ grad_ref) {
    constexpr int HPW = 64 / LPH;
    constexpr int G = LPH < 8 ? LPH : 8;  // reduce-scatter group for the level's 8 partial sums
    constexpr int VPL = 8 / G;            // values per lane after it (interleaved (ga, gs) pairs)
    const int lane = threadIdx.x & 63;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int wave = lb * 4 + (threadIdx.x >> 6);
    if (wave >= total_waves) return;  // wave-uniform
    const int row = wave / waves_per_row;
    const int hg = wave - row * waves_per_row;
    const int b = row / Lq;
    const int sub = lane % LPH;
    const int m_raw = hg * HPW + lane / LPH;
    const bool active = m_raw < M;
    const int m = active ? m_raw : 0;
    const int c0 = sub * CPL;
    const size_t MD = (size_t)M * D;
    const float* vbase = value + (size_t)b * S * MD + (size_t)m * D + c0;
    const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
    const size_t sbase = ((size_t)row * M + m) * kNS;

    VecF<CPL> g, o;
    load_row(g, gout + (size_t)row * MD + (size_t)m * D + c0, active);
    load_row(o, fout + (size_t)row * MD + (size_t)m * D + c0, active);
    float dl = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) dl += g.v[c] * o.v[c];
    const float delta = group_allreduce<LPH>(dl);

    const float* prow = proj + (size_t)row * proj_stride;
    float* gprow = grad_proj + (size_t)row * proj_stride;
#pragma unroll 1
    for (int l = 0; l < kL; ++l) {
        const int T = lvl_sel(lv.T, l), st = lvl_sel(lv.start, l);
        const float Tf = (float)T;
        int i0[kP];
        float lw[kP];
        bool ok1[kP], ok2[kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const float x = (active ? save_loc[sbase + l * kP + p] : 0.f) * Tf - 0.5f;
            const bool inside = active && x > -1.f && x < Tf;
            const float xf = floorf(inside ? x : 0.f);
            i0[p] = (int)xf;
            lw[p] = inside ? x - xf : 0.f;
            ok1[p] = inside && i0[p] >= 0;
            ok2[p] = inside && i0[p] + 1 <= T - 1;
        }
        VecF<CPL> v1[kP], v2[kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {  // all 2*P corner loads in flight together (clamped, selected later)
            const int a1 = min(max(i0[p], 0), T - 1), a2 = min(max(i0[p] + 1, 0), T - 1);
            v1[p].load(vbase + (size_t)(st + a1) * MD);
            v2[p].load(vbase + (size_t)(st + a2) * MD);
            if (mbase) {
                ok1[p] = ok1[p] && !mbase[st + a1];
                ok2[p] = ok2[p] && !mbase[st + a2];
            }
        }
        // part[2p] = sum_c g*val ; part[2p+1] = sum_c g*(v2 - v1) over this lane's channels
        float part[2 * kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const float hw = 1.f - lw[p];
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const float x1 = ok1[p] ? v1[p].v[c] : 0.f, x2 = ok2[p] ? v2[p].v[c] : 0.f;
                s1 += g.v[c] * (hw * x1 + lw[p] * x2);
                s2 += g.v[c] * (x2 - x1);
            }
            part[2 * p] = s1;
            part[2 * p + 1] = s2;
        }
        group_reduce_scatter<2 * kP, G>(part, lane);
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
#pragma unroll
            for (int d = G; d < LPH; d <<= 1) part[k] += __shfl_xor(part[k], d, PDVC_WAVE);
        }
        // group lane r (= sub % G) holds values [r*VPL, (r+1)*VPL) of the interleaved (ga, gs) list
        float ga, gs;
        int p;
        const int r = sub % G;
        if (VPL == 2) {
            p = r;
            ga = part[0];
            gs = part[1];
        } else {
            const float other = __shfl_xor(part[0], 1, PDVC_WAVE);
            p = r >> 1;
            ga = (r & 1) ? other : part[0];
            gs = (r & 1) ? part[0] : other;
        }
        const bool owner = active && sub < G && (VPL == 2 || (r & 1) == 0);
        const int j = l * kP + p;
        const float a = active ? save_attn[sbase + j] : 0.f;
        // CUDA: grad_loc_w = W * grad_w_weight * (top_grad * attn), summed over channels (.cuh:158)
        const float gloc = owner ? Tf * (gs * a) : 0.f;
        float g0 = gloc, g1 = 0.f;
        if (owner) {
            float goff;
            if (RD == 1) {
                goff = gloc / Tf;
            } else {
                const float rr1 = ref[((size_t)row * kL + l) * 2 + 1];
                const float t2 = gloc * 0.5f;
                goff = (t2 * rr1) / (float)kP;
                g1 = t2 * (prow[off_base + m * kNS + j] / (float)kP);
            }
            gprow[off_base + m * kNS + j] = goff;
            gprow[logit_base + m * kNS + j] = a * (ga - delta);
        }
        if (grad_ref) {
            // sum over every head and point of the row (all lanes), then atomics across waves of a row
#pragma unroll
            for (int d = 32; d > 0; d >>= 1) {
                g0 += __shfl_xor(g0, d, PDVC_WAVE);
                if (RD == 2) g1 += __shfl_xor(g1, d, PDVC_WAVE);
            }
            if (lane == 0) {
                float* dst = grad_ref + ((size_t)row * kL + l) * RD;
                if (waves_per_row == 1) {
                    dst[0] = g0;
                    if (RD == 2) dst[1] = g1;
                } else {
                    atomicAdd(dst, g0);
                    if (RD == 2) atomicAdd(dst + 1, g1);
                }
            }
        }
    }
}

// -------------------------------------------------------------------------------------------------
// backward, value side: one workgroup per (video, head, level, channel slice), the level's grad_value
// rows resident in LDS.  Every level receives exactly Lq*P samples per (video, head), so the work per
// workgroup is balanced by construction; each sample is read once, its two corner rows are accumulated
// with ds_add_f32, and the level is written back once with plain stores (one writer per element).
// Lanes: LPS = DC/4 lanes per sample, each owning channels {sub + LPS*k, k < 4} (dword loads coalesced
// over the LPS lanes; consecutive banks for the LDS adds), 64/LPS samples per wave-pass, 4 passes
// unrolled so that 16 gradient loads per lane are in flight.
// -------------------------------------------------------------------------------------------------
struct UnitMap {
    int nunits;              // units per (video, head)
    int level[16];
    int cslice[16];          // channel slice index within the level
    int dc[16];              // channels per slice (16, 32 or 64)
};

template <int ABL>  // diagnostic ablations (0 = the kernel): 1 = plain LDS stores, 2 = no gradient loads
__global__ __launch_bounds__(512) void msda1d_bwd_value_kernel(const uint8_t* __restrict__ vmask, Levels1d lv,
                                                                UnitMap um, int Lq, int S, int M, int D,
                                                                const float* __restrict__ gout,
                                                                const float* __restrict__ save_attn,
                                                                const float* __restrict__ save_loc,
                                                                float* __restrict__ grad_value) {
    extern __shared__ __attribute__((aligned(16))) float acc[];  // [T_l][DC + 1]
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int bm = lb / um.nunits;
    const int unit = lb - bm * um.nunits;
    const int b = bm / M, m = bm - b * M;
    const int l = um.level[unit];
    const int DC = um.dc[unit];
    const int c0 = um.cslice[unit] * DC;
    const int LPS = DC >> 2;         // lanes per sample (4 channels each, strided by LPS)
    const int SPP = 64 / LPS;        // samples per wave-pass
    const int LD = DC + 1;           // padded row: rows of different samples start on different banks
    const int T = lv.T[l], st = lv.start[l];
    const float Tf = (float)T;
    for (int i = threadIdx.x; i < T * LD; i += blockDim.x) acc[i] = 0.f;
    __syncthreads();

    const int sub = lane % LPS;
    const int slot = lane / LPS;
    const int nsamp = Lq * kP;
    const size_t MD = (size_t)M * D;
    const float* gbase = gout + (size_t)b * Lq * MD + (size_t)m * D + c0 + sub;
    const size_t sbase = ((size_t)b * Lq * M + m) * kNS + l * kP;
    // Interleaved assignment: the SPP*nw lanes-groups of one pass take samples nsamp/(SPP*nw) apart, so the
    // samples of one LDS atomic instruction come from distant queries (distinct rows); neighbouring queries
    // sample the same rows and would otherwise serialise on same-address ds_add_f32.
    const int groups = SPP * nw;
    const int gidx = wid * SPP + slot;
    const int per = (nsamp + groups - 1) / groups;
    constexpr int U = 8;  // samples per lane per iteration: 8 loc/attn loads, then 32 gradient loads in flight
    for (int it = 0; it < per; it += U) {
        float loc[U], att[U];
        int qv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int i = gidx * per + it + u;
            const bool ok = (it + u < per) && i < nsamp;
            i = ok ? i : 0;
            const int q = i / kP, p = i - q * kP;
            qv[u] = ok ? q : -1;
            const size_t si = sbase + (size_t)q * M * kNS + p;
            loc[u] = save_loc[si];
            att[u] = save_attn[si];
        }
        float gv[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float* gp = gbase + (size_t)(qv[u] < 0 ? 0 : qv[u]) * MD;
#pragma unroll
            for (int k = 0; k < 4; ++k) gv[u][k] = (ABL == 2) ? 1.f : gp[LPS * k];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float x = loc[u] * Tf - 0.5f;
            if (qv[u] >= 0 && x > -1.f && x < Tf) {
                const float xf = floorf(x);
                const int x0 = (int)xf;
                const float lw = x - xf, hw = 1.f - lw;
                if (x0 >= 0) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (ABL == 1) acc[x0 * LD + sub + LPS * k] = hw * (gv[u][k] * att[u]);
                        else atomicAdd(&acc[x0 * LD + sub + LPS * k], hw * (gv[u][k] * att[u]));
                    }
                }
                if (x0 + 1 <= T - 1) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (ABL == 1) acc[(x0 + 1) * LD + sub + LPS * k] = lw * (gv[u][k] * att[u]);
                        else atomicAdd(&acc[(x0 + 1) * LD + sub + LPS * k], lw * (gv[u][k] * att[u]));
                    }
                }
            }
        }
    }
    __syncthreads();
    const uint8_t* mrow = vmask ? vmask + (size_t)b * S + st : nullptr;
    for (int i = threadIdx.x; i < T * DC; i += blockDim.x) {
        const int r = i / DC, c = i - r * DC;
        const float v = (mrow && mrow[r]) ? 0.f : acc[r * LD + c];
        grad_value[((size_t)b * S + st + r) * MD + (size_t)m * D + c0 + c] = v;
    }
}

// -------------------------------------------------------------------------------------------------
// host side
// -------------------------------------------------------------------------------------------------
static int fill_levels(const int32_t* level_T, int num_levels, int num_point, Levels1d& lv, int& S) {
    PDVC_CHECK_ARG(level_T != nullptr, "level_T must not be NULL");
    if (num_levels != kL || num_point != kP)
        return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "fused 1-D path needs %d levels x %d points (got %d x %d)", kL,
                              kP, num_levels, num_point);
    S = 0;
    for (int l = 0; l < kL; ++l) {
        PDVC_CHECK_ARG(level_T[l] > 0, "level %d has non-positive length %d", l, level_T[l]);
        lv.T[l] = level_T[l];
        lv.start[l] = S;
        S += level_T[l];
    }
    return PDVC_OK;
}

struct Geometry {
    int cpl, lph, hpw, waves_per_row;
};

static int pick_geometry(int M, int D, Geometry& g) {
    // 4 channels (one float4) per lane keeps a level's 2*P corner loads in flight within the register budget
    // of 4 waves/SIMD; D = 128 needs 8 per lane (at most 16 lanes per head).
    if (D == 16 || D == 32 || D == 64) g.cpl = 4;
    else if (D == 128) g.cpl = 8;
    else return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "fused 1-D path supports head_dim 16/32/64/128, got %d", D);
    g.lph = D / g.cpl;
    g.hpw = 64 / g.lph;
    g.waves_per_row = (M + g.hpw - 1) / g.hpw;
    return PDVC_OK;
}

}  // namespace pdvc

using namespace pdvc;

template <int RD>
static void launch_fwd1d(const Geometry& g, dim3 grid, hipStream_t s, const float* value, const uint8_t* mask,
                         const float* proj, int ps, int ob, int lb, const float* ref, Levels1d lv, int Lq, int S,
                         int M, int D, int tw, float* out, float* sa, float* sl) {
#define ARGS value, mask, proj, ps, ob, lb, ref, lv, Lq, S, M, D, g.waves_per_row, tw, out, sa, sl
    if (g.cpl == 8) hipLaunchKernelGGL((msda1d_fwd_kernel<8, 16, RD>), grid, dim3(256), 0, s, ARGS);
    else if (g.lph == 4) hipLaunchKernelGGL((msda1d_fwd_kernel<4, 4, RD>), grid, dim3(256), 0, s, ARGS);
    else if (g.lph == 8) hipLaunchKernelGGL((msda1d_fwd_kernel<4, 8, RD>), grid, dim3(256), 0, s, ARGS);
    else hipLaunchKernelGGL((msda1d_fwd_kernel<4, 16, RD>), grid, dim3(256), 0, s, ARGS);
#undef ARGS
}

template <int RD>
static void launch_bwdq1d(const Geometry& g, dim3 grid, hipStream_t s, const float* value, const uint8_t* mask,
                          const float* proj, int ps, int ob, int lb, const float* ref, Levels1d lv, int Lq, int S,
                          int M, int D, int tw, const float* gout, const float* fout, const float* sa, const float* sl,
                          float* gp, float* gr) {
#define ARGS value, mask, proj, ps, ob, lb, ref, lv, Lq, S, M, D, g.waves_per_row, tw, gout, fout, sa, sl, gp, gr
    if (g.cpl == 8) hipLaunchKernelGGL((msda1d_bwd_query_kernel<8, 16, RD>), grid, dim3(256), 0, s, ARGS);
    else if (g.lph == 4) hipLaunchKernelGGL((msda1d_bwd_query_kernel<4, 4, RD>), grid, dim3(256), 0, s, ARGS);
    else if (g.lph == 8) hipLaunchKernelGGL((msda1d_bwd_query_kernel<4, 8, RD>), grid, dim3(256), 0, s, ARGS);
    else hipLaunchKernelGGL((msda1d_bwd_query_kernel<4, 16, RD>), grid, dim3(256), 0, s, ARGS);
#undef ARGS
}

extern "C" int pdvc_msda1d_forward_f32(const float* value, const uint8_t* value_pad_mask, const float* proj,
                                       int proj_stride, int off_base, int logit_base, const float* ref, int ref_dim,
                                       const int32_t* level_T, int num_levels, int batch, int num_query,
                                       int num_heads, int head_dim, int num_point, float* output, float* save_attn,
                                       float* save_loc, void* stream) {
    Levels1d lv;
    int S = 0;
    int rc = fill_levels(level_T, num_levels, num_point, lv, S);
    if (rc) return rc;
    Geometry g;
    if ((rc = pick_geometry(num_heads, head_dim, g))) return rc;
    PDVC_CHECK_ARG(ref_dim == 1 || ref_dim == 2, "ref_dim must be 1 or 2, got %d", ref_dim);
    PDVC_CHECK_ARG((save_attn == nullptr) == (save_loc == nullptr), "save_attn and save_loc go together");
    PDVC_CHECK_ARG(batch >= 0 && num_query >= 0, "negative sizes");
    const int NSM = num_heads * kNS;
    PDVC_CHECK_ARG(off_base >= 0 && logit_base >= 0 && off_base + NSM <= proj_stride && logit_base + NSM <= proj_stride,
                   "proj columns out of range (stride %d, off %d, logit %d, need %d)", proj_stride, off_base,
                   logit_base, NSM);
    const long rows = (long)batch * num_query;
    const long tw = rows * g.waves_per_row;
    if (tw == 0) return PDVC_OK;
    PDVC_CHECK_ARG(tw < (1L << 31) / 4, "too many rows");
    dim3 grid((unsigned)((tw + 3) / 4));
    hipStream_t s = (hipStream_t)stream;
    if (ref_dim == 1)
        launch_fwd1d<1>(g, grid, s, value, value_pad_mask, proj, proj_stride, off_base, logit_base, ref, lv, num_query,
                        S, num_heads, head_dim, (int)tw, output, save_attn, save_loc);
    else
        launch_fwd1d<2>(g, grid, s, value, value_pad_mask, proj, proj_stride, off_base, logit_base, ref, lv, num_query,
                        S, num_heads, head_dim, (int)tw, output, save_attn, save_loc);
    PDVC_CHECK_LAUNCH("msda1d_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_msda1d_backward_f32(const float* value, const uint8_t* value_pad_mask, const float* ref,
                                        int ref_dim, const float* proj, int proj_stride, int off_base, int logit_base,
                                        const int32_t* level_T, int num_levels, int batch, int num_query,
                                        int num_heads, int head_dim, int num_point, const float* grad_output,
                                        const float* output, const float* save_attn, const float* save_loc,
                                        float* grad_value,
                                        float* grad_proj, float* grad_ref, void* stream) {
    Levels1d lv;
    int S = 0;
    int rc = fill_levels(level_T, num_levels, num_point, lv, S);
    if (rc) return rc;
    Geometry g;
    if ((rc = pick_geometry(num_heads, head_dim, g))) return rc;
    PDVC_CHECK_ARG(ref_dim == 1 || ref_dim == 2, "ref_dim must be 1 or 2, got %d", ref_dim);
    PDVC_CHECK_ARG(save_attn && save_loc && output, "backward needs the forward's output, save_attn and save_loc");
    const int NSM = num_heads * kNS;
    PDVC_CHECK_ARG(off_base >= 0 && logit_base >= 0 && off_base + NSM <= proj_stride && logit_base + NSM <= proj_stride,
                   "proj columns out of range");
    hipStream_t s = (hipStream_t)stream;
    const long rows = (long)batch * num_query;
    const long tw = rows * g.waves_per_row;
    if (grad_ref && g.waves_per_row > 1 && rows > 0) {
        hipError_t e = hipMemsetAsync(grad_ref, 0, sizeof(float) * rows * kL * ref_dim, s);
        if (e != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "memset grad_ref: %s", hipGetErrorString(e));
    }
    if (tw > 0) {
        dim3 grid((unsigned)((tw + 3) / 4));
        if (ref_dim == 1)
            launch_bwdq1d<1>(g, grid, s, value, value_pad_mask, proj, proj_stride, off_base, logit_base, ref, lv,
                             num_query, S, num_heads, head_dim, (int)tw, grad_output, output, save_attn, save_loc,
                             grad_proj, grad_ref);
        else
            launch_bwdq1d<2>(g, grid, s, value, value_pad_mask, proj, proj_stride, off_base, logit_base, ref, lv,
                             num_query, S, num_heads, head_dim, (int)tw, grad_output, output, save_attn, save_loc,
                             grad_proj, grad_ref);
        PDVC_CHECK_LAUNCH("msda1d_bwd_query_kernel");
    }
    // grad_value: one workgroup per (video, head, level, channel slice); slices keep every LDS tile
    // <= ~68 KiB (two 512-thread workgroups per CU) with 16..64 channels per slice
    UnitMap um;
    um.nunits = 0;
    size_t lds = 0;
    for (int l = 0; l < kL; ++l) {
        int dc = head_dim < 64 ? head_dim : 64;
        while ((size_t)lv.T[l] * (dc + 1) * 4 > 68 * 1024 && dc > 16) dc /= 2;
        if (head_dim % dc != 0 || dc % 4 != 0 || (64 % (dc / 4)) != 0)
            return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "head_dim %d cannot be sliced for the value gradient", head_dim);
        const size_t need = sizeof(float) * (size_t)lv.T[l] * (dc + 1);
        if (need > 160 * 1024)
            return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "level %d (T=%d) too long for the LDS value tile", l, lv.T[l]);
        if (need > lds) lds = need;
        for (int c = 0; c < head_dim / dc; ++c) {
            if (um.nunits >= 16) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "too many value-gradient units");
            um.level[um.nunits] = l;
            um.cslice[um.nunits] = c;
            um.dc[um.nunits] = dc;
            ++um.nunits;
        }
    }
    const long nblk = (long)batch * num_heads * um.nunits;
    if (nblk > 0 && num_query > 0) {
        static bool attr = false;
        static int abl = 0;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)msda1d_bwd_value_kernel<0>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            (void)hipFuncSetAttribute((const void*)msda1d_bwd_value_kernel<1>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            (void)hipFuncSetAttribute((const void*)msda1d_bwd_value_kernel<2>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            const char* e = getenv("PDVC_ABLATE_VALUE");  // diagnostics only (timing builds; wrong results)
            abl = e ? atoi(e) : 0;
            attr = true;
        }
        if (abl == 1)
            hipLaunchKernelGGL(msda1d_bwd_value_kernel<1>, dim3((unsigned)nblk), dim3(512), lds, s, value_pad_mask, lv,
                               um, num_query, S, num_heads, head_dim, grad_output, save_attn, save_loc, grad_value);
        else if (abl == 2)
            hipLaunchKernelGGL(msda1d_bwd_value_kernel<2>, dim3((unsigned)nblk), dim3(512), lds, s, value_pad_mask, lv,
                               um, num_query, S, num_heads, head_dim, grad_output, save_attn, save_loc, grad_value);
        else
            hipLaunchKernelGGL(msda1d_bwd_value_kernel<0>, dim3((unsigned)nblk), dim3(512), lds, s, value_pad_mask, lv,
                               um, num_query, S, num_heads, head_dim, grad_output, save_attn, save_loc, grad_value);
        PDVC_CHECK_LAUNCH("msda1d_bwd_value_kernel");
    } else if (nblk > 0) {
        hipError_t e = hipMemsetAsync(grad_value, 0, sizeof(float) * (size_t)batch * S * num_heads * head_dim, s);
        if (e != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "memset grad_value: %s", hipGetErrorString(e));
    }
    return PDVC_OK;
}
