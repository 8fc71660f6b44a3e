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
//   * backward-value: destination-centric.  One workgroup per (video, head, level) builds an inverted index
//     of its samples in LDS (bucketed by floor of the sampling position) and sums, per grad_value row,
//     the contributions of exactly the samples whose corners touch it -- no float atomics at all (the
//     reference issues 2 global atomics per channel per sample, ~63 MB of atomics per video at T=512,
//     which would cap the kernel at the ~1.3 TB/s atomic rate) and every grad_value element has
//     exactly one writer.
//   * blocks are XCD-remapped so that all blocks of one video run on one XCD and share its L2.
#include <cstdlib>
#include <type_traits>

#include "pdvc_common.h"

namespace pdvc {

constexpr int kNS = 16;  // samples per (query, head) = L * P; PDVC: 4 levels x 4 points
constexpr int kP = 4;     // points per level
constexpr int kL = kL1d;  // levels (Levels1d, pdvc_common.h)

// save_attn / save_loc (written by the forward, read by both backward kernels): level-major (N, M, L, Lq, P), so
// the value-gradient workgroup of one (video, head, level) reads its samples as one contiguous slab, and the
// query side reads a wave's 4 consecutive queries of a level as one 64-B piece.
__device__ __forceinline__ size_t save_index(int b, int m, int l, int q, int p, int Lq, int M) {
    return ((((size_t)b * M + m) * kL + l) * Lq + q) * kP + p;
}

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
// Mapping shared by the forward and the query-side backward: one wave = QPW = 64/LPH consecutive queries of
// ONE (video, head); a workgroup = 4 waves = 4*QPW consecutive queries of that head.  Consecutive encoder
// queries are neighbouring positions of one level, so a workgroup's samples fall in a narrow window of every
// level: its value rows (256 B per head and position) are re-read from L1 instead of L2.  Within a lane
// group (LPH lanes = one query), lane `sub` owns samples j = sub + LPH*k for the parameter phase (coalesced
// logits/offsets, softmax by group shuffles) and hands each sample's row and corner weights to the group by
// shuffles for the gather phase, which is unrolled over the 16 samples with a scheduling barrier per level
// (each level's 2*P corner loads in flight together, no cross-level hoisting).
// -------------------------------------------------------------------------------------------------
template <int LPH>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
    for (int d = 1; d < LPH; d <<= 1) v = fmaxf(v, lane_swap(v, d));
    return v;
}

struct WaveQuery {
    int b, m, q, row, sub, gbase;
    bool active;
};

template <int LPH>
__device__ __forceinline__ WaveQuery wave_query(int wave, int lane, int Lq, int M) {
    constexpr int QPW = 64 / LPH;
    const int qg_per = (Lq + QPW - 1) / QPW;
    const int bm = wave / qg_per;
    const int qg = wave - bm * qg_per;
    WaveQuery w;
    w.b = bm / M;
    w.m = bm - w.b * M;
    const int q = qg * QPW + lane / LPH;
    w.active = q < Lq;
    w.q = w.active ? q : Lq - 1;
    w.row = w.b * Lq + w.q;
    w.sub = lane % LPH;
    w.gbase = lane - w.sub;
    return w;
}

// forward
template <int CPL, int LPH, int RD>
__global__ __launch_bounds__(256) void msda1d_fwd_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int D, int total_waves, float* __restrict__ out, float* __restrict__ save_attn,
    float* __restrict__ save_loc) {
    constexpr int JPL = kNS / LPH;  // samples owned per lane in the parameter phase
    const int lane = threadIdx.x & 63;
    const int wave = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
    if (wave >= total_waves) return;  // wave-uniform
    const WaveQuery w = wave_query<LPH>(wave, lane, Lq, M);
    const size_t MD = (size_t)M * D;
    const uint8_t* mbase = vmask ? vmask + (size_t)w.b * S : nullptr;
    const float* prow = proj + (size_t)w.row * proj_stride;

    // parameter phase (ms_deform_attn.py:168-177, same evaluation order): softmax weight, location, corner
    // row and the two corner weights (0 where the reference skips the corner or the row is padding)
    float lg[JPL], mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < JPL; ++k) {
        lg[k] = prow[logit_base + w.m * kNS + w.sub + LPH * k];
        mx = fmaxf(mx, lg[k]);
    }
    mx = group_max<LPH>(mx);
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < JPL; ++k) sum += expf(lg[k] - mx);
    sum = group_allreduce<LPH>(sum);
    int i0v[JPL];
    float w1v[JPL], w2v[JPL];
#pragma unroll
    for (int k = 0; k < JPL; ++k) {
        const int j = w.sub + LPH * k;
        const int l = j / kP;
        const int T = lvl_sel(lv.T, l), st = lvl_sel(lv.start, l);
        const float Tf = (float)T;
        const float aw = expf(lg[k] - mx) / sum;
        const float off = prow[off_base + w.m * kNS + j];
        const float r0 = ref[((size_t)w.row * kL + l) * RD];
        const float r1 = (RD == 2) ? ref[((size_t)w.row * kL + l) * RD + 1] : 0.f;
        const float loc = (RD == 1) ? r0 + off / Tf : r0 + ((off / (float)kP) * r1) * 0.5f;
        if (save_loc && w.active) {
            const size_t si = save_index(w.b, w.m, l, w.q, j % kP, Lq, M);
            save_loc[si] = loc;
            save_attn[si] = aw;
        }
        const float x = loc * Tf - 0.5f;  // w_im (.cuh:284); h_im == 0 for H == 1
        const bool inside = x > -1.f && x < Tf;
        const float xf = floorf(inside ? x : 0.f);
        const int i0 = (int)xf;
        const float lw = inside ? x - xf : 0.f;
        bool ok1 = inside && i0 >= 0, ok2 = inside && i0 + 1 <= T - 1;
        if (mbase) {
            ok1 = ok1 && !mbase[st + min(max(i0, 0), T - 1)];
            ok2 = ok2 && !mbase[st + min(max(i0 + 1, 0), T - 1)];
        }
        i0v[k] = i0;
        w1v[k] = ok1 ? (1.f - lw) * aw : 0.f;
        w2v[k] = ok2 ? lw * aw : 0.f;
    }

    const float* vbase = value + (size_t)w.b * S * MD + (size_t)w.m * D + w.sub * CPL;
    VecF<CPL> acc;
    acc.zero();
#pragma unroll
    for (int l = 0; l < kL; ++l) {
        const int T = lv.T[l], st = lv.start[l];
        VecF<CPL> v1[kP], v2[kP];
        float c1[kP], c2[kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const int j = l * kP + p;
            const int i0 = grp_bcast<LPH>(i0v[j / LPH], j % LPH);
            c1[p] = grp_bcast<LPH>(w1v[j / LPH], j % LPH);
            c2[p] = grp_bcast<LPH>(w2v[j / LPH], j % LPH);
            const int a1 = min(max(i0, 0), T - 1), a2 = min(max(i0 + 1, 0), T - 1);
            v1[p].load(vbase + (size_t)(st + a1) * MD);
            v2[p].load(vbase + (size_t)(st + a2) * MD);
        }
#pragma unroll
        for (int p = 0; p < kP; ++p) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) acc.v[c] += c1[p] * v1[p].v[c] + c2[p] * v2[p].v[c];
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (w.active) acc.store(out + (size_t)w.row * MD + (size_t)w.m * D + w.sub * CPL);
}

// -------------------------------------------------------------------------------------------------
// Forward at D = 64 with buffer loads (the query-side mapping of msda1d_bwd_query_dot_kernel): a lane owns one
// sample of its query (j = lane % 16) for the parameter phase, and the group gathers the sample's two corner rows
// through the broadcast row offset and corner weights.  The per-lane clamping and 64-bit address arithmetic of
// msda1d_fwd_kernel are replaced by one 32-bit offset per sample and the descriptor's range check (a corner outside
// its level reads a finite neighbouring row or zeros, and its weight is 0, as in the reference's skipped corner).
// Same parameter math, same accumulation order as msda1d_fwd_kernel: the same bits.
// -------------------------------------------------------------------------------------------------
template <int RD>
__global__ __launch_bounds__(256) void msda1d_fwd_buf_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int total_waves, float* __restrict__ out, float* __restrict__ save_attn, float* __restrict__ save_loc) {
    constexpr int D = 64;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
    if (wave >= total_waves) return;
    const WaveQuery w = wave_query<16>(wave, lane, Lq, M);
    const int MD = M * D;
    const int j = w.sub, l_own = j >> 2;
    int T_own = lv.T[0], st_own = lv.start[0];
#pragma unroll
    for (int l = 1; l < kL; ++l) {
        T_own = l_own >= l ? lv.T[l] : T_own;
        st_own = l_own >= l ? lv.start[l] : st_own;
    }
    const float Tf = (float)T_own;
    const float* prow = proj + (size_t)w.row * proj_stride;
    const float lg = prow[logit_base + w.m * kNS + j];
    const float off = prow[off_base + w.m * kNS + j];
    const float r0 = ref[((size_t)w.row * kL + l_own) * RD];
    const float r1 = (RD == 2) ? ref[((size_t)w.row * kL + l_own) * RD + 1] : 0.f;
    const float mx = group_max<16>(lg);
    const float sum = group_allreduce<16>(expf(lg - mx));
    const float aw = expf(lg - mx) / sum;
    const float loc = (RD == 1) ? r0 + off / Tf : r0 + ((off / (float)kP) * r1) * 0.5f;
    if (save_loc && w.active) {
        const size_t si = save_index(w.b, w.m, l_own, w.q, j & 3, Lq, M);
        save_loc[si] = loc;
        save_attn[si] = aw;
    }
    const float x = loc * Tf - 0.5f;
    const bool inside = x > -1.f && x < Tf;
    const float xf = floorf(inside ? x : 0.f);
    const int i0 = (int)xf;
    const float lw = inside ? x - xf : 0.f;
    bool ok1 = inside && i0 >= 0, ok2 = inside && i0 + 1 <= T_own - 1;
    if (vmask) {
        const uint8_t* mb = vmask + (size_t)w.b * S + st_own;
        ok1 = ok1 && !mb[min(max(i0, 0), T_own - 1)];
        ok2 = ok2 && !mb[min(max(i0 + 1, 0), T_own - 1)];
    }
    const float w1 = ok1 ? (1.f - lw) * aw : 0.f, w2 = ok2 ? lw * aw : 0.f;
    const int roff = (st_own + i0) * (MD * 4);
    const int coff = (w.m * D + w.sub * 4) * 4;
    const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(  // scalar: one video per wave
        (void*)(value + (size_t)__builtin_amdgcn_readfirstlane(w.b) * S * MD), (short)0, S * MD * 4, 0x00020000);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int l = 0; l < kL; ++l) {
        // the level's broadcasts and loads depend (opaquely) on all four of the previous level's sums, so the compiler
        // can neither hoist them nor defer the previous level's FMAs: one level's 8 corner loads live at a time
        // (hoisting all 32 took 200 VGPRs; a dependency on acc.x alone, 127)
        int rl = roff;
        float wl1 = w1, wl2 = w2;
        __asm__ volatile("" : "+v"(rl), "+v"(wl1), "+v"(wl2) : "v"(acc.x), "v"(acc.y), "v"(acc.z), "v"(acc.w));
        float4 v1[kP], v2[kP];
        float c1[kP], c2[kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const int o = grp_bcast<16>(rl, l * kP + p) + coff;
            c1[p] = grp_bcast<16>(wl1, l * kP + p);
            c2[p] = grp_bcast<16>(wl2, l * kP + p);
            const auto u1 = __builtin_amdgcn_raw_buffer_load_b128(vr, o, 0, 0);
            const auto u2 = __builtin_amdgcn_raw_buffer_load_b128(vr, o + MD * 4, 0, 0);
            v1[p] = make_float4(__uint_as_float(u1[0]), __uint_as_float(u1[1]), __uint_as_float(u1[2]),
                                __uint_as_float(u1[3]));
            v2[p] = make_float4(__uint_as_float(u2[0]), __uint_as_float(u2[1]), __uint_as_float(u2[2]),
                                __uint_as_float(u2[3]));
        }
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            acc.x += c1[p] * v1[p].x + c2[p] * v2[p].x;
            acc.y += c1[p] * v1[p].y + c2[p] * v2[p].y;
            acc.z += c1[p] * v1[p].z + c2[p] * v2[p].z;
            acc.w += c1[p] * v1[p].w + c2[p] * v2[p].w;
        }
    }
    if (w.active)
        *reinterpret_cast<float4*>(out + (size_t)w.row * MD + (size_t)w.m * D + w.sub * 4) = acc;
}

// -------------------------------------------------------------------------------------------------
// Whole-pyramid forward for the encoder's self-attention (Lq ~ S queries per (video, head)), D = 64.
// A 1024-thread workgroup takes one (video, head) and a block of up to 512 queries (16 lanes per query, 8
// queries per lane group).  The head's value rows (256 B per position) are staged in LDS level by level --
// level 0 (T_0 <= 512 rows, 128 KiB), then levels 1..3 together -- with coalesced float4 loads, and every
// corner row is gathered from LDS.  The value slice is read from HBM once per query block (twice per head at
// S = 960) instead of ~20 times through L1/L2: 0.79x the per-query kernel's time at 256 videos (tools/kbench.py).
// Parameter phase, corner clamping and accumulation order are msda1d_fwd_kernel's at LPH = 16: the same bits.
// (A backward-query twin, holding dOut slices for 4 queries per lane group, spilled and ran 2x slower than
// msda1d_bwd_query_kernel; the backward keeps the per-query mapping.)
// -------------------------------------------------------------------------------------------------
constexpr int kPyrThreads = 1024;
constexpr int kPyrQPS = 8;                                  // queries per 16-lane group
constexpr int kPyrQ = (kPyrThreads / 16) * kPyrQPS;        // 512 queries per workgroup
constexpr int kPyrRows = 512;                               // data rows per staging phase (256 B each): 128 KiB
constexpr int kPyrRowsG = kPyrRows + 2;                     // + a guard row at each end
constexpr size_t kPyrLds = (size_t)kPyrRowsG * 64 * sizeof(float);

// Guarded LDS layout of the whole-pyramid kernels: row 0 is a zero guard, a phase's data rows follow from row 1
// (level 0 alone; then levels 1..3 packed back to back), and one zero guard row closes them.  A sample's corner
// rows x0 and x0 + 1 with x0 in [-1, T - 1] (every sample inside the level's open interval) are then always rows
// of the buffer -- a guard, or a neighbouring level's row -- so the kernels read them without clamping: a corner
// outside its level carries weight 0 and the row it reads is finite.  (The clamps were 536 of the forward's
// ~3 800 VALU instructions per wave.)

// stage rows [r0, r0 + n) of one head (vsrc = value + b*S*MD + m*64) into LDS rows [1, n + 1), zero rows 0 and n + 1
__device__ __forceinline__ void pyr_stage_g(float4* __restrict__ lds, const float* __restrict__ vsrc, size_t MD,
                                            int r0, int n) {
    const float4* src = reinterpret_cast<const float4*>(vsrc);
    const size_t rs = MD / 4;
    const int total = n * 16;
#pragma unroll 4
    for (int i = threadIdx.x; i < total; i += kPyrThreads) lds[(size_t)(1 + (i >> 4)) * 16 + (i & 15)] =
        src[(size_t)(r0 + (i >> 4)) * rs + (i & 15)];
    if (threadIdx.x < 32) {
        const int row = threadIdx.x < 16 ? 0 : n + 1;
        lds[row * 16 + (threadIdx.x & 15)] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// pyr_stage_g with 2 loads in flight per thread (used while the parameter loads hold registers)
__device__ __forceinline__ void pyr_stage_g_lean(float4* __restrict__ lds, const float* __restrict__ vsrc, size_t MD,
                                                 int r0, int n) {
    const float4* src = reinterpret_cast<const float4*>(vsrc);
    const size_t rs = MD / 4;
    const int total = n * 16;
#pragma unroll 2
    for (int i = threadIdx.x; i < total; i += kPyrThreads) lds[(size_t)(1 + (i >> 4)) * 16 + (i & 15)] =
        src[(size_t)(r0 + (i >> 4)) * rs + (i & 15)];
    if (threadIdx.x < 32) {
        const int row = threadIdx.x < 16 ? 0 : n + 1;
        lds[row * 16 + (threadIdx.x & 15)] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// LDS row of level l's first position in its phase (guarded layout): level 0 alone, then levels 1..3 packed
__device__ __forceinline__ int pyr_base(const Levels1d& lv, int l) {
    return l <= 1 ? 1 : (l == 2 ? 1 + lv.T[1] : 1 + lv.T[1] + lv.T[2]);
}

// Per-sample LDS byte offset of corner row x0 (x0 in [-1, T-1] for a sample inside its level, 0 otherwise) in the
// guarded layout; the corner x0 + 1 is the next row (+256 B, a ds_read immediate)
__device__ __forceinline__ int pyr_corner(int base, int i0) { return (base + i0) * 256; }

// ABL (measurement only, PDVC_PYR_ABLATE): 1 = no HBM staging (LDS holds whatever it held), 2 = no gather phase
template <int RD, int ABL = 0>
__global__ __launch_bounds__(kPyrThreads) void msda1d_fwd_pyr_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int qblocks, float* __restrict__ out, float* __restrict__ save_attn, float* __restrict__ save_loc) {
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    const int blk = xcd_remap(blockIdx.x, gridDim.x);  // the query blocks and heads of a video share an XCD
    const int qb = blk % qblocks, bm = blk / qblocks;
    const int b = bm / M, m = bm - b * M;
    const int slot = threadIdx.x >> 4, sub = threadIdx.x & 15;
    const size_t MD = (size_t)M * 64;
    const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
    const float* vsrc = value + (size_t)b * S * MD + (size_t)m * 64;
    // this lane's 16 B of every LDS row
    const char* lrow = reinterpret_cast<const char*>(lds4) + sub * 16;

    // parameters of this lane's sample j = sub for its 8 queries (msda1d_fwd_kernel's arithmetic)
    const int l_own = sub >> 2;
    const int T_own = lvl_sel(lv.T, l_own), st_own = lvl_sel(lv.start, l_own);
    const int base_own = pyr_base(lv, l_own);
    const float Tf_own = (float)T_own;
    // issue every parameter load first, then stage level 0 while they are in flight (neither depends on the
    // other), then do the parameter math: the loads' latency hides under the staging
    float lgv[kPyrQPS], offv[kPyrQPS], r0v[kPyrQPS], r1v[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        const size_t row = (size_t)b * Lq + (q < Lq ? q : 0);
        const float* prow = proj + row * proj_stride;
        lgv[i] = prow[logit_base + m * kNS + sub];
        offv[i] = prow[off_base + m * kNS + sub];
        r0v[i] = ref[(row * kL + l_own) * RD];
        r1v[i] = (RD == 2) ? ref[(row * kL + l_own) * RD + 1] : 0.f;
    }
    // ABL == 3 (measurement only): workgroups of odd slot pairs run the levels in the other order (levels 1..3 staged
    // and gathered first), so that neighbouring CUs stage at different times
    const bool rev = ABL == 3 && ((blockIdx.x >> 3) & 1);
    if (ABL != 1) {
        if (rev) pyr_stage_g_lean(lds4, vsrc, MD, lv.start[1], lv.T[1] + lv.T[2] + lv.T[3]);
        else pyr_stage_g_lean(lds4, vsrc, MD, lv.start[0], lv.T[0]);
    }
    // per query: the owner lane's corner-row byte offset and its two corner weights, the attention weight folded in
    int adv[kPyrQPS];
    float w1v[kPyrQPS], w2v[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        const bool act = q < Lq;
        const float lg = lgv[i];
        const float mx = group_max<16>(lg);
        const float sum = group_allreduce<16>(expf(lg - mx));
        const float aw = expf(lg - mx) / sum;
        const float off = offv[i];
        const float r0 = r0v[i];
        const float r1 = r1v[i];
        const float loc = (RD == 1) ? r0 + off / Tf_own : r0 + ((off / (float)kP) * r1) * 0.5f;
        if (save_loc && act) {
            const size_t si = save_index(b, m, l_own, q, sub & 3, Lq, M);
            save_loc[si] = loc;
            save_attn[si] = aw;
        }
        const float x = loc * Tf_own - 0.5f;
        const bool inside = x > -1.f && x < Tf_own;
        const float xf = floorf(inside ? x : 0.f);
        const int i0 = (int)xf;  // in [-1, T - 1] inside, 0 outside
        const float lw = inside ? x - xf : 0.f;
        bool ok1 = inside && i0 >= 0, ok2 = inside && i0 + 1 <= T_own - 1;
        if (mbase) {
            ok1 = ok1 && !mbase[st_own + min(max(i0, 0), T_own - 1)];
            ok2 = ok2 && !mbase[st_own + min(max(i0 + 1, 0), T_own - 1)];
        }
        adv[i] = pyr_corner(base_own, i0);
        w1v[i] = ok1 ? (1.f - lw) * aw : 0.f;
        w2v[i] = ok2 ? lw * aw : 0.f;
    }

    float4 acc[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    // one level of every query of the lane group: the sample's corner offset and weights come from their owner lane
    // by DPP row_newbcast (a VALU modifier, so the LDS pipe serves only the corner-row reads); the level is a
    // compile-time constant, which the DPP pattern needs.  Per sample and lane: 3 broadcasts, 1 address add, 2 LDS
    // reads (the second at +256 B), 4 packed FMAs (acc = w1 * v[x0] + acc, then w2 * v[x0 + 1] + acc).
    float4 tok = make_float4(0.f, 0.f, 0.f, 0.f);
    auto level = [&](auto Lc) {
        constexpr int L = decltype(Lc)::value;
#pragma unroll
        for (int i = 0; i < kPyrQPS; ++i) {
            float4 v1[kP], v2[kP];
            float c1[kP], c2[kP];
            // this query's broadcasts depend (opaquely) on the previous query's sums: without it the compiler hoists
            // every broadcast and LDS read of the level and spills (1 563 spilled VGPRs)
            int ad = adv[i];
            float wa = w1v[i], wb = w2v[i];
            __asm__ volatile("" : "+v"(ad), "+v"(wa), "+v"(wb) : "v"(tok.x), "v"(tok.y), "v"(tok.z), "v"(tok.w));
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                const char* r = lrow + grp_bcast<16>(ad, L * kP + p);
                c1[p] = grp_bcast<16>(wa, L * kP + p);
                c2[p] = grp_bcast<16>(wb, L * kP + p);
                v1[p] = *reinterpret_cast<const float4*>(r);
                v2[p] = *reinterpret_cast<const float4*>(r + 256);
            }
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                acc[i].x = fmaf(c1[p], v1[p].x, acc[i].x);
                acc[i].y = fmaf(c1[p], v1[p].y, acc[i].y);
                acc[i].z = fmaf(c1[p], v1[p].z, acc[i].z);
                acc[i].w = fmaf(c1[p], v1[p].w, acc[i].w);
                acc[i].x = fmaf(c2[p], v2[p].x, acc[i].x);
                acc[i].y = fmaf(c2[p], v2[p].y, acc[i].y);
                acc[i].z = fmaf(c2[p], v2[p].z, acc[i].z);
                acc[i].w = fmaf(c2[p], v2[p].w, acc[i].w);
            }
            tok = acc[i];
        }
    };
    __syncthreads();  // the first phase's rows were staged before the parameter math
    if (rev) {
        level(std::integral_constant<int, 1>{});
        level(std::integral_constant<int, 2>{});
        level(std::integral_constant<int, 3>{});
        __syncthreads();
        pyr_stage_g(lds4, vsrc, MD, lv.start[0], lv.T[0]);
        __syncthreads();
        level(std::integral_constant<int, 0>{});
    } else {
        if (ABL != 2) level(std::integral_constant<int, 0>{});
        __syncthreads();  // levels 1..3 in one round trip
        if (ABL != 1) pyr_stage_g(lds4, vsrc, MD, lv.start[1], lv.T[1] + lv.T[2] + lv.T[3]);
        __syncthreads();
        if (ABL != 2) {
            level(std::integral_constant<int, 1>{});
            level(std::integral_constant<int, 2>{});
            level(std::integral_constant<int, 3>{});
        }
    }
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        if (q < Lq)
            *reinterpret_cast<float4*>(out + ((size_t)b * Lq + q) * MD + (size_t)m * 64 + sub * 4) = acc[i];
    }
}

// -------------------------------------------------------------------------------------------------
// msda1d_fwd_pyr2_kernel: msda1d_fwd_pyr_kernel's arithmetic (same bits) with the staging moved onto LDS-DMA
// (global_load_lds_dwordx4: HBM -> LDS with no VGPR round trip, 1 KiB = 4 rows per wave-instruction) and laid out
// in the whole 160 KiB so that it overlaps compute:
//   * the parameter loads are waited for first, then the first phase's rows are issued as DMAs and the parameter
//     math (softmax, locations, corner weights) runs while they land;
//   * a pyramid of S + 2 <= 640 rows (T <= 318: yc2's T = 256, S = 480) is staged whole, one phase, one barrier;
//   * otherwise (anet's T = 512, S = 960) level 0 takes rows [0, T0 + 2) and levels 1..3 are placed at the END of
//     the LDS (rows [640 - 1 - n1, 640)), so the part of them above level 0's rows is prefetched during level 0's
//     gather and only the rest is staged between the two gathers.
// Guarded layout as in msda1d_fwd_pyr_kernel: a zero row before level 0 and after the last staged level, levels
// 1..3 back to back (a corner outside its level reads a neighbour's finite row with weight 0).
// -------------------------------------------------------------------------------------------------
constexpr int kLdsRows = 640;                                     // 160 KiB of 256-B rows
constexpr size_t kPyr2LdsMax = (size_t)kLdsRows * 256;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

// LDS-DMA copy of n head rows (256 B: the head's 64 channels) from global rows [g0, g0 + n) of vsrc to LDS rows
// [r0, r0 + n): chunk c (4 rows, one wave-instruction) goes to wave c % 16; lanes past the end are masked off
__device__ __forceinline__ void pyr_dma_rows(float4* __restrict__ lds, const float* __restrict__ vsrc, size_t MD,
                                             int g0, int r0, int n) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int nch = (n + 3) >> 2;
    for (int c = wave; c < nch; c += kPyrThreads / 64) {
        const int row = c * 4 + (lane >> 4);
        char* dst = reinterpret_cast<char*>(lds) + (size_t)(r0 + c * 4) * 256;
        if (row < n)
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(vsrc + (size_t)(g0 + row) * MD + (lane & 15) * 4),
                                             (lds_void_t*)dst, 16, 0, 0);
    }
}

// the same copy issued by inline assembly: the compiler does not see these LDS writes, so it does not order the
// LDS reads that follow after them (it waits vmcnt(0) before the first ds_read after a builtin DMA, which would
// serialise a prefetch with the gather it is meant to hide under).  The caller keeps the reads off these rows
// and retires the DMAs itself (pyr_dma_wait, then a barrier) before the rows are read.
__device__ __forceinline__ void pyr_dma_rows_async(float4* __restrict__ lds, const float* __restrict__ vsrc,
                                                   size_t MD, int g0, int r0, int n) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int nch = (n + 3) >> 2;
    for (int c = wave; c < nch; c += kPyrThreads / 64) {
        const int row = c * 4 + (lane >> 4);
        const uint32_t dst = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(lds_void_t*)(reinterpret_cast<char*>(lds) + (size_t)(r0 + c * 4) * 256));
        if (row < n) {
            const float* src = vsrc + (size_t)(g0 + row) * MD + (lane & 15) * 4;
            int keep;
            __asm__ volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(src), "s"(dst)
                : "memory");
        }
    }
}

__device__ __forceinline__ void pyr_dma_wait() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0) only

__device__ __forceinline__ void pyr_zero_row(float4* __restrict__ lds, int row, int tid0) {
    const int t = (int)threadIdx.x - tid0;
    if (t >= 0 && t < 16) lds[(size_t)row * 16 + t] = make_float4(0.f, 0.f, 0.f, 0.f);
}

template <int RD>
__global__ __launch_bounds__(kPyrThreads) void msda1d_fwd_pyr2_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int qblocks, float* __restrict__ out, float* __restrict__ save_attn, float* __restrict__ save_loc,
    uint16_t* __restrict__ out16) {
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    const int blk = xcd_remap(blockIdx.x, gridDim.x);  // the query blocks and heads of a video share an XCD
    const int qb = blk % qblocks, bm = blk / qblocks;
    const int b = bm / M, m = bm - b * M;
    const int slot = threadIdx.x >> 4, sub = threadIdx.x & 15;
    const size_t MD = (size_t)M * 64;
    const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
    const float* vsrc = value + (size_t)b * S * MD + (size_t)m * 64;
    const char* lrow = reinterpret_cast<const char*>(lds4) + sub * 16;
    const int n0 = lv.T[0], n1 = lv.T[1] + lv.T[2] + lv.T[3];
    const bool single = n0 + n1 + 2 <= kLdsRows;
    const int p2 = single ? 1 + n0 : kLdsRows - 1 - n1;  // LDS row of level 1's first position

    // the guard rows first: a ds_write issued while DMAs are in flight waits for them (the compiler orders LDS
    // writes after pending LDS-DMA writes)
    pyr_zero_row(lds4, 0, 0);
    pyr_zero_row(lds4, single ? n0 + n1 + 1 : n0 + 1, 64);
    if (!single) pyr_zero_row(lds4, kLdsRows - 1, 128);
    const int l_own = sub >> 2;
    const int T_own = lvl_sel(lv.T, l_own), st_own = lvl_sel(lv.start, l_own);
    const int base_own = l_own == 0 ? 1 : p2 + (st_own - lv.start[1]);
    const float Tf_own = (float)T_own;
    float lgv[kPyrQPS], offv[kPyrQPS], r0v[kPyrQPS], r1v[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        const size_t row = (size_t)b * Lq + (q < Lq ? q : 0);
        const float* prow = proj + row * proj_stride;
        lgv[i] = prow[logit_base + m * kNS + sub];
        offv[i] = prow[off_base + m * kNS + sub];
        r0v[i] = ref[(row * kL + l_own) * RD];
        r1v[i] = (RD == 2) ? ref[(row * kL + l_own) * RD + 1] : 0.f;
    }
    // the parameters first (a use of them while DMAs are in flight would wait for the DMAs too), then the first
    // phase's rows as DMAs, landing while the parameter math runs
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): gfx9 encoding, lgkm/exp counts left at their maximum
    pyr_dma_rows(lds4, vsrc, MD, lv.start[0], 1, single ? n0 + n1 : n0);
    int adv[kPyrQPS];
    float w1v[kPyrQPS], w2v[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        const bool act = q < Lq;
        const float lg = lgv[i];
        const float mx = group_max<16>(lg);
        const float sum = group_allreduce<16>(expf(lg - mx));
        const float aw = expf(lg - mx) / sum;
        const float off = offv[i];
        const float r0 = r0v[i];
        const float r1 = r1v[i];
        const float loc = (RD == 1) ? r0 + off / Tf_own : r0 + ((off / (float)kP) * r1) * 0.5f;
        if (save_loc && act) {
            const size_t si = save_index(b, m, l_own, q, sub & 3, Lq, M);
            save_loc[si] = loc;
            save_attn[si] = aw;
        }
        const float x = loc * Tf_own - 0.5f;
        const bool inside = x > -1.f && x < Tf_own;
        const float xf = floorf(inside ? x : 0.f);
        const int i0 = (int)xf;
        const float lw = inside ? x - xf : 0.f;
        bool ok1 = inside && i0 >= 0, ok2 = inside && i0 + 1 <= T_own - 1;
        if (mbase) {
            ok1 = ok1 && !mbase[st_own + min(max(i0, 0), T_own - 1)];
            ok2 = ok2 && !mbase[st_own + min(max(i0 + 1, 0), T_own - 1)];
        }
        adv[i] = pyr_corner(base_own, i0);
        w1v[i] = ok1 ? (1.f - lw) * aw : 0.f;
        w2v[i] = ok2 ? lw * aw : 0.f;
    }

    PAcc4 acc[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) acc[i] = pacc_zero();
    PAcc4 tok = pacc_zero();
    // per sample and lane: 3 DPP broadcasts, 1 address add, 2 LDS reads, 4 v_pk_fma_f32 on the loaded registers
    auto level = [&](auto Lc) {
        constexpr int L = decltype(Lc)::value;
#pragma unroll
        for (int i = 0; i < kPyrQPS; ++i) {
            pf4 v1[kP], v2[kP];
            float c1[kP], c2[kP];
            int ad = adv[i];
            float wa = w1v[i], wb = w2v[i];
            __asm__ volatile("" : "+v"(ad), "+v"(wa), "+v"(wb) : "v"(tok.lo), "v"(tok.hi));
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                const char* r = lrow + grp_bcast<16>(ad, L * kP + p);
                c1[p] = grp_bcast<16>(wa, L * kP + p);
                c2[p] = grp_bcast<16>(wb, L * kP + p);
                v1[p] = *reinterpret_cast<const pf4*>(r);
                v2[p] = *reinterpret_cast<const pf4*>(r + 256);
            }
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                pacc_fma(acc[i], c1[p], v1[p]);
                pacc_fma(acc[i], c2[p], v2[p]);
            }
            tok = acc[i];
        }
    };
    __syncthreads();  // the first phase's DMAs have landed (every wave waited for its own before the barrier)
    if (single) {
        level(std::integral_constant<int, 0>{});
        level(std::integral_constant<int, 1>{});
        level(std::integral_constant<int, 2>{});
        level(std::integral_constant<int, 3>{});
    } else {
        // levels 1..3's rows above level 0's region land during level 0's gather
        const int pre = n0 + 2 > p2 ? n0 + 2 - p2 : 0;  // phase-2 rows [0, pre) overlap level 0's rows
        pyr_dma_rows_async(lds4, vsrc, MD, lv.start[1] + pre, p2 + pre, n1 - pre);
        level(std::integral_constant<int, 0>{});
        pyr_dma_wait();   // this wave's prefetch landed ...
        __syncthreads();  // ... and every wave's; level 0 read by every wave
        pyr_zero_row(lds4, p2 - 1, 0);
        pyr_dma_rows(lds4, vsrc, MD, lv.start[1], p2, pre);
        __syncthreads();
        level(std::integral_constant<int, 1>{});
        level(std::integral_constant<int, 2>{});
        level(std::integral_constant<int, 3>{});
    }
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        if (q < Lq) {
            const size_t o = ((size_t)b * Lq + q) * MD + (size_t)m * 64 + sub * 4;
            const float4 r = pacc_f4(acc[i]);
            *reinterpret_cast<float4*>(out + o) = r;
            if (out16) store_bf16x4(out16 + o, r.x, r.y, r.z, r.w);
        }
    }
}

// -------------------------------------------------------------------------------------------------
// msda1d_fwd_win_kernel: the whole-pyramid forward for pyramids whose level 0 does not fit one staging phase --
// 512 < T0 <= 1024 with T1 <= 512 and T2 + T3 <= 512 (anet_c3d's T = 1024: 1024 / 512 / 256 / 128, BASELINE.json
// configs[4]; at T0 = 1024 one head's level 0 is 256 KiB, past the 160 KiB of LDS).  Level 0 is staged in two
// WINDOWS of rows, [0, 513) and [512, T0), overlapping by one row: a sample's corner rows x0, x0 + 1 with
// x0 <= 511 lie in the first, with x0 >= 512 in the second (x0 + 1 = T0 reads the guard row after it).  The owner
// lane of a level-0 sample computes its LDS offset for both windows -- in the window that does not hold the sample it
// points at two zero rows kept past the staged rows, so the weights need no second copy -- and the gather phase of
// each window broadcasts its own offset
// (msda1d_fwd_pyr2_kernel's DPP row_newbcast).  Then level 1 alone, then levels 2 and 3 packed: four staging phases,
// every corner row read from LDS, the same arithmetic and accumulation order as msda1d_fwd_pyr2_kernel (per query:
// levels in order, points in order, corner x0 then x0 + 1 -- a level-0 sample contributes in exactly one window).
// -------------------------------------------------------------------------------------------------
constexpr int kWinSplit = 512;                                   // first level-0 row of the second window
constexpr int kWinRows = kWinSplit + 1;                          // data rows of the first window
constexpr int kWinZero = kWinRows + 2;                           // two zero rows: the out-of-window corners
constexpr size_t kWinLds = (size_t)(kWinZero + 2) * 256;          // guard, 513 rows, guard, the two zero rows

__host__ __device__ inline bool win_fits(const Levels1d& lv) {
    return lv.T[0] > kWinSplit && lv.T[0] <= 2 * kWinSplit && lv.T[1] <= kWinSplit &&
           lv.T[2] + lv.T[3] <= kWinSplit;
}

template <int RD>
__global__ __launch_bounds__(kPyrThreads) void msda1d_fwd_win_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int qblocks, float* __restrict__ out, float* __restrict__ save_attn, float* __restrict__ save_loc,
    uint16_t* __restrict__ out16) {
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    const int blk = xcd_remap(blockIdx.x, gridDim.x);  // the query blocks and heads of a video share an XCD
    const int qb = blk % qblocks, bm = blk / qblocks;
    const int b = bm / M, m = bm - b * M;
    const int slot = threadIdx.x >> 4, sub = threadIdx.x & 15;
    const size_t MD = (size_t)M * 64;
    const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
    const float* vsrc = value + (size_t)b * S * MD + (size_t)m * 64;
    const char* lrow = reinterpret_cast<const char*>(lds4) + sub * 16;
    pyr_zero_row(lds4, 0, 0);  // the leading guard row of every phase
    pyr_zero_row(lds4, kWinZero, 64);
    pyr_zero_row(lds4, kWinZero + 1, 128);
    const int l_own = sub >> 2;
    const int T_own = lvl_sel(lv.T, l_own), st_own = lvl_sel(lv.start, l_own);
    const int base_own = l_own == 3 ? 1 + lv.T[2] : 1;  // LDS row of the owner level's row 0 in its phase
    const float Tf_own = (float)T_own;
    float lgv[kPyrQPS], offv[kPyrQPS], r0v[kPyrQPS], r1v[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        const size_t row = (size_t)b * Lq + (q < Lq ? q : 0);
        const float* prow = proj + row * proj_stride;
        lgv[i] = prow[logit_base + m * kNS + sub];
        offv[i] = prow[off_base + m * kNS + sub];
        r0v[i] = ref[(row * kL + l_own) * RD];
        r1v[i] = (RD == 2) ? ref[(row * kL + l_own) * RD + 1] : 0.f;
    }
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): the parameters, before the first phase's DMAs are issued
    pyr_dma_rows(lds4, vsrc, MD, lv.start[0], 1, kWinRows);
    // per query: the owner's corner weights and its LDS offset for window A (level 0 rows [0, 513); every other
    // level's phase) and for window B (level 0 rows [512, T0))
    int adA[kPyrQPS], adB[kPyrQPS];
    float w1v[kPyrQPS], w2v[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        const bool act = q < Lq;
        const float lg = lgv[i];
        const float mx = group_max<16>(lg);
        const float sum = group_allreduce<16>(expf(lg - mx));
        const float aw = expf(lg - mx) / sum;
        const float off = offv[i];
        const float r0 = r0v[i];
        const float r1 = r1v[i];
        const float loc = (RD == 1) ? r0 + off / Tf_own : r0 + ((off / (float)kP) * r1) * 0.5f;
        if (save_loc && act) {
            const size_t si = save_index(b, m, l_own, q, sub & 3, Lq, M);
            save_loc[si] = loc;
            save_attn[si] = aw;
        }
        const float x = loc * Tf_own - 0.5f;
        const bool inside = x > -1.f && x < Tf_own;
        const float xf = floorf(inside ? x : 0.f);
        const int i0 = (int)xf;
        const float lw = inside ? x - xf : 0.f;
        bool ok1 = inside && i0 >= 0, ok2 = inside && i0 + 1 <= T_own - 1;
        if (mbase) {
            ok1 = ok1 && !mbase[st_own + min(max(i0, 0), T_own - 1)];
            ok2 = ok2 && !mbase[st_own + min(max(i0 + 1, 0), T_own - 1)];
        }
        w1v[i] = ok1 ? (1.f - lw) * aw : 0.f;
        w2v[i] = ok2 ? lw * aw : 0.f;
        const int ad = pyr_corner(base_own, i0);
        const bool inB = l_own == 0 && i0 >= kWinSplit;
        adA[i] = inB ? kWinZero * 256 : ad;
        adB[i] = inB ? ad - kWinSplit * 256 : kWinZero * 256;
    }
    PAcc4 acc[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) acc[i] = pacc_zero();
    PAcc4 tok = pacc_zero();
    auto level = [&](auto Lc, auto Bc) {
        constexpr int L = decltype(Lc)::value;
        constexpr bool B = decltype(Bc)::value;
#pragma unroll
        for (int i = 0; i < kPyrQPS; ++i) {
            pf4 v1[kP], v2[kP];
            float c1[kP], c2[kP];
            int ad = B ? adB[i] : adA[i];
            float wa = w1v[i], wb = w2v[i];
            __asm__ volatile("" : "+v"(ad), "+v"(wa), "+v"(wb) : "v"(tok.lo), "v"(tok.hi));
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                const char* r = lrow + grp_bcast<16>(ad, L * kP + p);
                c1[p] = grp_bcast<16>(wa, L * kP + p);
                c2[p] = grp_bcast<16>(wb, L * kP + p);
                v1[p] = *reinterpret_cast<const pf4*>(r);
                v2[p] = *reinterpret_cast<const pf4*>(r + 256);
            }
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                pacc_fma(acc[i], c1[p], v1[p]);
                pacc_fma(acc[i], c2[p], v2[p]);
            }
            tok = acc[i];
        }
    };
    using F = std::false_type;
    using Tt = std::true_type;
    pyr_dma_wait();
    __syncthreads();  // window A landed
    level(std::integral_constant<int, 0>{}, F{});
    __syncthreads();  // every wave is done with window A
    const int nB = lv.T[0] - kWinSplit;
    pyr_dma_rows(lds4, vsrc, MD, lv.start[0] + kWinSplit, 1, nB);
    pyr_zero_row(lds4, 1 + nB, 0);
    pyr_dma_wait();
    __syncthreads();
    level(std::integral_constant<int, 0>{}, Tt{});
    __syncthreads();
    pyr_dma_rows(lds4, vsrc, MD, lv.start[1], 1, lv.T[1]);
    pyr_zero_row(lds4, 1 + lv.T[1], 0);
    pyr_dma_wait();
    __syncthreads();
    level(std::integral_constant<int, 1>{}, F{});
    __syncthreads();
    const int n23 = lv.T[2] + lv.T[3];
    pyr_dma_rows(lds4, vsrc, MD, lv.start[2], 1, n23);
    pyr_zero_row(lds4, 1 + n23, 0);
    pyr_dma_wait();
    __syncthreads();
    level(std::integral_constant<int, 2>{}, F{});
    level(std::integral_constant<int, 3>{}, F{});
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        if (q < Lq) {
            const size_t o = ((size_t)b * Lq + q) * MD + (size_t)m * 64 + sub * 4;
            const float4 r = pacc_f4(acc[i]);
            *reinterpret_cast<float4*>(out + o) = r;
            if (out16) store_bf16x4(out16 + o, r.x, r.y, r.z, r.w);
        }
    }
}

// -------------------------------------------------------------------------------------------------
// backward, query side: grad of the offset and attention logits (+ reference points)
// softmax backward needs delta = sum_j a_j dL/da_j over the 16 samples of a (query, head).  Default (fout NULL):
// each level's owner lanes keep their (a_j, dL/da_j) pair in registers -- one pair per lane per level -- and the
// lane group sums a_j dL/da_j after the last level (the order of the reference's autograd softmax backward
// over grad_attn_weight).  With fout: delta = <dL/dout, out> (out = the forward output of this head), read as a
// second 256-B row per (query, head), which lets every level finish as soon as it is reduced.
// grad_ref sums over the heads of a query, which live in different waves: atomics (zeroed by the host).
// -------------------------------------------------------------------------------------------------
template <int CPL, int LPH, int RD>
__global__ __launch_bounds__(256) void msda1d_bwd_query_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int D, int total_waves, const float* __restrict__ gout, const float* __restrict__ fout,
    const float* __restrict__ save_attn, const float* __restrict__ save_loc, float* __restrict__ grad_proj,
    float* __restrict__ grad_ref) {
    constexpr int JPL = kNS / LPH;
    constexpr int G = LPH < 8 ? LPH : 8;  // reduce-scatter group for the level's 8 partial sums
    constexpr int VPL = 8 / G;            // values per lane after it (interleaved (ga, gs) pairs)
    const int lane = threadIdx.x & 63;
    const int wave = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
    if (wave >= total_waves) return;  // wave-uniform
    const WaveQuery w = wave_query<LPH>(wave, lane, Lq, M);
    const size_t MD = (size_t)M * D;
    const uint8_t* mbase = vmask ? vmask + (size_t)w.b * S : nullptr;
    const int c0 = w.sub * CPL;

    VecF<CPL> g;
    g.load(gout + (size_t)w.row * MD + (size_t)w.m * D + c0);
    float delta = 0.f;
    if (fout) {  // wave-uniform
        VecF<CPL> o;
        o.load(fout + (size_t)w.row * MD + (size_t)w.m * D + c0);
        float dl = 0.f;
#pragma unroll
        for (int c = 0; c < CPL; ++c) dl += g.v[c] * o.v[c];
        delta = group_allreduce<LPH>(dl);
    }
    float keep_ga[kL];  // dL/da of this lane's owned sample per level, and sum of a dL/da (fout == NULL)
    float dl_own = 0.f;

    // parameter phase: corner row and (masked) corner weights of the lane's samples
    int i0v[JPL];
    float lwv[JPL];
    int okv[JPL];
#pragma unroll
    for (int k = 0; k < JPL; ++k) {
        const int j = w.sub + LPH * k;
        const int l = j / kP;
        const int T = lvl_sel(lv.T, l), st = lvl_sel(lv.start, l);
        const float Tf = (float)T;
        const float x = save_loc[save_index(w.b, w.m, l, w.q, j % kP, Lq, M)] * Tf - 0.5f;
        const bool inside = x > -1.f && x < Tf;
        const float xf = floorf(inside ? x : 0.f);
        const int i0 = (int)xf;
        bool ok1 = inside && i0 >= 0, ok2 = inside && i0 + 1 <= T - 1;
        if (mbase) {
            ok1 = ok1 && !mbase[st + min(max(i0, 0), T - 1)];
            ok2 = ok2 && !mbase[st + min(max(i0 + 1, 0), T - 1)];
        }
        i0v[k] = i0;
        lwv[k] = inside ? x - xf : 0.f;
        okv[k] = (ok1 ? 1 : 0) | (ok2 ? 2 : 0);
    }

    const float* vbase = value + (size_t)w.b * S * MD + (size_t)w.m * D + c0;
    const float* prow = proj + (size_t)w.row * proj_stride;
    float* gprow = grad_proj + (size_t)w.row * proj_stride;
#pragma unroll
    for (int l = 0; l < kL; ++l) {
        const int T = lv.T[l], st = lv.start[l];
        const float Tf = (float)T;
        VecF<CPL> v1[kP], v2[kP];
        float lw[kP];
        int ok[kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {  // all 2*P corner loads in flight together (clamped, selected later)
            const int j = l * kP + p;
            const int i0 = grp_bcast<LPH>(i0v[j / LPH], j % LPH);
            lw[p] = grp_bcast<LPH>(lwv[j / LPH], j % LPH);
            ok[p] = grp_bcast<LPH>(okv[j / LPH], j % LPH);
            const int a1 = min(max(i0, 0), T - 1), a2 = min(max(i0 + 1, 0), T - 1);
            v1[p].load(vbase + (size_t)(st + a1) * MD);
            v2[p].load(vbase + (size_t)(st + a2) * MD);
        }
        // part[2p] = sum_c g*val ; part[2p+1] = sum_c g*(v2 - v1) over this lane's channels
        float part[2 * kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const float hw = 1.f - lw[p];
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const float x1 = (ok[p] & 1) ? v1[p].v[c] : 0.f, x2 = (ok[p] & 2) ? v2[p].v[c] : 0.f;
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
            for (int d = G; d < LPH; d <<= 1) part[k] += grp_swap(part[k], d);  // exact xor for d = 8
        }
        // group lane r (= sub % G) holds values [r*VPL, (r+1)*VPL) of the interleaved (ga, gs) list
        float ga, gs;
        int p;
        const int r = w.sub % G;
        if (VPL == 2) {
            p = r;
            ga = part[0];
            gs = part[1];
        } else {
            const float other = grp_swap(part[0], 1);
            p = r >> 1;
            ga = (r & 1) ? other : part[0];
            gs = (r & 1) ? part[0] : other;
        }
        const bool owner = w.active && w.sub < G && (VPL == 2 || (r & 1) == 0);
        const int j = l * kP + p;
        const float a = save_attn[save_index(w.b, w.m, l, w.q, p, Lq, M)];
        // CUDA: grad_loc_w = W * grad_w_weight * (top_grad * attn), summed over channels (.cuh:158)
        const float gloc = owner ? Tf * (gs * a) : 0.f;
        float g0 = gloc, g1 = 0.f;
        if (owner) {
            float goff;
            if (RD == 1) {
                goff = gloc / Tf;
            } else {
                const float rr1 = ref[((size_t)w.row * kL + l) * 2 + 1];
                const float t2 = gloc * 0.5f;
                goff = (t2 * rr1) / (float)kP;
                g1 = t2 * (prow[off_base + w.m * kNS + j] / (float)kP);
            }
            gprow[off_base + w.m * kNS + j] = goff;
            if (fout) gprow[logit_base + w.m * kNS + j] = a * (ga - delta);
        }
        keep_ga[l] = ga;
        dl_own += owner ? a * ga : 0.f;
        if (grad_ref) {
            // sum over the query's points of this level (its lane group), one atomic per (query, head, level)
            g0 = group_allreduce<LPH>(g0);
            if (RD == 2) g1 = group_allreduce<LPH>(g1);
            if (w.sub == 0 && w.active) {
                float* dst = grad_ref + ((size_t)w.row * kL + l) * RD;
                atomicAdd(dst, g0);
                if (RD == 2) atomicAdd(dst + 1, g1);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (!fout) {
        delta = group_allreduce<LPH>(dl_own);
        // the owned sample's point index and ownership do not depend on the level (see the loop above)
        const int r = w.sub % G;
        const int p = VPL == 2 ? r : r >> 1;
        if (w.active && w.sub < G && (VPL == 2 || (r & 1) == 0)) {
#pragma unroll
            for (int l = 0; l < kL; ++l) {
                const int j = l * kP + p;
                const float a = save_attn[save_index(w.b, w.m, l, w.q, p, Lq, M)];  // re-read (cached) rather than held across the levels
                gprow[logit_base + w.m * kNS + j] = a * (keep_ga[l] - delta);
            }
        }
    }
}

// -------------------------------------------------------------------------------------------------
// backward, query side, dot-product form (D = 64: 16 lanes x float4 per query, 4 queries per wave).
// Every quantity the query side needs from a sample's two corner rows is linear in the two dot products
//     d1 = <dL/dout, value[x0]>,   d2 = <dL/dout, value[x0 + 1]>    (this head's 64 channels)
// (.cuh:140-170: grad_attn = hw*d1 + lw*d2 and grad_loc = T * attn * (d2 - d1), each corner counted only where the
// reference samples it).  So the lanes form only the raw per-channel products (8 FMAs per sample and lane),
// reduce the level's 8 partials over the 16-lane group, and the lane that owns the sample (lane j = l*P + p,
// the one that read its location and weight) applies the corner weights and the masks once, after the
// reduction -- msda1d_bwd_query_kernel applies them per channel and lane (4x the VALU work) and recomputed the
// sample parameters on every lane through shuffles.  Corner rows are read with buffer loads: one 32-bit offset
// per sample (the second corner one row further), and a sample's clamping replaced by the
// descriptor's range check (the video's S rows; a corner outside the level reads a neighbouring level's row
// or zeros, and the mask removes it after the reduction).  The measured profile of msda1d_bwd_query_kernel was
// VALU issue (1 900 VALU instructions per wave, 44 per VMEM read); this form issues ~400.
// Reduction order per level: reduce-scatter over lane bits 8, 2, 1 (DPP), then an all-reduce over bit 4
// (ds_swizzle): lane sub holds value (sub & 8 ? 4 : 0) + (sub & 3) of [d1_0..d1_3, d2_0..d2_3], and one xor-8
// DPP exchange gives every lane the (d1, d2) pair of point sub & 3 -- so lane 4l + p, the owner of sample
// (l, p), ends each level holding exactly its own pair.
// -------------------------------------------------------------------------------------------------
template <int RD>
__global__ __launch_bounds__(256) void msda1d_bwd_query_dot_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int total_waves, const float* __restrict__ gout, const float* __restrict__ save_attn,
    const float* __restrict__ save_loc, float* __restrict__ grad_proj, float* __restrict__ grad_ref) {
    constexpr int D = 64;
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane tells the compiler, so the video / head / buffer descriptor
    // live in scalar registers (a per-lane descriptor costs a waterfall loop around every buffer load)
    const int wave = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
    if (wave >= total_waves) return;
    const WaveQuery w = wave_query<16>(wave, lane, Lq, M);
    const int MD = M * D;
    const int c0 = w.sub * 4;

    // this lane's sample j = sub: level l_own, its corner row, weights and masks (ms_deform_attn.py:168-177 math
    // as in the forward; the location and softmaxed weight come from the forward's save_loc / save_attn)
    const int j = w.sub, l_own = j >> 2;
    int T_own = lv.T[0], st_own = lv.start[0];  // branch-free per-lane level select
#pragma unroll
    for (int l = 1; l < kL; ++l) {
        T_own = l_own >= l ? lv.T[l] : T_own;
        st_own = l_own >= l ? lv.start[l] : st_own;
    }
    const float Tf = (float)T_own;
    const size_t si = save_index(w.b, w.m, l_own, w.q, j & 3, Lq, M);
    const float x = save_loc[si] * Tf - 0.5f;
    const float a = save_attn[si];
    const bool inside = x > -1.f && x < Tf;
    const float xf = floorf(inside ? x : 0.f);
    const int i0 = (int)xf;
    const float lw = inside ? x - xf : 0.f;
    bool ok1 = inside && i0 >= 0, ok2 = inside && i0 + 1 <= T_own - 1;
    if (vmask) {
        const uint8_t* mb = vmask + (size_t)w.b * S + st_own;
        ok1 = ok1 && !mb[min(max(i0, 0), T_own - 1)];
        ok2 = ok2 && !mb[min(max(i0 + 1, 0), T_own - 1)];
    }
    // byte offset of this sample's corner-1 row inside the video's value slice (broadcast to the group), and of
    // this lane's channels of head m inside a row
    const int roff = (st_own + i0) * (MD * 4);
    const int coff = (w.m * D + c0) * 4;

    float4 g = *reinterpret_cast<const float4*>(gout + (size_t)w.row * MD + (size_t)w.m * D + c0);
    const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(  // scalar: one video per wave
        (void*)(value + (size_t)__builtin_amdgcn_readfirstlane(w.b) * S * MD), (short)0, S * MD * 4, 0x00020000);
    float d1 = 0.f, d2 = 0.f;  // this lane's sample's full dot products
#pragma unroll
    for (int l = 0; l < kL; ++l) {
        float part[8];  // [d1_0..d1_3, d2_0..d2_3], this lane's 4 channels
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const int off = grp_bcast<16>(roff, l * kP + p) + coff;
            const auto u1 = __builtin_amdgcn_raw_buffer_load_b128(vr, off, 0, 0);
            const auto u2 = __builtin_amdgcn_raw_buffer_load_b128(vr, off + MD * 4, 0, 0);
            part[p] = g.x * __uint_as_float(u1[0]) + g.y * __uint_as_float(u1[1]) + g.z * __uint_as_float(u1[2]) +
                      g.w * __uint_as_float(u1[3]);
            part[4 + p] = g.x * __uint_as_float(u2[0]) + g.y * __uint_as_float(u2[1]) +
                          g.z * __uint_as_float(u2[2]) + g.w * __uint_as_float(u2[3]);
        }
        // reduce-scatter over lane bits 8, 2, 1: lane keeps value (sub & 8 ? 4 : 0) + (sub & 3)
        {
            const bool u8 = (lane & 8) != 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float send = u8 ? part[i] : part[i + 4];
                const float mine = u8 ? part[i + 4] : part[i];
                part[i] = mine + grp_swap(send, 8);
            }
            const bool u2b = (lane & 2) != 0;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float send = u2b ? part[i] : part[i + 2];
                const float mine = u2b ? part[i + 2] : part[i];
                part[i] = mine + grp_swap(send, 2);
            }
            const bool u1b = (lane & 1) != 0;
            const float send = u1b ? part[0] : part[1];
            const float mine = u1b ? part[1] : part[0];
            part[0] = mine + grp_swap(send, 1);
            part[0] += grp_swap(part[0], 4);
        }
        // lanes 0..7 hold d1 of point sub & 3, lanes 8..15 its d2; one xor-8 exchange pairs them
        const float other = grp_swap(part[0], 8);
        if (l_own == l) {
            d1 = (l < 2) ? part[0] : other;
            d2 = (l < 2) ? other : part[0];
        }
    }

    // owner math (.cuh:140-170): corner weights and masks after the reduction
    const float x1 = ok1 ? d1 : 0.f, x2 = ok2 ? d2 : 0.f;
    const float ga = (1.f - lw) * x1 + lw * x2;  // dL/da_j
    const float gloc = Tf * ((x2 - x1) * a);     // dL/dloc_j
    const float* prow = proj + (size_t)w.row * proj_stride;
    float* gprow = grad_proj + (size_t)w.row * proj_stride;
    float g0 = gloc, g1 = 0.f, goff;
    if (RD == 1) {
        goff = gloc / Tf;
    } else {
        const float rr1 = ref[((size_t)w.row * kL + l_own) * 2 + 1];
        const float t2 = gloc * 0.5f;
        goff = (t2 * rr1) / (float)kP;
        g1 = t2 * (prow[off_base + w.m * kNS + j] / (float)kP);
    }
    // softmax backward: delta = sum_j a_j dL/da_j over the (query, head)'s 16 samples
    const float delta = group_allreduce<16>(a * ga);
    if (w.active) {
        gprow[off_base + w.m * kNS + j] = goff;
        gprow[logit_base + w.m * kNS + j] = a * (ga - delta);
    }
    if (grad_ref) {  // per (query, level): sum over the level's 4 points = the lane quad; heads differ by wave
        g0 += grp_swap(g0, 1);
        g0 += grp_swap(g0, 2);
        if (RD == 2) {
            g1 += grp_swap(g1, 1);
            g1 += grp_swap(g1, 2);
        }
        if ((j & 3) == 0 && w.active) {
            float* dst = grad_ref + ((size_t)w.row * kL + l_own) * RD;
            atomicAdd(dst, g0);
            if (RD == 2) atomicAdd(dst + 1, g1);
        }
    }
}

// -------------------------------------------------------------------------------------------------
// Whole-pyramid twin of msda1d_bwd_query_dot_kernel for the encoder (Lq ~ S, D = 64): one 1024-thread workgroup per
// (video, head, block of up to 960 queries), the head's value rows staged in LDS level by level as in
// msda1d_fwd_pyr_kernel (level 0, then levels 1..3), every corner row read from LDS (ds_read_b128, 256 B/clk/CU)
// instead of through L1.  A 16-lane group takes 15 queries in turn; per query the dot-product form, its reduction
// and the owner-lane math of msda1d_bwd_query_dot_kernel, the sample's row index broadcast by DPP row_newbcast
// (VALU: the LDS pipe serves only the row reads).  Level 0's owners (lanes 0..3) finish their offset gradient in the
// first phase and carry dL/da to the second through LDS (15 KiB beside the 128 KiB of rows), where the softmax
// term of all 16 samples is formed.
// -------------------------------------------------------------------------------------------------
constexpr int kBqQPS = 15;                                   // queries per 16-lane group
constexpr int kBqQ = (kPyrThreads / 16) * kBqQPS;            // 960 queries per workgroup
constexpr size_t kBqLds = kPyrLds + (size_t)kBqQ * 4 * sizeof(float);

// QU: queries of a lane group run back to back per loop trip (interleavable by the scheduler: each query is a
// dependent chain of LDS reads, a 16-lane reduction and the owner math, and the LDS caps the CU at 4 waves/SIMD)
template <int RD, int QU = 1>
__global__ __launch_bounds__(kPyrThreads) void msda1d_bwd_query_pyr_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ proj,
    int proj_stride, int off_base, int logit_base, const float* __restrict__ ref, Levels1d lv, int Lq, int S, int M,
    int qblocks, const float* __restrict__ gout, const float* __restrict__ save_attn,
    const float* __restrict__ save_loc, float* __restrict__ grad_proj, float* __restrict__ grad_ref,
    uint16_t* __restrict__ gp16) {
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float* carry = reinterpret_cast<float*>(lds4 + kPyrRowsG * 16);  // [kBqQ][4]: dL/da of level 0's samples
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int qb = blk % qblocks, bm = blk / qblocks;
    const int b = bm / M, m = bm - b * M;
    const int slot = threadIdx.x >> 4, sub = threadIdx.x & 15, lane = threadIdx.x & 63;
    const int MD = M * 64;
    const float* vsrc = value + (size_t)b * S * MD + (size_t)m * 64;
    const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
    const int l_own = sub >> 2, p_own = sub & 3;
    int T_own = lv.T[0], st_own = lv.start[0];
#pragma unroll
    for (int l = 1; l < kL; ++l) {
        T_own = l_own >= l ? lv.T[l] : T_own;
        st_own = l_own >= l ? lv.start[l] : st_own;
    }
    const float Tf = (float)T_own;
    const int base_own = pyr_base(lv, l_own);
    const char* lrow = reinterpret_cast<const char*>(lds4) + sub * 16;  // this lane's 16 B of every LDS row

    // QU queries of this lane group (queries i0, i0 + 1, ..) through the levels [L0, L1): the lanes' own sample
    // parameters, the dot products of every sample of those levels from LDS reduced onto their owner lanes, then the
    // owner math of the lanes whose level is in range (offset gradient, grad_ref, dL/da).  The QU queries' loads, LDS
    // reads and reductions are independent chains written side by side, so they overlap (the carry / gradient
    // stores come last: they would otherwise order the next query's LDS reads behind them)
    auto run_queries = [&](int i0q, auto L0c, auto L1c) {
        constexpr int L0 = decltype(L0c)::value, L1 = decltype(L1c)::value;
        bool act[QU], inside[QU];
        size_t row[QU];
        float4 g[QU];
        float a[QU], lw[QU], d1[QU], d2[QU];
        int i0[QU], ad[QU];
#pragma unroll
        for (int u = 0; u < QU; ++u) {
            const int q0 = qb * kBqQ + slot + 64 * (i0q + u);
            act[u] = q0 < Lq;
            const int q = act[u] ? q0 : Lq - 1;
            row[u] = (size_t)b * Lq + q;
            g[u] = *reinterpret_cast<const float4*>(gout + row[u] * MD + (size_t)m * 64 + sub * 4);
            const size_t si = save_index(b, m, l_own, q, p_own, Lq, M);
            const float x = save_loc[si] * Tf - 0.5f;
            a[u] = save_attn[si];
            inside[u] = x > -1.f && x < Tf;
            const float xf = floorf(inside[u] ? x : 0.f);
            i0[u] = (int)xf;
            lw[u] = inside[u] ? x - xf : 0.f;
            ad[u] = pyr_corner(base_own, i0[u]);  // guarded layout: no clamps (msda1d_fwd_pyr_kernel)
            d1[u] = 0.f;
            d2[u] = 0.f;
        }
#pragma unroll
        for (int L = L0; L < L1; ++L) {
#pragma unroll
            for (int u = 0; u < QU; ++u) {
                float part[8];
                // the 4-channel dot products on packed fp32 pairs: v_pk_mul + v_pk_fma + one add per corner row
                const pf2 gxy = {g[u].x, g[u].y}, gzw = {g[u].z, g[u].w};
#pragma unroll
                for (int p = 0; p < kP; ++p) {
                    const char* r = lrow + grp_bcast<16>(ad[u], L * kP + p);
                    const pf4 u1 = *reinterpret_cast<const pf4*>(r);
                    const pf4 u2 = *reinterpret_cast<const pf4*>(r + 256);
                    const pf2 t1 = __builtin_elementwise_fma(gzw, u1.zw, gxy * u1.xy);
                    const pf2 t2 = __builtin_elementwise_fma(gzw, u2.zw, gxy * u2.xy);
                    part[p] = t1.x + t1.y;
                    part[4 + p] = t2.x + t2.y;
                }
                const bool u8 = (lane & 8) != 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float send = u8 ? part[k] : part[k + 4];
                    const float mine = u8 ? part[k + 4] : part[k];
                    part[k] = mine + grp_swap(send, 8);
                }
                const bool u2b = (lane & 2) != 0;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const float send = u2b ? part[k] : part[k + 2];
                    const float mine = u2b ? part[k + 2] : part[k];
                    part[k] = mine + grp_swap(send, 2);
                }
                const bool u1b = (lane & 1) != 0;
                const float send = u1b ? part[0] : part[1];
                const float mine = u1b ? part[1] : part[0];
                part[0] = mine + grp_swap(send, 1);
                part[0] += grp_swap(part[0], 4);
                const float other = grp_swap(part[0], 8);
                if (l_own == L) {
                    d1[u] = (L < 2) ? part[0] : other;
                    d2[u] = (L < 2) ? other : part[0];
                }
            }
        }
        // owner math of the lanes whose sample is in this phase (.cuh:140-170), as msda1d_bwd_query_dot_kernel
        const bool mine_phase = l_own >= L0 && l_own < L1;
#pragma unroll
        for (int u = 0; u < QU; ++u) {
            bool ok1 = inside[u] && i0[u] >= 0, ok2 = inside[u] && i0[u] + 1 <= T_own - 1;
            if (mbase) {
                ok1 = ok1 && !mbase[st_own + min(max(i0[u], 0), T_own - 1)];
                ok2 = ok2 && !mbase[st_own + min(max(i0[u] + 1, 0), T_own - 1)];
            }
            const float x1 = ok1 ? d1[u] : 0.f, x2 = ok2 ? d2[u] : 0.f;
            float ga = (1.f - lw[u]) * x1 + lw[u] * x2;
            const float gloc = Tf * ((x2 - x1) * a[u]);
            const float* prow = proj + row[u] * proj_stride;
            float* gprow = grad_proj + row[u] * proj_stride;
            float g0 = mine_phase ? gloc : 0.f, g1 = 0.f, goff;
            if (RD == 1) {
                goff = gloc / Tf;
            } else {
                const float rr1 = ref[(row[u] * kL + l_own) * 2 + 1];
                const float t2 = gloc * 0.5f;
                goff = (t2 * rr1) / (float)kP;
                g1 = mine_phase ? t2 * (prow[off_base + m * kNS + sub] / (float)kP) : 0.f;
            }
            if (act[u] && mine_phase) {
                gprow[off_base + m * kNS + sub] = goff;
                if (gp16) gp16[row[u] * proj_stride + off_base + m * kNS + sub] = (uint16_t)bf16_bits(goff);
            }
            if (grad_ref) {  // per (query, level): the lane quad of the level; heads differ by workgroup: atomics
                g0 += grp_swap(g0, 1);
                g0 += grp_swap(g0, 2);
                if (RD == 2) {
                    g1 += grp_swap(g1, 1);
                    g1 += grp_swap(g1, 2);
                }
                if (p_own == 0 && act[u] && mine_phase) {
                    float* dst = grad_ref + (row[u] * kL + l_own) * RD;
                    atomicAdd(dst, g0);
                    if (RD == 2) atomicAdd(dst + 1, g1);
                }
            }
            const int ci = (slot + 64 * (i0q + u)) * 4 + p_own;
            if (L0 == 0) {  // first phase: level 0's owners carry dL/da to the second
                if (l_own == 0) carry[ci] = ga;
            } else {  // second phase: the softmax term over all 16 samples, then every logit gradient
                if (l_own == 0) ga = carry[ci];
                const float delta = group_allreduce<16>(a[u] * ga);
                if (act[u]) {
                    const float gl = a[u] * (ga - delta);
                    gprow[logit_base + m * kNS + sub] = gl;
                    if (gp16) gp16[row[u] * proj_stride + logit_base + m * kNS + sub] = (uint16_t)bf16_bits(gl);
                }
            }
        }
    };

    pyr_stage_g(lds4, vsrc, MD, lv.start[0], lv.T[0]);
    __syncthreads();
    static_assert(kBqQPS % QU == 0, "QU must divide the queries per lane group");
#pragma unroll 1
    for (int i = 0; i < kBqQPS; i += QU) run_queries(i, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
    __syncthreads();
    pyr_stage_g(lds4, vsrc, MD, lv.start[1], lv.T[1] + lv.T[2] + lv.T[3]);
    __syncthreads();
#pragma unroll 1
    for (int i = 0; i < kBqQPS; i += QU) run_queries(i, std::integral_constant<int, 1>{}, std::integral_constant<int, 4>{});
}

// -------------------------------------------------------------------------------------------------
// backward, value side: destination-centric sum over an inverted index, no float atomics.
// One workgroup per (video, head, level) and chunk of queries.  Row t of the level receives
//     grad_value[t] = sum_{x0(s) = t} hw_s a_s g_q(s)  +  sum_{x0(s) = t-1} lw_s a_s g_q(s)
// over the samples s = (q, p) of that level.  The workgroup buckets its samples by key = x0 + 1 in LDS
// (counting sort: one LDS integer atomic per sample), so row t needs exactly the contiguous sorted
// range of buckets t (high corner) and t+1 (low corner).  Each wave owns a contiguous row range chosen
// so that the waves see equal sample counts, walks its buckets in order with two running accumulators
// (lane = channel, one 256-B gradient row load per sample, 8 in flight) and writes every row exactly
// once with plain coalesced stores -- rows no sample touches are written as zeros, so grad_value needs
// no memset.  (The first version accumulated with ds_add_f32 and ran ~7x slower: LDS float atomics
// were the kernel's whole cost, measured by replacing them with plain stores -- tools/kbench.py.)
// -------------------------------------------------------------------------------------------------
constexpr int kVW = 8;     // waves per value-gradient workgroup
constexpr int kVQPT = 4;  // queries per thread in its sort passes: a launch chunk holds <= kVQPT * kVW * 64 queries

// CW: channels per lane (D <= 64 -> 1, D = 128 -> 2).  G4 (D == 64): the gather phase runs on 16-lane groups
// with a float4 per lane instead of whole waves with one float per lane -- 32 row ranges per workgroup, and one
// wave-instruction loads the gradient rows of 4 samples (4x fewer loads, LDS index reads and loop iterations).
// UG: samples in flight per 16-lane group in the G4 walk (8: 96 VGPRs; 4: 66, more workgroups per CU where the LDS
// allows -- the decoder's short sample lists)
// B16: also writes the bf16 rounding of every row into gv16 (the bf16 mode; a separate instantiation, so the
// fp32 path keeps its registers: the pointer and its stores cost the depth-8 walk 9 spilled VGPRs)
// ABL (measurement only, PDVC_VAL_ABLATE): 1 = stop after the sort, 2 = walk without the gradient-row gathers
// (PDVC_VAL_ABLATE=1/2 select them for the depth-8 encoder walk, 3/4 for the depth-4 decoder walk)
template <int CW, bool G4, int UG = 8, bool B16 = false, int ABL = 0>
__global__ __launch_bounds__(kVW * 64, 6) void msda1d_bwd_value_kernel(const uint8_t* __restrict__ vmask, Levels1d lv,
                                                                     int Lq, int q0, int nq, int S, int M, int D,
                                                                     int accumulate,
                                                                     const float* __restrict__ gout,
                                                                     const float* __restrict__ save_attn,
                                                                     const float* __restrict__ save_loc,
                                                                     float* __restrict__ grad_value,
                                                                     float* __restrict__ level_sums,
                                                                     const int64_t* __restrict__ dshapes = nullptr,
                                                                     const int64_t* __restrict__ dlsi = nullptr,
                                                                     uint16_t* __restrict__ gv16 = nullptr) {
    extern __shared__ __attribute__((aligned(16))) int lds_i[];
    // the drop-in fast path passes its device level table: the kernel runs only for a 1-D pyramid (dropin_levels)
    if (dshapes != nullptr && !dropin_levels(dshapes, dlsi, S, lv)) return;
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int l = lb % kL;  // the 4 levels of one (video, head) read the same gradient rows: same XCD
    const int bm = lb / kL;
    const int b = bm / M, m = bm - b * M;
    const int T = lvl_sel(lv.T, l), st = lvl_sel(lv.start, l);
    const float Tf = (float)T;
    const int n = nq * kP;  // samples of this (video, head, level, query chunk)
    int* off = lds_i;                       // [T + 2]: bucket counts, then exclusive offsets
    int* cur = lds_i + (T + 2);             // [T + 2]: scatter cursors
    int* sq = lds_i + 2 * (T + 2);          // [n] query of each sorted sample
    float* clo = (float*)(sq + n);          // [n] hw * a  -> row x0
    float* chi = clo + n;                   // [n] lw * a  -> row x0 + 1
    // G4: 12 B per sorted sample instead -- (key << 16 | query) and (hw * a, lw * a) -- one ds_read_b32 and one
    // ds_read_b64 in the walk (16-B entries held the encoder at two workgroups per CU)
    uint32_t* eqk = reinterpret_cast<uint32_t*>(lds_i + 2 * (T + 2));
    float2* ew = reinterpret_cast<float2*>(lds_i + ((2 * (T + 2) + n + 1) & ~1));
    __shared__ int wsum[kVW];

    for (int i = threadIdx.x; i < T + 2; i += blockDim.x) off[i] = 0;
    __syncthreads();
    // 1) histogram of key = x0 + 1 in [0, T] (samples outside (-1, T) touch no row, as in the reference).  A thread
    // takes whole queries (one float4 = the level's 4 points, from the level-major slab) and keeps each sample's key
    // and fraction in registers for the scatter pass, so save_loc is read once.
    const size_t sbase = save_index(b, m, l, q0, 0, Lq, M);
    int key[kVQPT][kP];
    float lwv[kVQPT][kP];
    // a thread takes kVQPT consecutive queries: neighbouring lanes are kVQPT queries apart, so on the coarse levels
    // (where neighbouring queries sample the same rows) fewer lanes of one atomic hit the same counter.  A chunk of
    // at most one query per thread (the decoder: 100) spreads them one per thread instead (25 threads did all)
    const bool spread = nq <= (int)blockDim.x;
#pragma unroll
    for (int k = 0; k < kVQPT; ++k) {
        const int qi = spread ? (k == 0 ? (int)threadIdx.x : nq) : (int)threadIdx.x * kVQPT + k;
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            key[k][p] = -1;
            lwv[k][p] = 0.f;
        }
        if (qi < nq) {
            const float4 lc = *reinterpret_cast<const float4*>(save_loc + sbase + (size_t)qi * kP);
            const float xs[kP] = {lc.x, lc.y, lc.z, lc.w};
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                const float x = xs[p] * Tf - 0.5f;
                if (x > -1.f && x < Tf) {
                    const float xf = floorf(x);
                    key[k][p] = (int)xf + 1;
                    lwv[k][p] = x - xf;
                    atomicAdd(&off[key[k][p]], 1);
                }
            }
        }
    }
    __syncthreads();
    // G4: rows whose two buckets (t: high corner, t + 1: low corner) are both empty get no sample: zeros, written
    // here from the bucket counts so that the stores drain while the scan and the scatter run (written after the
    // scatter they were the decoder's longest phase: PDVC_VAL_ABLATE=3/4, sort 234 and walk-without-gathers 690 of
    // 799 us).  First query chunk only; later chunks add into what the first wrote.  Every other row is written by
    // the walk.
    if constexpr (G4 && ABL != 1) {
        if (!accumulate) {
            float* obz = grad_value + ((size_t)b * S + st) * M * D + (size_t)m * D + (lane & 15) * 4;
            uint16_t* obz16 = B16 ? gv16 + ((size_t)b * S + st) * M * D + (size_t)m * D + (lane & 15) * 4 : nullptr;
            for (int t = threadIdx.x >> 4; t < T; t += blockDim.x >> 4)
                if (off[t] == 0 && off[t + 1] == 0) {
                    *reinterpret_cast<float4*>(obz + (size_t)t * M * D) = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (B16) *reinterpret_cast<uint2*>(obz16 + (size_t)t * M * D) = make_uint2(0u, 0u);
                }
        }
    }
    // 2) exclusive scan of off[0 .. T+1] (off[T+1] = 0 before, total after): per-thread chunks + wave scan
    {
        const int len = T + 2;
        const int per = (len + blockDim.x - 1) / blockDim.x;
        const int i0 = threadIdx.x * per;
        int tot = 0;
        for (int i = i0; i < i0 + per && i < len; ++i) tot += off[i];
        int inc = tot;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(inc, d, 64);
            if (lane >= d) inc += y;
        }
        if (lane == 63) wsum[wid] = inc;
        __syncthreads();
        int base = 0;
        for (int w = 0; w < wid; ++w) base += wsum[w];
        int run = base + inc - tot;
        for (int i = i0; i < i0 + per && i < len; ++i) {
            const int c = off[i];
            off[i] = run;
            cur[i] = run;
            run += c;
        }
    }
    __syncthreads();
    // 3) scatter the samples into bucket order with their two corner coefficients
#pragma unroll
    for (int k = 0; k < kVQPT; ++k) {
        const int qi = spread ? (k == 0 ? (int)threadIdx.x : nq) : (int)threadIdx.x * kVQPT + k;
        if (qi < nq) {
            const float4 at = *reinterpret_cast<const float4*>(save_attn + sbase + (size_t)qi * kP);
            const float as[kP] = {at.x, at.y, at.z, at.w};
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                if (key[k][p] >= 0) {
                    const int pos = atomicAdd(&cur[key[k][p]], 1);
                    const float lo = (1.f - lwv[k][p]) * as[p], hi = lwv[k][p] * as[p];
                    if constexpr (G4) {
                        eqk[pos] = ((uint32_t)key[k][p] << 16) | (uint32_t)(q0 + qi);
                        ew[pos] = make_float2(lo, hi);
                    } else {
                        sq[pos] = q0 + qi;
                        clo[pos] = lo;
                        chi[pos] = hi;
                    }
                }
            }
        }
    }
    __syncthreads();
    if constexpr (ABL == 1) {  // keep the sort live: one word of it leaves the workgroup
        if (threadIdx.x == 0) grad_value[(size_t)blockIdx.x] = (float)off[T + 1] + __uint_as_float(eqk[0]);
        return;
    }
    // G4: the level's pad mask as ints in the scatter cursors' place (dead now), so that the walk reads it from LDS --
    // a global byte load there waits for every gather and store the wave has outstanding (vmcnt(0))
    const int* mk = cur;
    if constexpr (G4) {
        if (vmask) {
            for (int t = threadIdx.x; t < T; t += blockDim.x) cur[t] = vmask[(size_t)b * S + st + t];
            __syncthreads();
        }
    }
    // 4) row ranges: split points balance the sorted samples over the waves (or 16-lane groups)
    const int total = off[T + 1];
    constexpr int kParts = G4 ? kVW * 4 : kVW;
    auto split = [&](int w) -> int {
        if (w <= 0) return 0;
        if (w >= kParts) return T;
        const int target = (int)(((long)total * w) / kParts);
        int lo = 0, hi = T;  // smallest k in [0, T] with off[k] >= target
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (off[mid] >= target) hi = mid;
            else lo = mid + 1;
        }
        return lo;
    };
    const size_t MD = (size_t)M * D;
    const uint8_t* mrow = vmask ? vmask + (size_t)b * S + st : nullptr;
    constexpr int U = 8;
    if constexpr (G4) {
        // (rows no sample touches were zeroed right after the histogram, above)
        const int gl = lane & 15;
        float* ob = grad_value + ((size_t)b * S + st) * MD + (size_t)m * D + gl * 4;
        // bf16 mode: the rounding of every row written, at the same offsets (the value projection's operand)
        uint16_t* ob16 = B16 ? gv16 + ((size_t)b * S + st) * MD + (size_t)m * D + gl * 4 : nullptr;
        // walk: 16-lane group vg owns rows [r0, r1) and reads buckets r0 .. r1; one sorted entry and one gathered
        // gradient row per sample, two running rows (key - 1 and key), each row written once when its last bucket
        // has passed -- no per-row search, at most two row writes per change of key
        const int vg = wid * 4 + (lane >> 4);
        const int r0 = split(vg), r1 = split(vg + 1);
        const int jb = off[r0], je = off[r1 + 1];
        float4 psum = make_float4(0.f, 0.f, 0.f, 0.f);  // this chunk's contributions to the group's rows
        if (r0 < r1 && jb < je) {  // per-group control flow below: no cross-lane operations
            const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(gout + (size_t)b * Lq * MD), (short)0, (int)((size_t)Lq * MD * 4), 0x00020000);
            const int coff = (m * D + gl * 4) * 4, rowb = (int)MD * 4;
            const unsigned MDu = (unsigned)MD;  // < 2^24: the row offset is one v_mul_u32_u24 (a 64-bit one cost ~6 VALU)
            auto put = [&](int r, float4 v) {
                if (r >= r0 && r < r1) {
                    float4* orow = reinterpret_cast<float4*>(ob + __umul24((unsigned)r, MDu));
                    if (mrow && mk[r]) v = make_float4(0.f, 0.f, 0.f, 0.f);
                    psum.x += v.x;
                    psum.y += v.y;
                    psum.z += v.z;
                    psum.w += v.w;
                    if (accumulate) {
                        const float4 o = *orow;
                        v.x += o.x;
                        v.y += o.y;
                        v.z += o.z;
                        v.w += o.w;
                    }
                    *orow = v;
                    if (B16) store_bf16x4(ob16 + (size_t)r * MD, v.x, v.y, v.z, v.w);
                }
            };
            int k = (int)(eqk[jb] >> 16);
            PAcc4 alo = pacc_zero(), ahi = pacc_zero();  // rows k - 1 and k
            for (int j0 = jb; j0 < je; j0 += UG) {
                uint32_t e[UG];
                pf4 gv[UG];
#pragma unroll
                for (int u = 0; u < UG; ++u) e[u] = eqk[(j0 + u < je) ? j0 + u : je - 1];
#pragma unroll
                for (int u = 0; u < UG; ++u) {
                    if constexpr (ABL == 2) {
                        gv[u] = pf4{__uint_as_float(e[u]), 0.f, 0.f, 0.f};
                    } else {
                        const auto t =
                            __builtin_amdgcn_raw_buffer_load_b128(gr, (int)__umul24(e[u] & 0xffffu, (unsigned)rowb) + coff, 0, 0);
                        gv[u] = __builtin_bit_cast(pf4, t);
                    }
                }
#pragma unroll
                for (int u = 0; u < UG; ++u) {
                    if (j0 + u >= je) break;
                    const int kj = (int)(e[u] >> 16);
                    if (kj != k) {  // bucket k complete: row k - 1 final; row k too unless bucket k + 1 follows
                        put(k - 1, pacc_f4(alo));
                        if (kj == k + 1) {
                            alo = ahi;
                        } else {
                            put(k, pacc_f4(ahi));
                            alo = pacc_zero();
                        }
                        ahi = pacc_zero();
                        k = kj;
                    }
                    const float2 wgt = ew[j0 + u];
                    pacc_fma(alo, wgt.x, gv[u]);
                    pacc_fma(ahi, wgt.y, gv[u]);
                }
            }
            put(k - 1, pacc_f4(alo));
            put(k, pacc_f4(ahi));
        }
        if (level_sums) {  // the bias gradient's partial: column sums of the rows this workgroup wrote
#pragma unroll
            for (int d = 16; d < 64; d <<= 1) {
                psum.x += __shfl_xor(psum.x, d, 64);
                psum.y += __shfl_xor(psum.y, d, 64);
                psum.z += __shfl_xor(psum.z, d, 64);
                psum.w += __shfl_xor(psum.w, d, 64);
            }
            __syncthreads();  // every group's walk is done with the sorted entries: reuse their LDS
            float4* red = reinterpret_cast<float4*>(lds_i);
            if (lane < 16) red[wid * 16 + lane] = psum;
            __syncthreads();
            if (threadIdx.x < 16) {
                float4 t = red[threadIdx.x];
#pragma unroll
                for (int w = 1; w < kVW; ++w) {
                    const float4 u = red[w * 16 + threadIdx.x];
                    t.x += u.x;
                    t.y += u.y;
                    t.z += u.z;
                    t.w += u.w;
                }
                float4* o = reinterpret_cast<float4*>(level_sums + ((size_t)b * kL + l) * MD + (size_t)m * D) +
                            threadIdx.x;
                if (accumulate) {
                    const float4 u = *o;
                    t.x += u.x;
                    t.y += u.y;
                    t.z += u.z;
                    t.w += u.w;
                }
                *o = t;
            }
        }
        return;
    }
    const int r0 = split(wid), r1 = split(wid + 1);
    if (r0 >= r1) return;
    const float* gb = gout + (size_t)b * Lq * MD + (size_t)m * D;
    float* ob = grad_value + ((size_t)b * S + st) * MD + (size_t)m * D;
    float accp[CW], acch[CW];  // rows k-1 and k
#pragma unroll
    for (int c = 0; c < CW; ++c) accp[c] = acch[c] = 0.f;
    int k = r0;
    auto close_bucket = [&]() {  // bucket k is complete: row k-1 has both its corners
        const int r = k - 1;
        if (r >= r0) {
            const bool zero = mrow && mrow[r];
            float* orow = ob + (size_t)r * MD;
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                const int ch = lane + 64 * c;
                if (ch < D) {
                    float v = zero ? 0.f : accp[c];
                    if (accumulate) v += orow[ch];
                    orow[ch] = v;
                }
            }
        }
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            accp[c] = acch[c];
            acch[c] = 0.f;
        }
        ++k;
    };
    const int jb = off[r0], je = off[r1 + 1];
    for (int j0 = jb; j0 < je; j0 += U) {
        float gv[U][CW];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = (j0 + u < je) ? j0 + u : je - 1;
            const float* gp = gb + (size_t)sq[j] * MD;
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                const int ch = lane + 64 * c;
                gv[u][c] = gp[ch < D ? ch : 0];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + u;
            if (j >= je) break;
            while (j >= off[k + 1]) close_bucket();
            const float cl = clo[j], chh = chi[j];
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                accp[c] = fmaf(cl, gv[u][c], accp[c]);
                acch[c] = fmaf(chh, gv[u][c], acch[c]);
            }
        }
    }
    while (k <= r1) close_bucket();
}

// -------------------------------------------------------------------------------------------------
// The drop-in operator's 1-D fast path.  A reference user who keeps the stock MSDeformAttn module calls
// MultiScaleDeformableAttention.ms_deform_attn_forward/backward (pdvc/ops/src/vision.cpp:13-16) with PDVC's lifted
// pyramid: spatial_shapes [[1, T_l]] for every level (pdvc/ops/modules/ms_deform_attn.py:114-117), sampling
// locations (N, Lq, M, L, P, 2) and softmaxed weights (N, Lq, M, L, P).  The level table lives in device memory, so
// these kernels read it themselves (a few scalar loads) and run only when it is such a pyramid -- 4 levels, every
// H == 1, W > 0, the start index the prefix sum of W, sum W == S; the general 2-D kernels (msda_op.hip) take
// every other table.  No host read of spatial_shapes: the dispatch is a device-side branch on both paths.
// At H = 1 the y coordinate still matters (.cuh:34-85 with height 1): h = y - 0.5 must lie in (-1, 1), and exactly
// one row corner is in range -- row 0 as h_low (weight 1 - h, d/dh = -1) for h >= 0, as h_high (weight 1 + h,
// d/dh = +1) below -- so a sample is the 1-D sample scaled by fy = 1 - |h|.  PDVC passes y = 0.5: fy = 1.
// -------------------------------------------------------------------------------------------------
// the whole-pyramid drop-in kernels' condition: each staging phase fits the guarded 512-row layout (pick_pyr's)
__device__ __forceinline__ bool dropin_pyr_fits(const Levels1d& lv) {
    return lv.T[0] <= kPyrRows && lv.T[1] + lv.T[2] + lv.T[3] <= kPyrRows;
}

struct DropinSample {
    int roff;         // byte offset of corner row x0 inside the video's value rows
    int i0;           // corner row x0 within the level (in [-1, T - 1] inside, 0 outside)
    float lw, fy, sy; // fraction of x, the row-corner factor, d(fy)/dh
    float a;          // attention weight
    bool ok1, ok2;    // corners x0, x0 + 1 in range (the sample inside its level in x and y)
};

__device__ __forceinline__ DropinSample dropin_sample(float lx, float ly, float a, int T, int st, int MD) {
    DropinSample s;
    const float Tf = (float)T;
    const float x = lx * Tf - 0.5f;  // w_im (.cuh:283-284)
    const float h = ly - 0.5f;       // h_im at height 1
    const bool inside = x > -1.f && x < Tf && h > -1.f && h < 1.f;
    const float xf = floorf(inside ? x : 0.f);
    const int i0 = (int)xf;
    s.lw = inside ? x - xf : 0.f;
    s.fy = inside ? (h >= 0.f ? 1.f - h : 1.f + h) : 0.f;
    s.sy = inside ? (h >= 0.f ? -1.f : 1.f) : 0.f;
    s.ok1 = inside && i0 >= 0;
    s.ok2 = inside && i0 + 1 <= T - 1;
    s.roff = (st + i0) * (MD * 4);  // a corner below the video's rows reads 0 through the buffer range check
    s.i0 = i0;
    s.a = a;
    return s;
}

// forward: msda1d_fwd_buf_kernel's mapping (one wave per 4 queries of one (video, head), 16 lanes x float4 per query,
// lane j owns sample j for the parameter phase), reading the drop-in layout's locations and weights
__global__ __launch_bounds__(256) void msda_dropin_fwd_kernel(const float* __restrict__ value,
                                                              const int64_t* __restrict__ shapes,
                                                              const int64_t* __restrict__ lsi,
                                                              const float* __restrict__ loc,
                                                              const float* __restrict__ attn, int Lq, int S, int M,
                                                              int total_waves, int pyr_first,
                                                              float* __restrict__ out) {
    constexpr int D = 64;
    Levels1d lv;
    if (!dropin_levels(shapes, lsi, S, lv)) return;  // a 2-D table: msda2d_fwd_kernel's
    if (pyr_first && dropin_pyr_fits(lv)) return;    // msda_dropin_fwd_pyr_kernel's
    const int lane = threadIdx.x & 63;
    const int wave0 = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
    // one wave per 4 queries of one (video, head); grid-strided, so that after a pyramid launch (pyr_first) a small
    // grid retires at once when the pyramid took the call
    for (int wave = wave0; wave < total_waves; wave += 4 * (int)gridDim.x) {
        const WaveQuery w = wave_query<16>(wave, lane, Lq, M);
        const int MD = M * D;
        const int j = w.sub, l_own = j >> 2;
        const size_t si = ((size_t)w.row * M + w.m) * kNS + j;  // (N, Lq, M, L, P) index of this lane's sample
        const float2 lc = *reinterpret_cast<const float2*>(loc + 2 * si);
        const DropinSample sm = dropin_sample(lc.x, lc.y, attn[si], lvl_sel(lv.T, l_own), lvl_sel(lv.start, l_own), MD);
        const float w1 = sm.ok1 ? ((1.f - sm.lw) * sm.fy) * sm.a : 0.f, w2 = sm.ok2 ? (sm.lw * sm.fy) * sm.a : 0.f;
        const int coff = (w.m * D + w.sub * 4) * 4;
        const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(value + (size_t)__builtin_amdgcn_readfirstlane(w.b) * S * MD), (short)0, S * MD * 4, 0x00020000);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    #pragma unroll
        for (int l = 0; l < kL; ++l) {
            int rl = sm.roff;
            float wl1 = w1, wl2 = w2;
            __asm__ volatile("" : "+v"(rl), "+v"(wl1), "+v"(wl2) : "v"(acc.x), "v"(acc.y), "v"(acc.z), "v"(acc.w));
            float4 v1[kP], v2[kP];
            float c1[kP], c2[kP];
    #pragma unroll
            for (int p = 0; p < kP; ++p) {
                const int o = grp_bcast<16>(rl, l * kP + p) + coff;
                c1[p] = grp_bcast<16>(wl1, l * kP + p);
                c2[p] = grp_bcast<16>(wl2, l * kP + p);
                const auto u1 = __builtin_amdgcn_raw_buffer_load_b128(vr, o, 0, 0);
                const auto u2 = __builtin_amdgcn_raw_buffer_load_b128(vr, o + MD * 4, 0, 0);
                v1[p] = make_float4(__uint_as_float(u1[0]), __uint_as_float(u1[1]), __uint_as_float(u1[2]),
                                    __uint_as_float(u1[3]));
                v2[p] = make_float4(__uint_as_float(u2[0]), __uint_as_float(u2[1]), __uint_as_float(u2[2]),
                                    __uint_as_float(u2[3]));
            }
    #pragma unroll
            for (int p = 0; p < kP; ++p) {
                acc.x = fmaf(c1[p], v1[p].x, acc.x);
                acc.y = fmaf(c1[p], v1[p].y, acc.y);
                acc.z = fmaf(c1[p], v1[p].z, acc.z);
                acc.w = fmaf(c1[p], v1[p].w, acc.w);
                acc.x = fmaf(c2[p], v2[p].x, acc.x);
                acc.y = fmaf(c2[p], v2[p].y, acc.y);
                acc.z = fmaf(c2[p], v2[p].z, acc.z);
                acc.w = fmaf(c2[p], v2[p].w, acc.w);
            }
        }
        if (w.active)
            *reinterpret_cast<float4*>(out + (size_t)w.row * MD + (size_t)w.m * D + w.sub * 4) = acc;
    }
}

// backward, query side: msda1d_bwd_query_dot_kernel's dot-product form and reduction; the owner lane writes
// grad_sampling_loc (x, y) and grad_attn_weight in the drop-in layout (.cuh:88-160 at height 1: dL/da = fy * dot,
// dL/dx = W * a * fy * (d2 - d1), dL/dy = a * sy * dot with dot = hw * d1 + lw * d2 over the corners in range), and
// the level-major (location x, a * fy) slab the value-gradient kernel sorts
__global__ __launch_bounds__(256) void msda_dropin_bwd_query_kernel(
    const float* __restrict__ value, const int64_t* __restrict__ shapes, const int64_t* __restrict__ lsi,
    const float* __restrict__ loc, const float* __restrict__ attn, int Lq, int S, int M, int total_waves,
    int pyr_first, const float* __restrict__ gout, float* __restrict__ grad_loc, float* __restrict__ grad_attn,
    float* __restrict__ save_attn, float* __restrict__ save_loc) {
    constexpr int D = 64;
    Levels1d lv;
    if (!dropin_levels(shapes, lsi, S, lv)) return;
    if (pyr_first && dropin_pyr_fits(lv)) return;  // msda_dropin_bwd_query_pyr_kernel's
    const int lane = threadIdx.x & 63;
    const int wave0 = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
    // one wave per 4 queries of one (video, head); grid-strided, so that after a pyramid launch (pyr_first) a small
    // grid retires at once when the pyramid took the call
    for (int wave = wave0; wave < total_waves; wave += 4 * (int)gridDim.x) {
        const WaveQuery w = wave_query<16>(wave, lane, Lq, M);
        const int MD = M * D;
        const int c0 = w.sub * 4;
        const int j = w.sub, l_own = j >> 2;
        const int T_own = lvl_sel(lv.T, l_own);
        const size_t si = ((size_t)w.row * M + w.m) * kNS + j;
        const float2 lc = *reinterpret_cast<const float2*>(loc + 2 * si);
        const DropinSample sm = dropin_sample(lc.x, lc.y, attn[si], T_own, lvl_sel(lv.start, l_own), MD);
        if (w.active) {
            const size_t vi = save_index(w.b, w.m, l_own, w.q, j & 3, Lq, M);
            save_loc[vi] = lc.x;
            save_attn[vi] = sm.a * sm.fy;
        }
        const int coff = (w.m * D + c0) * 4;
        const float4 g = *reinterpret_cast<const float4*>(gout + (size_t)w.row * MD + (size_t)w.m * D + c0);
        const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(value + (size_t)__builtin_amdgcn_readfirstlane(w.b) * S * MD), (short)0, S * MD * 4, 0x00020000);
        float d1 = 0.f, d2 = 0.f;
    #pragma unroll
        for (int l = 0; l < kL; ++l) {
            float part[8];
    #pragma unroll
            for (int p = 0; p < kP; ++p) {
                const int off = grp_bcast<16>(sm.roff, l * kP + p) + coff;
                const auto u1 = __builtin_amdgcn_raw_buffer_load_b128(vr, off, 0, 0);
                const auto u2 = __builtin_amdgcn_raw_buffer_load_b128(vr, off + MD * 4, 0, 0);
                part[p] = g.x * __uint_as_float(u1[0]) + g.y * __uint_as_float(u1[1]) + g.z * __uint_as_float(u1[2]) +
                          g.w * __uint_as_float(u1[3]);
                part[4 + p] = g.x * __uint_as_float(u2[0]) + g.y * __uint_as_float(u2[1]) +
                              g.z * __uint_as_float(u2[2]) + g.w * __uint_as_float(u2[3]);
            }
            const bool u8 = (lane & 8) != 0;
    #pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float send = u8 ? part[i] : part[i + 4];
                const float mine = u8 ? part[i + 4] : part[i];
                part[i] = mine + grp_swap(send, 8);
            }
            const bool u2b = (lane & 2) != 0;
    #pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float send = u2b ? part[i] : part[i + 2];
                const float mine = u2b ? part[i + 2] : part[i];
                part[i] = mine + grp_swap(send, 2);
            }
            const bool u1b = (lane & 1) != 0;
            const float send = u1b ? part[0] : part[1];
            const float mine = u1b ? part[1] : part[0];
            part[0] = mine + grp_swap(send, 1);
            part[0] += grp_swap(part[0], 4);
            const float other = grp_swap(part[0], 8);
            if (l_own == l) {
                d1 = (l < 2) ? part[0] : other;
                d2 = (l < 2) ? other : part[0];
            }
        }
        const float x1 = sm.ok1 ? d1 : 0.f, x2 = sm.ok2 ? d2 : 0.f;
        const float dot = (1.f - sm.lw) * x1 + sm.lw * x2;
        if (w.active) {
            grad_attn[si] = sm.fy * dot;
            *reinterpret_cast<float2*>(grad_loc + 2 * si) =
                make_float2((float)T_own * ((sm.a * sm.fy) * (x2 - x1)), sm.a * (sm.sy * dot));
        }
    }
}

// -------------------------------------------------------------------------------------------------
// The drop-in operator's encoder-shaped calls (4 Lq >= S: each position is sampled many times) on the whole-pyramid
// kernels, as the product path's encoder runs: the head's value rows staged in LDS and every corner row read from
// there (msda1d_fwd_pyr2_kernel's LDS-DMA staging; msda1d_bwd_query_pyr_kernel's two phases), the parameter phase
// reading the drop-in layout (locations (N, Lq, M, L, P, 2), softmaxed weights) and the level table read on the
// device.  They return without work when the table is not a lifted 1-D pyramid or a staging phase would not fit
// (dropin_pyr_fits); the L2-gather kernels above, launched after them with pyr_first = 1, take exactly those calls.
// -------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kPyrThreads) void msda_dropin_fwd_pyr_kernel(
    const float* __restrict__ value, const int64_t* __restrict__ shapes, const int64_t* __restrict__ lsi,
    const float* __restrict__ loc, const float* __restrict__ attn, int Lq, int S, int M, int qblocks,
    float* __restrict__ out) {
    Levels1d lv;
    if (!dropin_levels(shapes, lsi, S, lv) || !dropin_pyr_fits(lv)) return;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    const int blk = xcd_remap(blockIdx.x, gridDim.x);  // the query blocks and heads of a video share an XCD
    const int qb = blk % qblocks, bm = blk / qblocks;
    const int b = bm / M, m = bm - b * M;
    const int slot = threadIdx.x >> 4, sub = threadIdx.x & 15;
    const size_t MD = (size_t)M * 64;
    const float* vsrc = value + (size_t)b * S * MD + (size_t)m * 64;
    const char* lrow = reinterpret_cast<const char*>(lds4) + sub * 16;
    const int n0 = lv.T[0], n1 = lv.T[1] + lv.T[2] + lv.T[3];
    const bool single = n0 + n1 + 2 <= kLdsRows;
    const int p2 = single ? 1 + n0 : kLdsRows - 1 - n1;  // LDS row of level 1's first position
    pyr_zero_row(lds4, 0, 0);
    pyr_zero_row(lds4, single ? n0 + n1 + 1 : n0 + 1, 64);
    if (!single) pyr_zero_row(lds4, kLdsRows - 1, 128);
    const int l_own = sub >> 2;
    const int T_own = lvl_sel(lv.T, l_own), st_own = lvl_sel(lv.start, l_own);
    const int base_own = l_own == 0 ? 1 : p2 + (st_own - lv.start[1]);
    float2 lcv[kPyrQPS];
    float av[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        const size_t si = (((size_t)b * Lq + (q < Lq ? q : 0)) * M + m) * kNS + sub;
        lcv[i] = *reinterpret_cast<const float2*>(loc + 2 * si);
        av[i] = attn[si];
    }
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): the parameters before the DMAs (msda1d_fwd_pyr2_kernel)
    pyr_dma_rows(lds4, vsrc, MD, lv.start[0], 1, single ? n0 + n1 : n0);
    int adv[kPyrQPS];
    float w1v[kPyrQPS], w2v[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {  // msda_dropin_fwd_kernel's corner weights, bit for bit
        const DropinSample sm = dropin_sample(lcv[i].x, lcv[i].y, av[i], T_own, 0, 0);
        adv[i] = pyr_corner(base_own, sm.i0);
        w1v[i] = sm.ok1 ? ((1.f - sm.lw) * sm.fy) * sm.a : 0.f;
        w2v[i] = sm.ok2 ? (sm.lw * sm.fy) * sm.a : 0.f;
    }
    PAcc4 acc[kPyrQPS];
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) acc[i] = pacc_zero();
    PAcc4 tok = pacc_zero();
    auto level = [&](auto Lc) {
        constexpr int L = decltype(Lc)::value;
#pragma unroll
        for (int i = 0; i < kPyrQPS; ++i) {
            pf4 v1[kP], v2[kP];
            float c1[kP], c2[kP];
            int ad = adv[i];
            float wa = w1v[i], wb = w2v[i];
            __asm__ volatile("" : "+v"(ad), "+v"(wa), "+v"(wb) : "v"(tok.lo), "v"(tok.hi));
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                const char* r = lrow + grp_bcast<16>(ad, L * kP + p);
                c1[p] = grp_bcast<16>(wa, L * kP + p);
                c2[p] = grp_bcast<16>(wb, L * kP + p);
                v1[p] = *reinterpret_cast<const pf4*>(r);
                v2[p] = *reinterpret_cast<const pf4*>(r + 256);
            }
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                pacc_fma(acc[i], c1[p], v1[p]);
                pacc_fma(acc[i], c2[p], v2[p]);
            }
            tok = acc[i];
        }
    };
    __syncthreads();
    if (single) {
        level(std::integral_constant<int, 0>{});
        level(std::integral_constant<int, 1>{});
        level(std::integral_constant<int, 2>{});
        level(std::integral_constant<int, 3>{});
    } else {
        const int pre = n0 + 2 > p2 ? n0 + 2 - p2 : 0;
        pyr_dma_rows_async(lds4, vsrc, MD, lv.start[1] + pre, p2 + pre, n1 - pre);
        level(std::integral_constant<int, 0>{});
        pyr_dma_wait();
        __syncthreads();
        pyr_zero_row(lds4, p2 - 1, 0);
        pyr_dma_rows(lds4, vsrc, MD, lv.start[1], p2, pre);
        __syncthreads();
        level(std::integral_constant<int, 1>{});
        level(std::integral_constant<int, 2>{});
        level(std::integral_constant<int, 3>{});
    }
#pragma unroll
    for (int i = 0; i < kPyrQPS; ++i) {
        const int q = qb * kPyrQ + slot + 64 * i;
        if (q < Lq)
            *reinterpret_cast<float4*>(out + ((size_t)b * Lq + q) * MD + (size_t)m * 64 + sub * 4) = pacc_f4(acc[i]);
    }
}

// backward, query side: msda1d_bwd_query_pyr_kernel's staging (level 0, then levels 1..3) and dot-product reduction;
// each phase's owner lanes write grad_attn and grad_loc of their samples in the drop-in layout (msda_dropin_bwd_query_
// kernel's owner math: no softmax here, so nothing is carried between the phases), and the first phase writes the
// level-major (location x, a * fy) slab of every sample for the value-gradient kernel
// Each query's global inputs (dOut row, location pair, weight) are loaded during the previous query, before its stores,
// and the stores are unconditional buffer stores (an inactive lane's offset is past the descriptor's range, which drops
// it): vmcnt counts loads and stores together in issue order, so inputs loaded after a query's stores would wait for
// their write acknowledgements, and a store under a branch leaves hipcc a store-less path to count by, so it waits for
// everything.  740 -> 719 us per launch at 256 videos (profiles/r04_vmcnt_store_coupling.txt).
__global__ __launch_bounds__(kPyrThreads) void msda_dropin_bwd_query_pyr_kernel(
    const float* __restrict__ value, const int64_t* __restrict__ shapes, const int64_t* __restrict__ lsi,
    const float* __restrict__ loc, const float* __restrict__ attn, int Lq, int S, int M, int qblocks,
    const float* __restrict__ gout, float* __restrict__ grad_loc, float* __restrict__ grad_attn,
    float* __restrict__ save_attn, float* __restrict__ save_loc) {
    Levels1d lv;
    if (!dropin_levels(shapes, lsi, S, lv) || !dropin_pyr_fits(lv)) return;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int qb = blk % qblocks, bm = blk / qblocks;
    const int b = bm / M, m = bm - b * M;
    const int slot = threadIdx.x >> 4, sub = threadIdx.x & 15, lane = threadIdx.x & 63;
    const int MD = M * 64;
    const float* vsrc = value + (size_t)b * S * MD + (size_t)m * 64;
    const int l_own = sub >> 2, p_own = sub & 3;
    const int T_own = lvl_sel(lv.T, l_own);
    const float Tf = (float)T_own;
    const int base_own = pyr_base(lv, l_own);
    const char* lrow = reinterpret_cast<const char*>(lds4) + sub * 16;

    float4 pg;  // the next query's inputs
    float2 plc;
    float pat;
    auto fetch = [&](int iq) {
        const int q0 = qb * kBqQ + slot + 64 * iq;
        const size_t row = (size_t)b * Lq + (q0 < Lq ? q0 : Lq - 1);
        pg = *reinterpret_cast<const float4*>(gout + row * MD + (size_t)m * 64 + sub * 4);
        const size_t si = (row * M + m) * kNS + sub;
        plc = *reinterpret_cast<const float2*>(loc + 2 * si);
        pat = attn[si];
    };
    // stores: one video's rows per descriptor; an inactive lane's offset is the descriptor's size (dropped)
    const int ga_bytes = Lq * M * kNS * 4, sv_bytes = kL * Lq * kP * 4;
    const __amdgpu_buffer_rsrc_t gar = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(grad_attn + (size_t)b * Lq * M * kNS), (short)0, ga_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t glr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(grad_loc + 2 * (size_t)b * Lq * M * kNS), (short)0, 2 * ga_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t slr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(save_loc + save_index(b, m, 0, 0, 0, Lq, M)), (short)0, sv_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t sar = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(save_attn + save_index(b, m, 0, 0, 0, Lq, M)), (short)0, sv_bytes, 0x00020000);
    auto run_query = [&](int iq, auto L0c, auto L1c) {
        constexpr int L0 = decltype(L0c)::value, L1 = decltype(L1c)::value;
        const int q0 = qb * kBqQ + slot + 64 * iq;
        const bool act = q0 < Lq;
        const int q = act ? q0 : Lq - 1;
        const float4 g = pg;
        const float2 lc = plc;
        const DropinSample sm = dropin_sample(lc.x, lc.y, pat, T_own, 0, 0);
        const int ad = pyr_corner(base_own, sm.i0);
        float d1 = 0.f, d2 = 0.f;
        const pf2 gxy = {g.x, g.y}, gzw = {g.z, g.w};
#pragma unroll
        for (int L = L0; L < L1; ++L) {
            float part[8];
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                const char* r = lrow + grp_bcast<16>(ad, L * kP + p);
                const pf4 u1 = *reinterpret_cast<const pf4*>(r);
                const pf4 u2 = *reinterpret_cast<const pf4*>(r + 256);
                const pf2 t1 = __builtin_elementwise_fma(gzw, u1.zw, gxy * u1.xy);
                const pf2 t2 = __builtin_elementwise_fma(gzw, u2.zw, gxy * u2.xy);
                part[p] = t1.x + t1.y;
                part[4 + p] = t2.x + t2.y;
            }
            const bool u8 = (lane & 8) != 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float send = u8 ? part[k] : part[k + 4];
                const float mine = u8 ? part[k + 4] : part[k];
                part[k] = mine + grp_swap(send, 8);
            }
            const bool u2b = (lane & 2) != 0;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const float send = u2b ? part[k] : part[k + 2];
                const float mine = u2b ? part[k + 2] : part[k];
                part[k] = mine + grp_swap(send, 2);
            }
            const bool u1b = (lane & 1) != 0;
            const float send = u1b ? part[0] : part[1];
            const float mine = u1b ? part[1] : part[0];
            part[0] = mine + grp_swap(send, 1);
            part[0] += grp_swap(part[0], 4);
            const float other = grp_swap(part[0], 8);
            if (l_own == L) {
                d1 = (L < 2) ? part[0] : other;
                d2 = (L < 2) ? other : part[0];
            }
        }
        fetch(iq + 1 < kBqQPS ? iq + 1 : 0);  // after every use of g, before the stores
        const int ls = (l_own * Lq + q) * kP + p_own;  // save slab offset inside (b, m)
        if (L0 == 0) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lc.x), slr, act ? ls * 4 : sv_bytes, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sm.a * sm.fy), sar, act ? ls * 4 : sv_bytes, 0, 0);
        }
        const bool st = act && l_own >= L0 && l_own < L1;
        const float x1 = sm.ok1 ? d1 : 0.f, x2 = sm.ok2 ? d2 : 0.f;
        const float dot = (1.f - sm.lw) * x1 + sm.lw * x2;
        const int li = (q * M + m) * kNS + sub;  // sample index inside the video
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sm.fy * dot), gar, st ? li * 4 : ga_bytes, 0, 0);
        using u2 = unsigned int __attribute__((ext_vector_type(2)));
        const u2 glv = u2{__float_as_uint(Tf * ((sm.a * sm.fy) * (x2 - x1))), __float_as_uint(sm.a * (sm.sy * dot))};
        __builtin_amdgcn_raw_buffer_store_b64(glv, glr, st ? li * 8 : 2 * ga_bytes, 0, 0);
    };
    fetch(0);

    pyr_stage_g(lds4, vsrc, MD, lv.start[0], lv.T[0]);
    __syncthreads();
#pragma unroll 1
    for (int i = 0; i < kBqQPS; ++i) run_query(i, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
    __syncthreads();
    pyr_stage_g(lds4, vsrc, MD, lv.start[1], lv.T[1] + lv.T[2] + lv.T[3]);
    __syncthreads();
#pragma unroll 1
    for (int i = 0; i < kBqQPS; ++i) run_query(i, std::integral_constant<int, 1>{}, std::integral_constant<int, 4>{});
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
    int cpl, lph;
};

// waves of the query-tile mapping: one per (video, head, group of 64/LPH queries)
static long query_waves(const Geometry& g, int batch, int num_heads, int num_query) {
    const int qpw = 64 / g.lph;
    return (long)batch * num_heads * ((num_query + qpw - 1) / qpw);
}

static int pick_geometry(int M, int D, Geometry& g) {
    // 4 channels (one float4) per lane keeps a level's 2*P corner loads in flight within the register budget
    // of 4 waves/SIMD; D = 128 needs 8 per lane (at most 16 lanes per head).
    if (D == 16 || D == 32 || D == 64) g.cpl = 4;
    else if (D == 128) g.cpl = 8;
    else return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "fused 1-D path supports head_dim 16/32/64/128, got %d", D);
    g.lph = D / g.cpl;
    return PDVC_OK;
}

// Query blocks for the whole-pyramid kernels, or 0 when they do not apply: D = 64, enough queries per
// (video, head) to amortise staging the head's value rows (4 * Lq >= S: the encoder, Lq == S), level 0 and
// levels 1..3 each within the 512-row LDS buffer.  PDVC_MSDA_PYR=0 in the environment turns them off (A/B).
static int pick_pyr(const Levels1d& lv, int S, int num_query, int head_dim, int per_block) {
    static const int enabled = [] {
        const char* e = getenv("PDVC_MSDA_PYR");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    if (!enabled || head_dim != 64 || num_query <= 0 || 4L * num_query < S) return 0;
    if (lv.T[0] > kPyrRows || lv.T[1] + lv.T[2] + lv.T[3] > kPyrRows) return 0;
    return (num_query + per_block - 1) / per_block;
}

// value-gradient walk depth (PDVC_VALUE_UG=4 / 8 forces it): 4 where a level holds few samples per row (the
// decoder, 4 * Lq < S: its workgroups' LDS is small, so the 66-VGPR form fits more of them per CU -- 206 -> 177 us at
// 256 videos), 8 for the encoder (LDS-limited to two workgroups per CU anyway; 8 in flight: 770 -> 700 us)
// the windowed whole-pyramid kernels (msda1d_fwd_win_kernel) where pick_pyr's staging does not fit: encoder-shaped
// calls (4 Lq >= S) at D = 64 on a pyramid with win_fits; PDVC_MSDA_WIN=0 keeps the L2-gather kernels (A/B)
static bool win_ok(const Levels1d& lv, int num_query, int S, int head_dim) {
    static const bool on = [] {
        const char* e = getenv("PDVC_MSDA_WIN");
        return !(e && e[0] == '0');
    }();
    return on && head_dim == 64 && num_query > 0 && 4L * num_query >= S && win_fits(lv);
}

static int value_ug(int num_query, int S) {
    static const int forced = [] {
        const char* e = getenv("PDVC_VALUE_UG");
        return e ? atoi(e) : 0;
    }();
    if (forced == 4 || forced == 8) return forced;
    return 4L * num_query < S ? 4 : 8;
}

// 16-lane-group gather for the value gradient at D = 64 (PDVC_MSDA_G4=0 selects the wave-per-range form)
static bool value_g4() {
    static const bool on = [] {
        const char* e = getenv("PDVC_MSDA_G4");
        return !(e && e[0] == '0');
    }();
    return on;
}

// backward-query kernel at D = 64: PDVC_MSDA_BWDQ=0 msda1d_bwd_query_kernel, 2 msda1d_bwd_query_dot_kernel
// everywhere, anything else (default) the whole-pyramid twin where it applies (encoder: 630 vs 680 us at 256
// videos, tools/msda_ab.sh) and the dot kernel elsewhere.  PDVC_MSDA_PYR=0 turns both pyramid kernels off.
static int bwdq_mode() {
    static const int mode = [] {
        const char* e = getenv("PDVC_MSDA_BWDQ");
        return (e && e[0] == '0') ? 0 : (e && e[0] == '2') ? 2 : 1;
    }();
    return mode;
}

static int bwdq_pyr_attrs() {
    static std::atomic<int> done[kMaxDevices];
    const int b = (int)kBqLds;
    return lds_optin(done, {{(const void*)msda1d_bwd_query_pyr_kernel<1>, b},
                            {(const void*)msda1d_bwd_query_pyr_kernel<2>, b},
                            {(const void*)msda1d_bwd_query_pyr_kernel<1, 3>, b},
                            {(const void*)msda1d_bwd_query_pyr_kernel<2, 3>, b},
                            {(const void*)msda1d_bwd_query_pyr_kernel<1, 5>, b},
                            {(const void*)msda1d_bwd_query_pyr_kernel<2, 5>, b}},
                     "msda1d_bwd_query_pyr_kernel");
}

// buffer-load forward at D = 64 (PDVC_MSDA_FWDBUF=0 selects the whole-pyramid / per-query kernels: A/B)
static bool fwd_buf() {
    static const bool on = [] {
        const char* e = getenv("PDVC_MSDA_FWDBUF");
        return !(e && e[0] == '0');
    }();
    return on;
}

static int pyr_attrs() {
    static std::atomic<int> done[kMaxDevices];
    return lds_optin(done, {{(const void*)msda1d_fwd_pyr_kernel<1>, (int)kPyrLds},
                            {(const void*)msda1d_fwd_pyr_kernel<2>, (int)kPyrLds},
                            {(const void*)msda1d_fwd_pyr2_kernel<1>, (int)kPyr2LdsMax},
                            {(const void*)msda1d_fwd_pyr2_kernel<2>, (int)kPyr2LdsMax}},
                     "msda1d pyramid kernels");
}

// LDS-DMA pyramid forward (msda1d_fwd_pyr2_kernel; PDVC_PYR_DMA=0 selects msda1d_fwd_pyr_kernel: A/B)
static bool pyr_dma() {
    static const bool on = [] {
        const char* e = getenv("PDVC_PYR_DMA");
        return !(e && e[0] == '0');
    }();
    return on;
}

}  // namespace pdvc

using namespace pdvc;

template <int RD>
static void launch_fwd1d(const Geometry& g, dim3 grid, hipStream_t s, const float* value, const uint8_t* mask,
                         const float* proj, int ps, int ob, int lb, const float* ref, Levels1d lv, int Lq, int S,
                         int M, int D, int tw, float* out, float* sa, float* sl) {
#define ARGS value, mask, proj, ps, ob, lb, ref, lv, Lq, S, M, D, tw, out, sa, sl
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
#define ARGS value, mask, proj, ps, ob, lb, ref, lv, Lq, S, M, D, tw, gout, fout, sa, sl, gp, gr
    if (g.cpl == 8) hipLaunchKernelGGL((msda1d_bwd_query_kernel<8, 16, RD>), grid, dim3(256), 0, s, ARGS);
    else if (g.lph == 4) hipLaunchKernelGGL((msda1d_bwd_query_kernel<4, 4, RD>), grid, dim3(256), 0, s, ARGS);
    else if (g.lph == 8) hipLaunchKernelGGL((msda1d_bwd_query_kernel<4, 8, RD>), grid, dim3(256), 0, s, ARGS);
    else hipLaunchKernelGGL((msda1d_bwd_query_kernel<4, 16, RD>), grid, dim3(256), 0, s, ARGS);
#undef ARGS
}

// out16 (bf16 mode): the output's bf16 rounding beside it -- only on the LDS-DMA pyramid path (the encoder's
// self-attention); any other path returns PDVC_ERR_UNSUPPORTED before launching anything
static int msda1d_forward_impl(const float* value, const uint8_t* value_pad_mask, const float* proj, int proj_stride,
                               int off_base, int logit_base, const float* ref, int ref_dim, const int32_t* level_T,
                               int num_levels, int batch, int num_query, int num_heads, int head_dim, int num_point,
                               float* output, float* save_attn, float* save_loc, uint16_t* out16, void* stream) {
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
    const long tw = query_waves(g, batch, num_heads, num_query);
    if (tw == 0) return PDVC_OK;
    PDVC_CHECK_ARG(tw < (1L << 31) / 4, "too many rows");
    dim3 grid((unsigned)((tw + 3) / 4));
    hipStream_t s = (hipStream_t)stream;
    if (const int qb = pick_pyr(lv, S, num_query, head_dim, kPyrQ)) {
        if ((rc = pyr_attrs())) return rc;
        PDVC_CHECK_ARG((long)batch * num_heads * qb < (1L << 31), "too many query blocks");
        dim3 pg((unsigned)(batch * num_heads * qb));
        if (out16 && !pyr_dma())
            return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "bf16 output only on the LDS-DMA pyramid path");
        static const int ablate = [] {
            const char* e = getenv("PDVC_PYR_ABLATE");
            return e ? atoi(e) : 0;
        }();
        if (ablate >= 1 && ablate <= 3 && ref_dim == 1 && !out16) {  // measurement only (tools/kbench.py)
            const void* k = ablate == 1 ? (const void*)msda1d_fwd_pyr_kernel<1, 1>
                            : ablate == 2 ? (const void*)msda1d_fwd_pyr_kernel<1, 2>
                                          : (const void*)msda1d_fwd_pyr_kernel<1, 3>;
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPyrLds);
            if (ablate == 1)
                hipLaunchKernelGGL((msda1d_fwd_pyr_kernel<1, 1>), pg, dim3(kPyrThreads), kPyrLds, s, value,
                                   value_pad_mask, proj, proj_stride, off_base, logit_base, ref, lv, num_query, S,
                                   num_heads, qb, output, save_attn, save_loc);
            else if (ablate == 3)
                hipLaunchKernelGGL((msda1d_fwd_pyr_kernel<1, 3>), pg, dim3(kPyrThreads), kPyrLds, s, value,
                                   value_pad_mask, proj, proj_stride, off_base, logit_base, ref, lv, num_query, S,
                                   num_heads, qb, output, save_attn, save_loc);
            else
                hipLaunchKernelGGL((msda1d_fwd_pyr_kernel<1, 2>), pg, dim3(kPyrThreads), kPyrLds, s, value,
                                   value_pad_mask, proj, proj_stride, off_base, logit_base, ref, lv, num_query, S,
                                   num_heads, qb, output, save_attn, save_loc);
        } else if (pyr_dma()) {
            const int n_all = lv.T[0] + lv.T[1] + lv.T[2] + lv.T[3] + 2;
            const size_t lds = n_all <= kLdsRows ? (size_t)n_all * 256 : kPyr2LdsMax;
            if (ref_dim == 1)
                hipLaunchKernelGGL((msda1d_fwd_pyr2_kernel<1>), pg, dim3(kPyrThreads), lds, s, value, value_pad_mask,
                                   proj, proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, qb,
                                   output, save_attn, save_loc, out16);
            else
                hipLaunchKernelGGL((msda1d_fwd_pyr2_kernel<2>), pg, dim3(kPyrThreads), lds, s, value, value_pad_mask,
                                   proj, proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, qb,
                                   output, save_attn, save_loc, out16);
        } else if (ref_dim == 1)
            hipLaunchKernelGGL((msda1d_fwd_pyr_kernel<1>), pg, dim3(kPyrThreads), kPyrLds, s, value, value_pad_mask,
                               proj, proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, qb, output,
                               save_attn, save_loc);
        else
            hipLaunchKernelGGL((msda1d_fwd_pyr_kernel<2>), pg, dim3(kPyrThreads), kPyrLds, s, value, value_pad_mask,
                               proj, proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, qb, output,
                               save_attn, save_loc);
        PDVC_CHECK_LAUNCH("msda1d_fwd_pyr_kernel");
        return PDVC_OK;
    }
    if (win_ok(lv, num_query, S, head_dim)) {  // level 0 past one staging phase: two row windows
        static std::atomic<int> done[kMaxDevices];
        if ((rc = lds_optin(done, {{(const void*)msda1d_fwd_win_kernel<1>, (int)kWinLds},
                                   {(const void*)msda1d_fwd_win_kernel<2>, (int)kWinLds}},
                            "msda1d_fwd_win_kernel")))
            return rc;
        const int qb = (num_query + kPyrQ - 1) / kPyrQ;
        PDVC_CHECK_ARG((long)batch * num_heads * qb < (1L << 31), "too many query blocks");
        dim3 pg((unsigned)(batch * num_heads * qb));
        if (ref_dim == 1)
            hipLaunchKernelGGL((msda1d_fwd_win_kernel<1>), pg, dim3(kPyrThreads), kWinLds, s, value, value_pad_mask,
                               proj, proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, qb, output,
                               save_attn, save_loc, out16);
        else
            hipLaunchKernelGGL((msda1d_fwd_win_kernel<2>), pg, dim3(kPyrThreads), kWinLds, s, value, value_pad_mask,
                               proj, proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, qb, output,
                               save_attn, save_loc, out16);
        PDVC_CHECK_LAUNCH("msda1d_fwd_win_kernel");
        return PDVC_OK;
    }
    if (out16) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "bf16 output only on the LDS-DMA pyramid path");
    if (head_dim == 64 && fwd_buf() && (long)S * num_heads * head_dim * 4 < (1L << 31)) {
        if (ref_dim == 1)
            hipLaunchKernelGGL((msda1d_fwd_buf_kernel<1>), grid, dim3(256), 0, s, value, value_pad_mask, proj,
                               proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, (int)tw, output,
                               save_attn, save_loc);
        else
            hipLaunchKernelGGL((msda1d_fwd_buf_kernel<2>), grid, dim3(256), 0, s, value, value_pad_mask, proj,
                               proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, (int)tw, output,
                               save_attn, save_loc);
        PDVC_CHECK_LAUNCH("msda1d_fwd_buf_kernel");
        return PDVC_OK;
    }
    if (ref_dim == 1)
        launch_fwd1d<1>(g, grid, s, value, value_pad_mask, proj, proj_stride, off_base, logit_base, ref, lv, num_query,
                        S, num_heads, head_dim, (int)tw, output, save_attn, save_loc);
    else
        launch_fwd1d<2>(g, grid, s, value, value_pad_mask, proj, proj_stride, off_base, logit_base, ref, lv, num_query,
                        S, num_heads, head_dim, (int)tw, output, save_attn, save_loc);
    PDVC_CHECK_LAUNCH("msda1d_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_level_pos_rows_backward_f32(const float* dpos, const int32_t* level_T, int num_levels, int N,
                                                int S, int C, float* partials, void* stream);

extern "C" int pdvc_msda1d_forward_f32(const float* value, const uint8_t* value_pad_mask, const float* proj,
                                       int proj_stride, int off_base, int logit_base, const float* ref, int ref_dim,
                                       const int32_t* level_T, int num_levels, int batch, int num_query,
                                       int num_heads, int head_dim, int num_point, float* output, float* save_attn,
                                       float* save_loc, void* stream) {
    return msda1d_forward_impl(value, value_pad_mask, proj, proj_stride, off_base, logit_base, ref, ref_dim, level_T,
                               num_levels, batch, num_query, num_heads, head_dim, num_point, output, save_attn,
                               save_loc, nullptr, stream);
}

extern "C" int pdvc_msda1d_forward_f32_bf16out(const float* value, const uint8_t* value_pad_mask, const float* proj,
                                               int proj_stride, int off_base, int logit_base, const float* ref,
                                               int ref_dim, const int32_t* level_T, int num_levels, int batch,
                                               int num_query, int num_heads, int head_dim, int num_point,
                                               float* output, float* save_attn, float* save_loc, uint16_t* out16,
                                               void* stream) {
    PDVC_CHECK_ARG(out16 != nullptr && ((uintptr_t)out16 % 8) == 0, "out16 must be an 8-byte aligned bf16 buffer");
    return msda1d_forward_impl(value, value_pad_mask, proj, proj_stride, off_base, logit_base, ref, ref_dim, level_T,
                               num_levels, batch, num_query, num_heads, head_dim, num_point, output, save_attn,
                               save_loc, out16, stream);
}

// gv16 / gp16 (bf16 mode): the bf16 roundings of grad_value / grad_proj beside them -- only where the encoder's
// pyramid backward-query kernel and the 16-lane value-gradient walk run and grad_proj is all offset and logit
// columns (proj_stride = 2 * num_heads * 16); otherwise PDVC_ERR_UNSUPPORTED before launching anything
static int msda1d_backward_impl(const float* value, const uint8_t* value_pad_mask, const float* ref, int ref_dim,
                                const float* proj, int proj_stride, int off_base, int logit_base,
                                const int32_t* level_T, int num_levels, int batch, int num_query, int num_heads,
                                int head_dim, int num_point, const float* grad_output, const float* output,
                                const float* save_attn, const float* save_loc, float* grad_value, float* grad_proj,
                                float* grad_ref, float* grad_value_level_sums, uint16_t* gv16, uint16_t* gp16,
                                void* stream) {
    float* level_sums = grad_value_level_sums;
    if (level_sums)
        PDVC_CHECK_ARG(((long)num_heads * head_dim) % 4 == 0 && ((uintptr_t)level_sums % 16) == 0 &&
                           ((uintptr_t)grad_value % 16) == 0,
                       "level sums need num_heads * head_dim %% 4 == 0 and 16-byte aligned buffers");
    Levels1d lv;
    int S = 0;
    int rc = fill_levels(level_T, num_levels, num_point, lv, S);
    if (rc) return rc;
    Geometry g;
    if ((rc = pick_geometry(num_heads, head_dim, g))) return rc;
    PDVC_CHECK_ARG(ref_dim == 1 || ref_dim == 2, "ref_dim must be 1 or 2, got %d", ref_dim);
    PDVC_CHECK_ARG(save_attn && save_loc, "backward needs the forward's save_attn and save_loc");
    const int NSM = num_heads * kNS;
    PDVC_CHECK_ARG(off_base >= 0 && logit_base >= 0 && off_base + NSM <= proj_stride && logit_base + NSM <= proj_stride,
                   "proj columns out of range");
    hipStream_t s = (hipStream_t)stream;
    const long rows = (long)batch * num_query;
    const long tw = query_waves(g, batch, num_heads, num_query);
    if (grad_ref && rows > 0) {  // accumulated over the heads with atomics
        hipError_t e = zero_async(grad_ref, (size_t)rows * kL * ref_dim, s);
        if (e != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "memset grad_ref: %s", hipGetErrorString(e));
    }
    const int bq_blocks = (tw > 0 && bwdq_mode() == 1) ? pick_pyr(lv, S, num_query, head_dim, kBqQ) : 0;
    if (gv16 || gp16) {
        int Tm = 0;
        for (int l = 0; l < kL; ++l) Tm = lv.T[l] > Tm ? lv.T[l] : Tm;
        const bool g4ok = head_dim == 64 && value_g4() && (long)num_query * num_heads * head_dim * 4 < (1L << 31) &&
                          num_query < 65536 && Tm < 65535;
        // grad_proj's rounding needs the encoder's pyramid backward-query kernel; grad_value's alone (gp16 null: the
        // decoder's cross-attention, whose query side runs the dot kernel) only the 16-lane value walk
        if (!g4ok || (uintptr_t)gv16 % 8 || (gp16 && (bq_blocks <= 0 || proj_stride != 2 * NSM || (uintptr_t)gp16 % 2)))
            return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "bf16 gradients: grad_proj's only on the encoder's pyramid path");
    }
    if (bq_blocks > 0) {
        if ((rc = bwdq_pyr_attrs())) return rc;
        PDVC_CHECK_ARG((long)batch * num_heads * bq_blocks < (1L << 31), "too many query blocks");
        dim3 pg((unsigned)(batch * num_heads * bq_blocks));
        static const int qu = [] {  // queries per loop trip (PDVC_BQ_QU = 1 | 3 | 5: A/B); 3: encoder backward
            const char* e = getenv("PDVC_BQ_QU");  // 4 605 -> 4 500 us at 1024 videos (profiles/r04_bwdq_qu_ab.txt)
            const int v = e ? atoi(e) : 3;
            return (v == 1 || v == 5) ? v : 3;
        }();
#define BQ_LAUNCH(R, Q)                                                                                           \
    hipLaunchKernelGGL((msda1d_bwd_query_pyr_kernel<R, Q>), pg, dim3(kPyrThreads), kBqLds, s, value, value_pad_mask, \
                       proj, proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, bq_blocks,        \
                       grad_output, save_attn, save_loc, grad_proj, grad_ref, gp16)
        if (ref_dim == 1) {
            if (qu == 3) BQ_LAUNCH(1, 3);
            else if (qu == 5) BQ_LAUNCH(1, 5);
            else BQ_LAUNCH(1, 1);
        } else {
            if (qu == 3) BQ_LAUNCH(2, 3);
            else if (qu == 5) BQ_LAUNCH(2, 5);
            else BQ_LAUNCH(2, 1);
        }
#undef BQ_LAUNCH
        PDVC_CHECK_LAUNCH("msda1d_bwd_query_pyr_kernel");
    } else if (tw > 0 && head_dim == 64 && bwdq_mode() != 0 && (long)S * num_heads * head_dim * 4 < (1L << 31)) {
        dim3 grid((unsigned)((tw + 3) / 4));
        if (ref_dim == 1)
            hipLaunchKernelGGL((msda1d_bwd_query_dot_kernel<1>), grid, dim3(256), 0, s, value, value_pad_mask, proj,
                               proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, (int)tw,
                               grad_output, save_attn, save_loc, grad_proj, grad_ref);
        else
            hipLaunchKernelGGL((msda1d_bwd_query_dot_kernel<2>), grid, dim3(256), 0, s, value, value_pad_mask, proj,
                               proj_stride, off_base, logit_base, ref, lv, num_query, S, num_heads, (int)tw,
                               grad_output, save_attn, save_loc, grad_proj, grad_ref);
        PDVC_CHECK_LAUNCH("msda1d_bwd_query_dot_kernel");
    } else if (tw > 0) {
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
    // grad_value: one workgroup per (video, head, level) and query chunk; the chunk keeps the LDS index
    // (2 (T+2) ints + 12 B per sample) within 96 KiB; later chunks add into the rows the first wrote
    PDVC_CHECK_ARG(head_dim <= 128, "value gradient supports head_dim <= 128, got %d", head_dim);
    const long nblk = (long)batch * num_heads * kL;
    if (nblk > 0) {
        if (num_query == 0) {
            hipError_t e = zero_async(grad_value, (size_t)batch * S * num_heads * head_dim, s);
            if (e == hipSuccess && level_sums)
                e = zero_async(level_sums, (size_t)batch * kL * num_heads * head_dim, s);
            if (e != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "memset grad_value: %s", hipGetErrorString(e));
            return PDVC_OK;
        }
        int Tmax = 0;
        for (int l = 0; l < kL; ++l) Tmax = lv.T[l] > Tmax ? lv.T[l] : Tmax;
        // G4 packs (key, query) into 16 bits each
        const bool g4 = head_dim == 64 && value_g4() && (long)num_query * num_heads * head_dim * 4 < (1L << 31) &&
                        num_query < 65536 && Tmax < 65535;
        const long per_sample = 12;  // LDS bytes per sorted sample (both forms)
        const long budget = 96 * 1024 - 8L * (Tmax + 2) - 16;
        if (budget < per_sample * kP) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "level length %d too long", Tmax);
        int qchunk = (int)(budget / (per_sample * kP));
        if (qchunk > kVQPT * kVW * 64) qchunk = kVQPT * kVW * 64;
        if (qchunk > num_query) qchunk = num_query;
        static std::atomic<int> done[kMaxDevices];  // dynamic LDS <= 96 KiB by construction of qchunk (+32 B static)
        if ((rc = lds_optin(done, {{(const void*)msda1d_bwd_value_kernel<1, false>, 96 * 1024},
                                   {(const void*)msda1d_bwd_value_kernel<2, false>, 96 * 1024},
                                   {(const void*)msda1d_bwd_value_kernel<1, true>, 96 * 1024},
                                   {(const void*)msda1d_bwd_value_kernel<1, true, 4>, 96 * 1024},
                                   {(const void*)msda1d_bwd_value_kernel<1, true, 4, true>, 96 * 1024}},
                            "msda1d_bwd_value_kernel")))
            return rc;
        for (int q0 = 0; q0 < num_query; q0 += qchunk) {
            const int nq = (num_query - q0) < qchunk ? (num_query - q0) : qchunk;
            size_t lds = sizeof(int) * (2 * (size_t)(Tmax + 2) + 3 * (size_t)nq * kP + 2);
            if (g4 && level_sums && lds < kVW * 16 * 16) lds = kVW * 16 * 16;  // the level-sum reduction
            float* gsums = g4 ? level_sums : nullptr;
            const int acc = q0 > 0;
#define VAL_LAUNCH(UGV, B16V)                                                                                       \
    hipLaunchKernelGGL((msda1d_bwd_value_kernel<1, true, UGV, B16V>), dim3((unsigned)nblk), dim3(kVW * 64), lds, s, \
                       value_pad_mask, lv, num_query, q0, nq, S, num_heads, head_dim, acc, grad_output, save_attn,  \
                       save_loc, grad_value, gsums, (const int64_t*)nullptr, (const int64_t*)nullptr, gv16)
            static const int vabl = [] {
                const char* e = getenv("PDVC_VAL_ABLATE");
                return e ? atoi(e) : 0;
            }();
            if (g4 && !gv16 && (vabl == 3 || vabl == 4) && value_ug(num_query, S) == 4) {  // measurement only
                const void* k = vabl == 3 ? (const void*)msda1d_bwd_value_kernel<1, true, 4, false, 1>
                                          : (const void*)msda1d_bwd_value_kernel<1, true, 4, false, 2>;
                (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
                if (vabl == 3)
                    hipLaunchKernelGGL((msda1d_bwd_value_kernel<1, true, 4, false, 1>), dim3((unsigned)nblk),
                                       dim3(kVW * 64), lds, s, value_pad_mask, lv, num_query, q0, nq, S, num_heads,
                                       head_dim, acc, grad_output, save_attn, save_loc, grad_value, gsums,
                                       (const int64_t*)nullptr, (const int64_t*)nullptr, gv16);
                else
                    hipLaunchKernelGGL((msda1d_bwd_value_kernel<1, true, 4, false, 2>), dim3((unsigned)nblk),
                                       dim3(kVW * 64), lds, s, value_pad_mask, lv, num_query, q0, nq, S, num_heads,
                                       head_dim, acc, grad_output, save_attn, save_loc, grad_value, gsums,
                                       (const int64_t*)nullptr, (const int64_t*)nullptr, gv16);
            } else if (g4 && !gv16 && (vabl == 1 || vabl == 2) && value_ug(num_query, S) == 8) {  // measurement only
                const void* k = vabl == 1 ? (const void*)msda1d_bwd_value_kernel<1, true, 8, false, 1>
                                          : (const void*)msda1d_bwd_value_kernel<1, true, 8, false, 2>;
                (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
                if (vabl == 1)
                    hipLaunchKernelGGL((msda1d_bwd_value_kernel<1, true, 8, false, 1>), dim3((unsigned)nblk),
                                       dim3(kVW * 64), lds, s, value_pad_mask, lv, num_query, q0, nq, S, num_heads,
                                       head_dim, acc, grad_output, save_attn, save_loc, grad_value, gsums,
                                       (const int64_t*)nullptr, (const int64_t*)nullptr, gv16);
                else
                    hipLaunchKernelGGL((msda1d_bwd_value_kernel<1, true, 8, false, 2>), dim3((unsigned)nblk),
                                       dim3(kVW * 64), lds, s, value_pad_mask, lv, num_query, q0, nq, S, num_heads,
                                       head_dim, acc, grad_output, save_attn, save_loc, grad_value, gsums,
                                       (const int64_t*)nullptr, (const int64_t*)nullptr, gv16);
            } else if (g4 && gv16) VAL_LAUNCH(4, true);  // the bf16 stores spill the depth-8 walk (7 VGPRs): depth 4
            else if (g4 && value_ug(num_query, S) == 4) VAL_LAUNCH(4, false);
            else if (g4) VAL_LAUNCH(8, false);
#undef VAL_LAUNCH
            else if (head_dim <= 64)
                hipLaunchKernelGGL((msda1d_bwd_value_kernel<1, false>), dim3((unsigned)nblk), dim3(kVW * 64), lds, s,
                                   value_pad_mask, lv, num_query, q0, nq, S, num_heads, head_dim, acc, grad_output,
                                   save_attn, save_loc, grad_value, gsums);
            else
                hipLaunchKernelGGL((msda1d_bwd_value_kernel<2, false>), dim3((unsigned)nblk), dim3(kVW * 64), lds, s,
                                   value_pad_mask, lv, num_query, q0, nq, S, num_heads, head_dim, acc, grad_output,
                                   save_attn, save_loc, grad_value, gsums);
            PDVC_CHECK_LAUNCH("msda1d_bwd_value_kernel");
        }
        if (level_sums && !g4) {  // the other value-gradient forms: one read of grad_value
            int32_t lt[kL];
            for (int l = 0; l < kL; ++l) lt[l] = lv.T[l];
            rc = pdvc_level_pos_rows_backward_f32(grad_value, lt, kL, batch, S, num_heads * head_dim, level_sums, s);
            if (rc) return rc;
        }
    }
    return PDVC_OK;
}

extern "C" int pdvc_msda1d_backward_ex_f32(const float* value, const uint8_t* value_pad_mask, const float* ref,
                                           int ref_dim, const float* proj, int proj_stride, int off_base,
                                           int logit_base, const int32_t* level_T, int num_levels, int batch,
                                           int num_query, int num_heads, int head_dim, int num_point,
                                           const float* grad_output, const float* output, const float* save_attn,
                                           const float* save_loc, float* grad_value, float* grad_proj,
                                           float* grad_ref, float* grad_value_level_sums, void* stream) {
    return msda1d_backward_impl(value, value_pad_mask, ref, ref_dim, proj, proj_stride, off_base, logit_base, level_T,
                                num_levels, batch, num_query, num_heads, head_dim, num_point, grad_output, output,
                                save_attn, save_loc, grad_value, grad_proj, grad_ref, grad_value_level_sums, nullptr,
                                nullptr, stream);
}

extern "C" int pdvc_msda1d_backward_ex_f32_bf16out(const float* value, const uint8_t* value_pad_mask,
                                                   const float* ref, int ref_dim, const float* proj, int proj_stride,
                                                   int off_base, int logit_base, const int32_t* level_T,
                                                   int num_levels, int batch, int num_query, int num_heads,
                                                   int head_dim, int num_point, const float* grad_output,
                                                   const float* output, const float* save_attn, const float* save_loc,
                                                   float* grad_value, float* grad_proj, float* grad_ref,
                                                   float* grad_value_level_sums, uint16_t* grad_value16,
                                                   uint16_t* grad_proj16, void* stream) {
    PDVC_CHECK_ARG(grad_value16 != nullptr, "grad_value16 is required (grad_proj16 may be null)");
    return msda1d_backward_impl(value, value_pad_mask, ref, ref_dim, proj, proj_stride, off_base, logit_base, level_T,
                                num_levels, batch, num_query, num_heads, head_dim, num_point, grad_output, output,
                                save_attn, save_loc, grad_value, grad_proj, grad_ref, grad_value_level_sums,
                                grad_value16, grad_proj16, stream);
}

extern "C" int pdvc_msda1d_backward_f32(const float* value, const uint8_t* value_pad_mask, const float* ref,
                                        int ref_dim, const float* proj, int proj_stride, int off_base, int logit_base,
                                        const int32_t* level_T, int num_levels, int batch, int num_query,
                                        int num_heads, int head_dim, int num_point, const float* grad_output,
                                        const float* output, const float* save_attn, const float* save_loc,
                                        float* grad_value, float* grad_proj, float* grad_ref, void* stream) {
    return pdvc_msda1d_backward_ex_f32(value, value_pad_mask, ref, ref_dim, proj, proj_stride, off_base, logit_base,
                                       level_T, num_levels, batch, num_query, num_heads, head_dim, num_point,
                                       grad_output, output, save_attn, save_loc, grad_value, grad_proj, grad_ref,
                                       nullptr, stream);
}

// ---- the drop-in operator's 1-D fast path (msda_op.hip dispatches here; the level table is checked on the device) ----
namespace pdvc {

// host-side conditions: D = 64, 4 levels x 4 points, offsets within the kernels' 32-bit arithmetic; PDVC_DROPIN_1D=0
// turns the path off (A/B)
bool dropin1d_applies(int S, int M, int D, int L, int Lq, int P) {
    static const bool on = [] {
        const char* e = getenv("PDVC_DROPIN_1D");
        return !(e && e[0] == '0');
    }();
    return on && D == 64 && L == kL && P == kP && Lq > 0 && Lq < 65536 && S < 65535 &&
           (long)S * M * D * 4 < (1L << 31) && (long)Lq * M * D * 4 < (1L << 31);
}

// whole-pyramid drop-in kernels for encoder-shaped calls (4 Lq >= S, pick_pyr's rule); PDVC_DROPIN_PYR=0 keeps every
// call on the L2-gather kernels (A/B).  Returns the query blocks per (video, head), 0 when the pyramid form is off.
static int dropin_pyr_blocks(int S, int Lq, int per_block) {
    static const bool on = [] {
        const char* e = getenv("PDVC_DROPIN_PYR");
        return !(e && e[0] == '0');
    }();
    if (!on || 4L * Lq < S) return 0;
    static std::atomic<int> done[kMaxDevices];
    const bool attr = lds_optin(done, {{(const void*)msda_dropin_fwd_pyr_kernel, (int)kPyr2LdsMax},
                                       {(const void*)msda_dropin_bwd_query_pyr_kernel, (int)kPyrLds}},
                                "msda_dropin pyramid kernels") == PDVC_OK;
    return attr ? (Lq + per_block - 1) / per_block : 0;
}

// the gather-form launch after a pyramid launch is needed only when a staging phase might not fit: with S <= 512
// every level table summing to S fits (dropin_pyr_fits), and the fallback is skipped
static bool dropin_may_not_fit(int S) { return S > kPyrRows; }

// grid of the gather kernels: one workgroup per 4 waves, or -- behind a pyramid launch, where it usually retires at
// once -- one chip's worth (8 workgroups of 4 waves on each of the 256 CUs), grid-strided over the waves
static unsigned dropin_gather_grid(long tw, int pyr_first) {
    const long full = (tw + 3) / 4;
    return (unsigned)(pyr_first && full > 2048 ? 2048 : full);
}

int dropin1d_forward(const float* value, const int64_t* shapes, const int64_t* lsi, const float* loc,
                     const float* attn, int N, int S, int M, int Lq, float* out, hipStream_t s) {
    const long tw = (long)N * M * ((Lq + 3) / 4);
    if (tw == 0) return PDVC_OK;
    PDVC_CHECK_ARG(tw < (1L << 31) / 4, "too many rows");
    int pyr_first = 0;
    if (const int qb = dropin_pyr_blocks(S, Lq, kPyrQ)) {
        PDVC_CHECK_ARG((long)N * M * qb < (1L << 31), "too many query blocks");
        hipLaunchKernelGGL(msda_dropin_fwd_pyr_kernel, dim3((unsigned)(N * M * qb)), dim3(kPyrThreads), kPyr2LdsMax, s,
                           value, shapes, lsi, loc, attn, Lq, S, M, qb, out);
        PDVC_CHECK_LAUNCH("msda_dropin_fwd_pyr_kernel");
        pyr_first = 1;
        if (!dropin_may_not_fit(S)) return PDVC_OK;
    }
    hipLaunchKernelGGL(msda_dropin_fwd_kernel, dim3(dropin_gather_grid(tw, pyr_first)), dim3(256), 0, s, value, shapes,
                       lsi, loc, attn, Lq, S, M, (int)tw, pyr_first, out);
    PDVC_CHECK_LAUNCH("msda_dropin_fwd_kernel");
    return PDVC_OK;
}

// workspace: 2 * N * Lq * M * 16 floats (the level-major location / weight slab of the value gradient)
int dropin1d_backward(const float* value, const int64_t* shapes, const int64_t* lsi, const float* loc,
                      const float* attn, const float* gout, int N, int S, int M, int Lq, float* grad_value,
                      float* grad_loc, float* grad_attn, float* workspace, hipStream_t s) {
    const long tw = (long)N * M * ((Lq + 3) / 4);
    if (tw == 0) return PDVC_OK;
    PDVC_CHECK_ARG(tw < (1L << 31) / 4, "too many rows");
    float* save_attn = workspace;
    float* save_loc = workspace + (size_t)N * Lq * M * kNS;
    int pyr_first = 0;
    if (const int qb = dropin_pyr_blocks(S, Lq, kBqQ)) {
        PDVC_CHECK_ARG((long)N * M * qb < (1L << 31), "too many query blocks");
        hipLaunchKernelGGL(msda_dropin_bwd_query_pyr_kernel, dim3((unsigned)(N * M * qb)), dim3(kPyrThreads), kPyrLds,
                           s, value, shapes, lsi, loc, attn, Lq, S, M, qb, gout, grad_loc, grad_attn, save_attn,
                           save_loc);
        PDVC_CHECK_LAUNCH("msda_dropin_bwd_query_pyr_kernel");
        pyr_first = 1;
    }
    if (!pyr_first || dropin_may_not_fit(S)) {
        hipLaunchKernelGGL(msda_dropin_bwd_query_kernel, dim3(dropin_gather_grid(tw, pyr_first)), dim3(256), 0, s, value,
                           shapes, lsi, loc, attn, Lq, S, M, (int)tw, pyr_first, gout, grad_loc, grad_attn, save_attn,
                           save_loc);
        PDVC_CHECK_LAUNCH("msda_dropin_bwd_query_kernel");
    }
    // value gradient: msda1d_bwd_value_kernel on the slab, its LDS sized for the longest possible level (S)
    static std::atomic<int> done[kMaxDevices];
    if (const int rc = lds_optin(done, {{(const void*)msda1d_bwd_value_kernel<1, true>, 96 * 1024},
                                        {(const void*)msda1d_bwd_value_kernel<1, true, 4>, 96 * 1024}},
                                 "msda1d_bwd_value_kernel"))
        return rc;
    const long per_sample = 12;
    const long budget = 96 * 1024 - 8L * (S + 2) - 16;
    if (budget < per_sample * kP) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "spatial size %d too long", S);
    int qchunk = (int)(budget / (per_sample * kP));
    if (qchunk > kVQPT * kVW * 64) qchunk = kVQPT * kVW * 64;
    if (qchunk > Lq) qchunk = Lq;
    const long nblk = (long)N * M * kL;
    Levels1d lv{};  // read on the device
    for (int q0 = 0; q0 < Lq; q0 += qchunk) {
        const int nq = (Lq - q0) < qchunk ? (Lq - q0) : qchunk;
        const size_t lds = sizeof(int) * (2 * (size_t)(S + 2) + 3 * (size_t)nq * kP + 2);
        const int acc = q0 > 0;
        if (value_ug(Lq, S) == 4)
            hipLaunchKernelGGL((msda1d_bwd_value_kernel<1, true, 4>), dim3((unsigned)nblk), dim3(kVW * 64), lds, s,
                               nullptr, lv, Lq, q0, nq, S, M, 64, acc, gout, save_attn, save_loc, grad_value, nullptr,
                               shapes, lsi);
        else
            hipLaunchKernelGGL((msda1d_bwd_value_kernel<1, true>), dim3((unsigned)nblk), dim3(kVW * 64), lds, s,
                               nullptr, lv, Lq, q0, nq, S, M, 64, acc, gout, save_attn, save_loc, grad_value, nullptr,
                               shapes, lsi);
        PDVC_CHECK_LAUNCH("msda1d_bwd_value_kernel (drop-in)");
    }
    return PDVC_OK;
}

}  // namespace pdvc
