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

// One wave per (row, head group, level, pair of points): waves_per_row = head groups x kSplit, so the
// R ~ 256 caption rows of a step still put >= 2048 waves on the chip (one wave per row left 255 of 256
// CUs with a single wave).  A head's D channels are spread over LPH lanes, CPL = 8 consecutive floats each.
constexpr int kSPW = 2;              // samples per wave
constexpr int kSplit = cNS / kSPW;   // waves per (row, head group)

template <int CPL, int LPH, int RD>
__global__ __launch_bounds__(256) void cap_gather_fwd_kernel(const float* __restrict__ value,
                                                              const uint8_t* __restrict__ vmask,
                                                              const int32_t* __restrict__ row_video,
                                                              const float* __restrict__ offsets, int off_stride,
                                                              int off_col0, const float* __restrict__ off_add,
                                                              const float* __restrict__ ref, int rd1_rows,
                                                              CapLevels lv, int S, int M, int D, int waves_per_row,
                                                              int total_waves, float* __restrict__ samples,
                                                              float* __restrict__ save_loc, int remap) {
    constexpr int HPW = 64 / LPH;
    const int lane = threadIdx.x & 63;
    const int wave = (remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (wave >= total_waves) return;
    const int r = wave / waves_per_row;
    const int wr = wave - r * waves_per_row;
    const int hg = wr / kSplit;
    const int j0 = (wr - hg * kSplit) * kSPW;
    const int l = j0 / cP;
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
    const int T = lv.T[0] * (l == 0) + lv.T[1] * (l == 1) + lv.T[2] * (l == 2) + lv.T[3] * (l == 3);
    const int st = lv.start[0] * (l == 0) + lv.start[1] * (l == 1) + lv.start[2] * (l == 2) + lv.start[3] * (l == 3);
    const float r0 = ref[((size_t)r * cL + l) * RD];
    const float r1 = (RD == 2) ? ref[((size_t)r * cL + l) * RD + 1] : 0.f;
    int x0[kSPW];
    float nw[kSPW], ne[kSPW];
#pragma unroll
    for (int u = 0; u < kSPW; ++u) {
        const int j = j0 + u;
        const float off = off_add ? orow[j] + off_add[((size_t)r * M + m) * cNS + j] : orow[j];
        const float loc = centre_only ? r0 + off / (float)T : r0 + ((off / (float)cP) * r1) * 0.5f;
        if (save_loc && sub == 0) save_loc[((size_t)r * M + m) * cNS + j] = loc;
        float gm;
        const float ix = border_ix(loc, T, gm);
        const float xf = floorf(ix);
        x0[u] = (int)xf;
        // iy == 0 (H == 1): nw = (x0+1-ix)*1, ne = (ix-x0)*1, the y0+1 row is outside
        nw[u] = ((float)(x0[u] + 1) - ix);
        ne[u] = (ix - xf);
    }
    VecF<CPL> v0[kSPW], v1[kSPW];
    bool ok0[kSPW], ok1[kSPW];
#pragma unroll
    for (int u = 0; u < kSPW; ++u) {  // all corner rows in flight together (clamped, selected after)
        const int a1 = min(x0[u] + 1, T - 1);
        v0[u].load(vbase + (size_t)(st + x0[u]) * MD);
        v1[u].load(vbase + (size_t)(st + a1) * MD);
        ok0[u] = !(mbase && mbase[st + x0[u]]);
        ok1[u] = x0[u] + 1 < T && !(mbase && mbase[st + a1]);
    }
#pragma unroll
    for (int u = 0; u < kSPW; ++u) {
        VecF<CPL> o;
#pragma unroll
        for (int c = 0; c < CPL; ++c)
            o.v[c] = (ok0[u] ? v0[u].v[c] : 0.f) * nw[u] + (ok1[u] ? v1[u].v[c] : 0.f) * ne[u];
        o.store(samples + (((size_t)r * M + m) * cNS + j0 + u) * D + c0);
    }
}

template <int CPL, int LPH, int RD>
__global__ __launch_bounds__(256) void cap_gather_bwd_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const int32_t* __restrict__ row_video,
    const float* __restrict__ offsets, int off_stride, int off_col0, const float* __restrict__ off_add,
    const float* __restrict__ ref, int rd1_rows, CapLevels lv, int S, int M, int D, int waves_per_row,
    int total_waves, const float* __restrict__ save_loc,
    const float* __restrict__ gsamp, float* __restrict__ grad_value, float* __restrict__ grad_off,
    float* __restrict__ grad_ref, const float* __restrict__ value2, const float* __restrict__ gsamp2, int remap) {
    constexpr int HPW = 64 / LPH;
    const int lane = threadIdx.x & 63;
    const int wave = (remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (wave >= total_waves) return;
    const int r = wave / waves_per_row;
    const int wr = wave - r * waves_per_row;
    const int hg = wr / kSplit;
    const int j0 = (wr - hg * kSplit) * kSPW;
    const int l = j0 / cP;
    const int sub = lane % LPH;
    const int m_raw = hg * HPW + lane / LPH;
    const bool active = m_raw < M;
    const int m = active ? m_raw : 0;
    // lane-strided channels (sub + LPH*c): every atomic wave-instruction adds one contiguous LPH*4-byte
    // segment per head (256 B at D = 512), the shape global float atomics run at full rate with
    const int c0 = sub;
    const int b = row_video[r];
    const size_t MD = (size_t)M * D;
    const float* vbase = value + (size_t)b * S * MD + (size_t)m * D + c0;
    float* gvbase = grad_value + (size_t)b * S * MD + (size_t)m * D + c0;
    const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
    const int T = lv.T[0] * (l == 0) + lv.T[1] * (l == 1) + lv.T[2] * (l == 2) + lv.T[3] * (l == 3);
    const int st = lv.start[0] * (l == 0) + lv.start[1] * (l == 1) + lv.start[2] * (l == 2) + lv.start[3] * (l == 3);

    float loc[kSPW], gm[kSPW], nw[kSPW], ne[kSPW];
    int x0[kSPW];
#pragma unroll
    for (int u = 0; u < kSPW; ++u) {
        loc[u] = active ? save_loc[((size_t)r * M + m) * cNS + j0 + u] : 0.f;
        const float ix = border_ix(loc[u], T, gm[u]);
        const float xf = floorf(ix);
        x0[u] = (int)xf;
        nw[u] = ((float)(x0[u] + 1) - ix);
        ne[u] = (ix - xf);
    }
    float g[kSPW][CPL], v0[kSPW][CPL], v1[kSPW][CPL];
    bool ok0[kSPW], ok1[kSPW];
#pragma unroll
    for (int u = 0; u < kSPW; ++u) {
        const int a1 = min(x0[u] + 1, T - 1);
        const float* gp = gsamp + (((size_t)r * M + m) * cNS + j0 + u) * D + c0;
        const float* p0 = vbase + (size_t)(st + x0[u]) * MD;
        const float* p1 = vbase + (size_t)(st + a1) * MD;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            g[u][c] = gp[LPH * c];
            v0[u][c] = p0[LPH * c];
            v1[u][c] = p1[LPH * c];
        }
        ok0[u] = active && !(mbase && mbase[st + x0[u]]);
        ok1[u] = active && x0[u] + 1 < T && !(mbase && mbase[st + a1]);
    }
    float part[kSPW];
#pragma unroll
    for (int u = 0; u < kSPW; ++u) {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const float gv = active ? g[u][c] : 0.f;
            if (grad_value) {  // NULL: the value gradient comes from cap_value_grad_kernel after all steps
                if (ok0[u]) atomicAdd(gvbase + (size_t)(st + x0[u]) * MD + LPH * c, nw[u] * gv);
                if (ok1[u]) atomicAdd(gvbase + (size_t)(st + x0[u] + 1) * MD + LPH * c, ne[u] * gv);
            }
            s += gv * ((ok1[u] ? v1[u][c] : 0.f) - (ok0[u] ? v0[u][c] : 0.f));  // gix = -vnw + vne
        }
        part[u] = s;
    }
    if (value2) {  // a second sampled tensor at the same locations (no padding mask): its location gradient adds in
        const float* v2base = value2 + (size_t)b * S * MD + (size_t)m * D + c0;
#pragma unroll
        for (int u = 0; u < kSPW; ++u) {
            const int a1 = min(x0[u] + 1, T - 1);
            const float* gp = gsamp2 + (((size_t)r * M + m) * cNS + j0 + u) * D + c0;
            const float* p0 = v2base + (size_t)(st + x0[u]) * MD;
            const float* p1 = v2base + (size_t)(st + a1) * MD;
            const bool hi = x0[u] + 1 < T;
            float s2 = 0.f;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const float gv = active ? gp[LPH * c] : 0.f;
                s2 += gv * ((hi ? p1[LPH * c] : 0.f) - p0[LPH * c]);
            }
            part[u] += s2;
        }
    }
    // sum over the LPH lanes of the head (all lanes end with the head's totals)
#pragma unroll
    for (int u = 0; u < kSPW; ++u) {
#pragma unroll
        for (int d = 1; d < LPH; d <<= 1) part[u] += lane_swap(part[u], d);
    }
    const bool owner = active && sub == 0;
    const bool centre_only = (RD == 1) || (r < rd1_rows);
    float gr0 = 0.f, gr1 = 0.f;
    const float r1 = (RD == 2 && !centre_only) ? ref[((size_t)r * cL + l) * 2 + 1] : 0.f;
#pragma unroll
    for (int u = 0; u < kSPW; ++u) {
        const int j = j0 + u;
        const float gloc = 2.f * (gm[u] * part[u]);  // grid = 2*loc - 1
        float goff;
        if (centre_only) {
            goff = gloc / (float)T;
            gr0 += gloc;
        } else {
            const float t2 = gloc * 0.5f;
            goff = (t2 * r1) / (float)cP;
            float o = active ? offsets[(size_t)r * off_stride + off_col0 + m * cNS + j] : 0.f;
            if (active && off_add) o += off_add[((size_t)r * M + m) * cNS + j];
            gr0 += gloc;
            gr1 += t2 * (o / (float)cP);
        }
        if (owner) grad_off[(size_t)r * off_stride + off_col0 + m * cNS + j] = goff;
    }
    if (grad_ref) {
        // heads of this wave: sum the owners' values over the wave, one atomic per (wave, level)
        float v0 = owner ? gr0 : 0.f, v1 = owner ? gr1 : 0.f;
#pragma unroll
        for (int d = LPH; d < 64; d <<= 1) {
            v0 += lane_swap(v0, d);
            if (RD == 2) v1 += lane_swap(v1, d);
        }
        if (lane == 0) {
            atomicAdd(grad_ref + ((size_t)r * cL + l) * RD, v0);
            if (RD == 2) atomicAdd(grad_ref + ((size_t)r * cL + l) * RD + 1, v1);
        }
    }
}

// -------------------------------------------------------------------------------------------------
// Value gradient of the caption sampling, all decoder steps at once, destination-sorted (no float atomics).
// The per-step backward (cap_gather_bwd_kernel with grad_value == NULL) leaves the value gradient out; after
// the recurrence this kernel sums, for every value row, the contributions of the samples of every step whose
// border-clipped corners touch it: row t of level l gets  sum_{x0(s) = t} nw_s g_s + sum_{x0(s) = t-1} ne_s g_s
// over the samples s = (step, row of the video, point of level l), g_s the sample's gradient row (D floats).
// One 512-thread workgroup per (video, head, level): an LDS counting sort of its samples by key x0 + 1, then
// each wave walks a contiguous row range (balanced by sample count) with two running accumulators -- the
// mapping of msda1d_bwd_value_kernel (msda1d.hip) with per-sample gradient rows.  Every row is written once
// (zeros where no sample lands), so grad_value needs no memset; with `accumulate` a later chunk of steps adds.
// The per-step kernel's atomics were 2 x 134 MB per step at 512 videos, capped by the ~1.3 TB/s atomic rate.
// -------------------------------------------------------------------------------------------------
constexpr int kCVW = 8;  // waves per workgroup

template <int CW>  // channels per lane: D <= 64 * CW, channel = lane + 64 c
__global__ __launch_bounds__(kCVW * 64) void cap_value_grad_kernel(
    const uint8_t* __restrict__ vmask, CapLevels lv, int S, int M, int D, int R, int s0, int ns, int accumulate,
    const int32_t* __restrict__ vr_start, const int32_t* __restrict__ vr_rows, const float* __restrict__ save_loc,
    const float* __restrict__ gsamp, float* __restrict__ grad_value, float* __restrict__ level_sums,
    const int32_t* __restrict__ step_rows, const float* __restrict__ grow, const float* __restrict__ gscale,
    uint16_t* __restrict__ gv16) {
    extern __shared__ __attribute__((aligned(16))) int lds_c[];
    __shared__ int wsum[kCVW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int l = lb % cL;
    const int bm = lb / cL;
    const int b = bm / M, m = bm - b * M;
    const int T = lv.T[0] * (l == 0) + lv.T[1] * (l == 1) + lv.T[2] * (l == 2) + lv.T[3] * (l == 3);
    const int st = lv.start[0] * (l == 0) + lv.start[1] * (l == 1) + lv.start[2] * (l == 2) + lv.start[3] * (l == 3);
    const int rb0 = vr_start[b], nr = vr_start[b + 1] - rb0;
    const int per_step = nr * cP;
    const int n = ns * per_step;
    int* off = lds_c;                // [T + 2]
    int* cur = lds_c + (T + 2);      // [T + 2]
    int* sq = lds_c + 2 * (T + 2);   // [n] gradient row of each sorted sample
    float* clo = (float*)(sq + n);   // [n] nw (0 where the corner is masked) -> row x0
    float* chi = clo + n;            // [n] ne (0 where x0 + 1 is outside or masked) -> row x0 + 1
    const uint8_t* mrow = vmask ? vmask + (size_t)b * S + st : nullptr;
    for (int i = threadIdx.x; i < T + 2; i += blockDim.x) off[i] = 0;
    __syncthreads();
    // step_rows (steps x [start, count]): the rows each step of the recurrence computed (a video's rows stop at its
    // last step, caption_decode.py); samples of the other (step, row) pairs were never formed and are skipped
    auto sample = [&](int i, int& gidx) -> float {  // clipped pixel coordinate of sample i (-1: skipped); gidx its row
        const int step = s0 + i / per_step, rem = i - (i / per_step) * per_step;
        const int r = vr_rows[rb0 + rem / cP], j = l * cP + rem % cP;
        if (step_rows && (r < step_rows[2 * step] || r >= step_rows[2 * step] + step_rows[2 * step + 1])) return -1.f;
        const size_t si = (((size_t)step * R + r) * M + m) * cNS + j;
        gidx = (int)si;
        float gm;
        return border_ix(save_loc[si], T, gm);
    };
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int gidx;
        const float ix = sample(i, gidx);
        if (ix >= 0.f) atomicAdd(&off[(int)floorf(ix) + 1], 1);
    }
    __syncthreads();
    {  // exclusive scan of off[0 .. T+1]
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
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int gidx;
        const float ix = sample(i, gidx);
        if (ix < 0.f) continue;
        const float xf = floorf(ix);
        const int x0 = (int)xf;
        const bool ok0 = !(mrow && mrow[x0]);
        const bool ok1 = x0 + 1 < T && !(mrow && mrow[x0 + 1]);
        const int pos = atomicAdd(&cur[x0 + 1], 1);
        sq[pos] = gidx;
        clo[pos] = ok0 ? ((float)(x0 + 1) - ix) : 0.f;
        chi[pos] = ok1 ? (ix - xf) : 0.f;
    }
    __syncthreads();
    const int total = off[T + 1];
    auto split = [&](int w) -> int {
        if (w <= 0) return 0;
        if (w >= kCVW) return T;
        const int target = (int)(((long)total * w) / kCVW);
        int lo = 0, hi = T;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (off[mid] >= target) hi = mid;
            else lo = mid + 1;
        }
        return lo;
    };
    const int r0 = split(wid), r1 = split(wid + 1);
    const size_t MD = (size_t)M * D;
    float psum[CW];  // this chunk's contributions to the wave's rows (the level sums)
#pragma unroll
    for (int c = 0; c < CW; ++c) psum[c] = 0.f;
    if (r0 < r1) {
    float* ob = grad_value + ((size_t)b * S + st) * MD + (size_t)m * D;
    // bf16 mode: every row's rounding too, at the same offsets (the last chunk of steps writes the final rows)
    uint16_t* ob16 = gv16 ? gv16 + ((size_t)b * S + st) * MD + (size_t)m * D : nullptr;
    float accp[CW], acch[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c) accp[c] = acch[c] = 0.f;
    int k = r0;
    auto close_bucket = [&]() {  // bucket k complete: row k-1 has both its corners
        const int r = k - 1;
        if (r >= r0) {
            float* orow = ob + (size_t)r * MD;
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                const int ch = lane + 64 * c;
                if (ch < D) {
                    float v = accp[c];
                    psum[c] += v;
                    if (accumulate) v += orow[ch];
                    orow[ch] = v;
                    if (ob16) ob16[(size_t)r * MD + ch] = (uint16_t)bf16_bits(v);
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
    constexpr int U = 4;
    for (int j0 = jb; j0 < je; j0 += U) {
        float gv[U][CW];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = (j0 + u < je) ? j0 + u : je - 1;
            const int si = sq[j];
            if (grow) {  // rank-1 sample gradients: gscale[s] * grow[(step, row, head)] (the fused caption backward's
                         // p_k * dres, formed here with the same product instead of stored 16 times per row)
                const float sc = gscale[si];
                const float* gp = grow + (size_t)(si / cNS) * D;
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    const int ch = lane + 64 * c;
                    gv[u][c] = sc * gp[ch < D ? ch : 0];
                }
            } else {
                const float* gp = gsamp + (size_t)si * D;
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    const int ch = lane + 64 * c;
                    gv[u][c] = gp[ch < D ? ch : 0];
                }
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
    if (level_sums) {  // the bias gradient's partial: column sums of the rows this workgroup wrote
        __syncthreads();  // every wave is done with the sorted samples: reuse their LDS
        float* red = reinterpret_cast<float*>(lds_c);
#pragma unroll
        for (int c = 0; c < CW; ++c) red[(wid * CW + c) * 64 + lane] = psum[c];
        __syncthreads();
        for (int i = threadIdx.x; i < 64 * CW; i += blockDim.x) {
            const int c = i >> 6, ln = i & 63, ch = ln + 64 * c;
            if (ch < D) {
                float t = red[c * 64 + ln];
                for (int w = 1; w < kCVW; ++w) t += red[(w * CW + c) * 64 + ln];
                float* o = level_sums + ((size_t)b * cL + l) * MD + (size_t)m * D + ch;
                if (accumulate) t += *o;
                *o = t;
            }
        }
    }
}

// XCD-aware wave order (PDVC_CAP_XCD=0: the dispatch order, A/B): a video's caption rows are consecutive in every
// layout (pdvc/batch_layout.py), so with xcd_remap its waves run on one XCD, together, and the corner rows its events
// and points share (the coarse levels above all) come from that XCD's L2
static int cap_remap() {
    static const int on = [] {
        const char* e = getenv("PDVC_CAP_XCD");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    return on;
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
    wpr = ((num_heads + hpw - 1) / hpw) * kSplit;
    return PDVC_OK;
}


// -------------------------------------------------------------------------------------------------
// One caption step's sampling and soft attention in one launch, for the 512-wide head every cfg uses (cap_nheads 1;
// D = A = 512; pdvc/ops/functions/caption_decode.py): one 128-thread workgroup per (row, head), a float4 of channels
// per thread -- the mapping of softattn_fwd4_kernel (capstep.hip).  Threads 0..15 form sample j's location and
// corners (cap_gather_fwd_kernel's math) into LDS; every thread then reads its 16 bytes of the two corner rows of the
// value and of U for the 16 samples (2 KiB rows, coalesced), forms clip_k and att_k, and the soft attention follows
// as softattn_fwd4_kernel computes it (the same per-thread sums, block reduction and softmax).  clip, att, save_loc
// and probs are written for the backward; the separate soft-attention pass no longer reads clip and att back.
// -------------------------------------------------------------------------------------------------
constexpr int kCSA = 128;  // threads per fused caption-step workgroup (512 channels as float4s)

template <int RD, int CH>
__global__ __launch_bounds__(kCSA) void cap_softattn_fwd_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ U,
    const int32_t* __restrict__ row_video, const float* __restrict__ offsets, int off_stride, int off_col0,
    const float* __restrict__ off_add, const float* __restrict__ ref, int rd1_rows, CapLevels lv, int S, int M,
    const float* __restrict__ att_h, int ldh, const float* __restrict__ aw, const float* __restrict__ ab,
    float* __restrict__ clip, float* __restrict__ save_loc, float* __restrict__ att, float* __restrict__ probs,
    float* __restrict__ res) {
    constexpr int D = 512, D4 = D / 4;
    __shared__ int srow0[cNS], srow1[cNS], sfl[cNS];
    __shared__ float snw[cNS], sne[cNS], red[3 * cNS];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int r = wg / M, m = wg - r * M;
    const int b = row_video[r];
    const size_t MD = (size_t)M * D;
    const size_t so = (size_t)wg * cNS;  // (r * M + m) * 16
    if (tid < cNS) {
        const int j = tid, l = j >> 2;
        const int T = lv.T[0] * (l == 0) + lv.T[1] * (l == 1) + lv.T[2] * (l == 2) + lv.T[3] * (l == 3);
        const int st = lv.start[0] * (l == 0) + lv.start[1] * (l == 1) + lv.start[2] * (l == 2) + lv.start[3] * (l == 3);
        const float* orow = offsets + (size_t)r * off_stride + off_col0 + m * cNS;
        const float off = off_add ? orow[j] + off_add[((size_t)r * M + m) * cNS + j] : orow[j];
        const bool centre_only = (RD == 1) || (r < rd1_rows);
        const float r0 = ref[((size_t)r * cL + l) * RD];
        const float r1 = (RD == 2) ? ref[((size_t)r * cL + l) * RD + 1] : 0.f;
        const float loc = centre_only ? r0 + off / (float)T : r0 + ((off / (float)cP) * r1) * 0.5f;
        save_loc[so + j] = loc;
        float gm;
        const float ix = border_ix(loc, T, gm);
        const float xf = floorf(ix);
        const int x0 = (int)xf, a1 = min(x0 + 1, T - 1);
        const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
        const bool ok0 = !(mbase && mbase[st + x0]);
        const bool ok1 = x0 + 1 < T && !(mbase && mbase[st + a1]);
        srow0[j] = st + x0;
        srow1[j] = st + a1;
        sfl[j] = (ok0 ? 1 : 0) | (ok1 ? 2 : 0) | (x0 + 1 < T ? 4 : 0);
        snw[j] = ((float)(x0 + 1) - ix);
        sne[j] = (ix - xf);
    }
    __syncthreads();
    const float4* vb = reinterpret_cast<const float4*>(value + (size_t)b * S * MD + (size_t)m * D) + tid;
    const float4* ub = reinterpret_cast<const float4*>(U + (size_t)b * S * MD + (size_t)m * D) + tid;
    const size_t MD4 = MD / 4;
    const float4 hv = reinterpret_cast<const float4*>(att_h + (size_t)r * ldh)[tid];
    const float4 wv = reinterpret_cast<const float4*>(aw)[tid];
    float4* c4 = reinterpret_cast<float4*>(clip + so * D) + tid;
    float4* a4 = reinterpret_cast<float4*>(att + so * D) + tid;
    float4 cl[cNS];
    float part[cNS];
#pragma unroll
    for (int k0 = 0; k0 < cNS; k0 += CH) {  // CH samples' corner rows per chunk (CH = 4: 228 registers, 1: 160)
        float4 v0[CH], v1[CH], u0[CH], u1[CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const size_t o0 = (size_t)srow0[k0 + q] * MD4, o1 = (size_t)srow1[k0 + q] * MD4;
            v0[q] = vb[o0];
            v1[q] = vb[o1];
            u0[q] = ub[o0];
            u1[q] = ub[o1];
        }
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int k = k0 + q, fl = sfl[k];
            const float nw = snw[k], ne = sne[k];
            const bool k0ok = fl & 1, k1ok = fl & 2, hi = fl & 4;
            cl[k] = make_float4((k0ok ? v0[q].x : 0.f) * nw + (k1ok ? v1[q].x : 0.f) * ne,
                                (k0ok ? v0[q].y : 0.f) * nw + (k1ok ? v1[q].y : 0.f) * ne,
                                (k0ok ? v0[q].z : 0.f) * nw + (k1ok ? v1[q].z : 0.f) * ne,
                                (k0ok ? v0[q].w : 0.f) * nw + (k1ok ? v1[q].w : 0.f) * ne);
            const float4 a = make_float4(u0[q].x * nw + (hi ? u1[q].x : 0.f) * ne, u0[q].y * nw + (hi ? u1[q].y : 0.f) * ne,
                                         u0[q].z * nw + (hi ? u1[q].z : 0.f) * ne, u0[q].w * nw + (hi ? u1[q].w : 0.f) * ne);
            if (clip) {  // NULL: the fused backward re-forms the samples from their corners
                c4[(size_t)k * D4] = cl[k];
                a4[(size_t)k * D4] = a;
            }
            part[k] = 0.f + (tanhf(a.x + hv.x) * wv.x + tanhf(a.y + hv.y) * wv.y + tanhf(a.z + hv.z) * wv.z +
                             tanhf(a.w + hv.w) * wv.w);
        }
    }
    // softattn_fwd4_kernel's block sum, softmax and weighted sum
    group_reduce_scatter<cNS, 16>(part, lane);
    float v = part[0];
    v += lane_swap(v, 16);
    v += __shfl_xor(v, 32, 64);
    if (lane < cNS) red[wid * cNS + lane] = v;
    __syncthreads();
    if (tid < cNS) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kCSA / 64; ++w) t += red[w * cNS + tid];
        red[2 * cNS + tid] = t;
    }
    __syncthreads();
    const float* dots = red + 2 * cNS;
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < cNS; ++k) mx = fmaxf(mx, dots[k] + ab[0]);
    float p[cNS], sum = 0.f;
#pragma unroll
    for (int k = 0; k < cNS; ++k) {
        p[k] = expf(dots[k] + ab[0] - mx);
        sum += p[k];
    }
    const float inv = 1.f / sum;
#pragma unroll
    for (int k = 0; k < cNS; ++k) p[k] = p[k] * inv;
    if (tid < cNS) {
        float pj = 0.f;
#pragma unroll
        for (int k = 0; k < cNS; ++k) pj = (k == tid) ? p[k] : pj;
        probs[so + tid] = pj;
    }
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < cNS; ++k) {
        o.x += p[k] * cl[k].x;
        o.y += p[k] * cl[k].y;
        o.z += p[k] * cl[k].z;
        o.w += p[k] * cl[k].w;
    }
    reinterpret_cast<float4*>(res + (size_t)r * MD + (size_t)m * D)[tid] = o;
}

// The backward of cap_softattn_fwd_kernel (512-wide head; the u_grad form of the caption decode): softattn_bwd4_kernel
// (capstep.hip) and cap_gather_bwd_kernel with value2 = U in one launch.  The samples and att are re-formed from the
// corner rows the location gradient reads anyway (the forward then writes neither); the sample gradients (p_k * dres)
// and att gradients are written for the destination-sorted value / U passes after the loop.  A sample's location
// gradient, dsample_k . (v1 - v0) + datt_k . (u1 - u0), factors as p_k (dres . (v1 - v0)) + dd_k (w (1 - t^2)) . (u1 - u0)
// (dd_k the softmax backward's scalar): its two channel sums are reduced with the 16 dots in one block reduction,
// and only the 16 tanh rows stay in registers for the att gradients.  One 128-thread workgroup per (row, head).
constexpr int cRED = 3 * cNS;  // dots, value-difference sums, U-difference sums

template <int RD, int CH>
__global__ __launch_bounds__(kCSA) void cap_softattn_bwd_kernel(
    const float* __restrict__ value, const uint8_t* __restrict__ vmask, const float* __restrict__ U,
    const int32_t* __restrict__ row_video, const float* __restrict__ offsets, int off_stride, int off_col0,
    const float* __restrict__ off_add, const float* __restrict__ ref, int rd1_rows, CapLevels lv, int S, int M,
    const float* __restrict__ save_loc, const float* __restrict__ probs, const float* __restrict__ gres,
    const float* __restrict__ att_h, int ldh, const float* __restrict__ aw, float* __restrict__ gatt,
    float* __restrict__ gatt_h, int ldgh, float* __restrict__ gclip, float* __restrict__ gaw_part,
    float* __restrict__ gab_part, float* __restrict__ grad_off, float* __restrict__ grad_ref) {
    constexpr int D = 512, D4 = D / 4;
    __shared__ int srow0[cNS], srow1[cNS], sfl[cNS];
    __shared__ float snw[cNS], sne[cNS], red[(kCSA / 64 + 1) * cRED];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int r = wg / M, m = wg - r * M;
    const int b = row_video[r];
    const size_t MD = (size_t)M * D;
    const size_t so = (size_t)wg * cNS;
    float gm = 0.f;
    int T = 1;
    if (tid < cNS) {
        const int j = tid, l = j >> 2;
        T = lv.T[0] * (l == 0) + lv.T[1] * (l == 1) + lv.T[2] * (l == 2) + lv.T[3] * (l == 3);
        const int st = lv.start[0] * (l == 0) + lv.start[1] * (l == 1) + lv.start[2] * (l == 2) + lv.start[3] * (l == 3);
        const float ix = border_ix(save_loc[so + j], T, gm);
        const float xf = floorf(ix);
        const int x0 = (int)xf, a1 = min(x0 + 1, T - 1);
        const uint8_t* mbase = vmask ? vmask + (size_t)b * S : nullptr;
        const bool ok0 = !(mbase && mbase[st + x0]);
        const bool ok1 = x0 + 1 < T && !(mbase && mbase[st + a1]);
        srow0[j] = st + x0;
        srow1[j] = st + a1;
        sfl[j] = (ok0 ? 1 : 0) | (ok1 ? 2 : 0) | (x0 + 1 < T ? 4 : 0);
        snw[j] = ((float)(x0 + 1) - ix);
        sne[j] = (ix - xf);
    }
    __syncthreads();
    const float4* vb = reinterpret_cast<const float4*>(value + (size_t)b * S * MD + (size_t)m * D) + tid;
    const float4* ub = reinterpret_cast<const float4*>(U + (size_t)b * S * MD + (size_t)m * D) + tid;
    const size_t MD4 = MD / 4;
    const float4 g = reinterpret_cast<const float4*>(gres + (size_t)r * MD + (size_t)m * D)[tid];
    const float4 hv = reinterpret_cast<const float4*>(att_h + (size_t)r * ldh)[tid];
    const float4 wv = reinterpret_cast<const float4*>(aw)[tid];
    float p[cNS];
#pragma unroll
    for (int k = 0; k < cNS; ++k) p[k] = probs[so + k];
    float4* gc4 = reinterpret_cast<float4*>(gclip + so * D) + tid;
    float4 th[cNS];    // tanh(att_k + att_h)
    float part[cRED];  // [0,16): dres . sample_k   [16,32): dres . (v1 - v0)_k   [32,48): (w (1 - t^2)) . (u1 - u0)_k
#pragma unroll
    for (int k0 = 0; k0 < cNS; k0 += CH) {  // CH samples' corner rows per chunk
        float4 v0[CH], v1[CH], u0[CH], u1[CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const size_t o0 = (size_t)srow0[k0 + q] * MD4, o1 = (size_t)srow1[k0 + q] * MD4;
            v0[q] = vb[o0];
            v1[q] = vb[o1];
            u0[q] = ub[o0];
            u1[q] = ub[o1];
        }
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int k = k0 + q, fl = sfl[k];
            const float nw = snw[k], ne = sne[k];
            const bool k0ok = fl & 1, k1ok = fl & 2, hi = fl & 4;
            const float4 a0 = make_float4(k0ok ? v0[q].x : 0.f, k0ok ? v0[q].y : 0.f, k0ok ? v0[q].z : 0.f,
                                          k0ok ? v0[q].w : 0.f);
            const float4 a1 = make_float4(k1ok ? v1[q].x : 0.f, k1ok ? v1[q].y : 0.f, k1ok ? v1[q].z : 0.f,
                                          k1ok ? v1[q].w : 0.f);
            const float4 cl = make_float4(a0.x * nw + a1.x * ne, a0.y * nw + a1.y * ne, a0.z * nw + a1.z * ne,
                                          a0.w * nw + a1.w * ne);
            const float4 h1 = make_float4(hi ? u1[q].x : 0.f, hi ? u1[q].y : 0.f, hi ? u1[q].z : 0.f,
                                          hi ? u1[q].w : 0.f);
            const float4 at = make_float4(u0[q].x * nw + h1.x * ne, u0[q].y * nw + h1.y * ne,
                                          u0[q].z * nw + h1.z * ne, u0[q].w * nw + h1.w * ne);
            th[k] = make_float4(tanhf(at.x + hv.x), tanhf(at.y + hv.y), tanhf(at.z + hv.z), tanhf(at.w + hv.w));
            part[k] = 0.f + (g.x * cl.x + g.y * cl.y + g.z * cl.z + g.w * cl.w);
            part[cNS + k] = g.x * (a1.x - a0.x) + g.y * (a1.y - a0.y) + g.z * (a1.z - a0.z) + g.w * (a1.w - a0.w);
            part[2 * cNS + k] = wv.x * (1.f - th[k].x * th[k].x) * (h1.x - u0[q].x) +
                                wv.y * (1.f - th[k].y * th[k].y) * (h1.y - u0[q].y) +
                                wv.z * (1.f - th[k].z * th[k].z) * (h1.z - u0[q].z) +
                                wv.w * (1.f - th[k].w * th[k].w) * (h1.w - u0[q].w);
            if (gclip) gc4[(size_t)k * D4] = make_float4(p[k] * g.x, p[k] * g.y, p[k] * g.z, p[k] * g.w);
        }
        // CH = 4: one chunk's 16 rows in flight at a time (454 registers without the barrier, 449 with: one wave per
        // SIMD); CH = 1: 252 registers, two waves per SIMD, the scheduler hoisting the next samples' loads itself
        if constexpr (CH > 1) __builtin_amdgcn_sched_barrier(0);
    }
    // the 48 channel sums over the workgroup: lane r of each 16-lane group ends with values [3r, 3r + 3)
    group_reduce_scatter<cRED, 16>(part, lane);
#pragma unroll
    for (int i = 0; i < cRED / 16; ++i) {
        float v = part[i];
        v += lane_swap(v, 16);
        v += __shfl_xor(v, 32, 64);
        if (lane < 16) red[wid * cRED + lane * (cRED / 16) + i] = v;
    }
    __syncthreads();
    if (tid < cRED) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kCSA / 64; ++w) t += red[w * cRED + tid];
        red[(kCSA / 64) * cRED + tid] = t;
    }
    __syncthreads();
    const float* dp = red + (kCSA / 64) * cRED;  // dots, then the two difference sums
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < cNS; ++k) t += p[k] * dp[k];
    float dd[cNS], sb = 0.f;
#pragma unroll
    for (int k = 0; k < cNS; ++k) {
        dd[k] = p[k] * (dp[k] - t);
        sb += dd[k];
    }
    if (tid == 0) gab_part[wg] = sb;
    float4* ga4 = reinterpret_cast<float4*>(gatt + so * D) + tid;
    float4 gh = make_float4(0.f, 0.f, 0.f, 0.f), gw = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < cNS; ++k) {
        const float tx = th[k].x, ty = th[k].y, tz = th[k].z, tw = th[k].w;
        const float4 dpre = make_float4(dd[k] * wv.x * (1.f - tx * tx), dd[k] * wv.y * (1.f - ty * ty),
                                        dd[k] * wv.z * (1.f - tz * tz), dd[k] * wv.w * (1.f - tw * tw));
        ga4[(size_t)k * D4] = dpre;
        gh.x += dpre.x; gh.y += dpre.y; gh.z += dpre.z; gh.w += dpre.w;
        gw.x += dd[k] * tx; gw.y += dd[k] * ty; gw.z += dd[k] * tz; gw.w += dd[k] * tw;
    }
    if (M == 1) {
        reinterpret_cast<float4*>(gatt_h + (size_t)r * ldgh)[tid] = gh;
    } else {
        float* gp = gatt_h + (size_t)r * ldgh + 4 * tid;
        atomicAdd(gp, gh.x); atomicAdd(gp + 1, gh.y); atomicAdd(gp + 2, gh.z); atomicAdd(gp + 3, gh.w);
    }
    reinterpret_cast<float4*>(gaw_part + (size_t)wg * D)[tid] = gw;
    if (tid < cNS) {  // offset and reference gradients of sample j (cap_gather_bwd_kernel's chain)
        const int j = tid, l = j >> 2;
        float pj = 0.f, dj = 0.f;
#pragma unroll
        for (int k = 0; k < cNS; ++k) {
            pj = (k == j) ? p[k] : pj;
            dj = (k == j) ? dd[k] : dj;
        }
        const float s = pj * dp[cNS + j] + dj * dp[2 * cNS + j];
        const bool centre_only = (RD == 1) || (r < rd1_rows);
        const float gloc = 2.f * (gm * s);  // grid = 2*loc - 1
        float goff, gr0 = gloc, gr1 = 0.f;
        if (centre_only) {
            goff = gloc / (float)T;
        } else {
            const float r1 = ref[((size_t)r * cL + l) * 2 + 1];
            const float t2 = gloc * 0.5f;
            goff = (t2 * r1) / (float)cP;
            float o = offsets[(size_t)r * off_stride + off_col0 + m * cNS + j];
            if (off_add) o += off_add[((size_t)r * M + m) * cNS + j];
            gr1 = t2 * (o / (float)cP);
        }
        grad_off[(size_t)r * off_stride + off_col0 + m * cNS + j] = goff;
        if (grad_ref) {  // the level's four points summed, one atomic per (row, head, level)
            gr0 += lane_swap(gr0, 1);
            gr0 += lane_swap(gr0, 2);
            if (RD == 2) {
                gr1 += lane_swap(gr1, 1);
                gr1 += lane_swap(gr1, 2);
            }
            if ((j & 3) == 0) {
                atomicAdd(grad_ref + ((size_t)r * cL + l) * RD, gr0);
                if (RD == 2) atomicAdd(grad_ref + ((size_t)r * cL + l) * RD + 1, gr1);
            }
        }
    }
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
                     off_add, ref, rd1_rows, lv, S, num_heads, head_dim, wpr, (int)tw, samples, save_loc, cap_remap())
    } else {
        CAP_DISPATCH(cap_gather_fwd_kernel, 2, grid, s, value, value_pad_mask, row_video, offsets, off_stride, off_col0,
                     off_add, ref, rd1_rows, lv, S, num_heads, head_dim, wpr, (int)tw, samples, save_loc, cap_remap())
    }
    PDVC_CHECK_LAUNCH("cap_gather_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_cap_gather_backward2_f32(const float* value, const uint8_t* value_pad_mask,
                                             const int32_t* row_video, const float* offsets, int off_stride,
                                             int off_col0, const float* off_add, const float* ref, int ref_dim,
                                             int rd1_rows, const int32_t* level_T, int num_levels, int batch, int rows,
                                             int num_heads, int head_dim, int num_point, const float* save_loc,
                                             const float* grad_samples, float* grad_value, float* grad_offsets,
                                             float* grad_ref, const float* value2, const float* grad_samples2,
                                             void* stream) {
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
                     grad_value, grad_offsets, grad_ref, value2, grad_samples2, cap_remap())
    } else {
        CAP_DISPATCH(cap_gather_bwd_kernel, 2, grid, s, value, value_pad_mask, row_video, offsets, off_stride, off_col0,
                     off_add, ref, rd1_rows, lv, S, num_heads, head_dim, wpr, (int)tw, save_loc, grad_samples,
                     grad_value, grad_offsets, grad_ref, value2, grad_samples2, cap_remap())
    }
    PDVC_CHECK_LAUNCH("cap_gather_bwd_kernel");
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
    return pdvc_cap_gather_backward2_f32(value, value_pad_mask, row_video, offsets, off_stride, off_col0, off_add, ref,
                                         ref_dim, rd1_rows, level_T, num_levels, batch, rows, num_heads, head_dim,
                                         num_point, save_loc, grad_samples, grad_value, grad_offsets, grad_ref, nullptr,
                                         nullptr, stream);
}

extern "C" int pdvc_cap_value_grad_ex_f32(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels,
                                          int batch, int num_heads, int head_dim, int num_point, int rows, int steps,
                                          int max_rows_per_video, const int32_t* video_row_start,
                                          const int32_t* video_rows, const float* save_loc, const float* grad_samples,
                                          float* grad_value, float* grad_value_level_sums, void* stream) {
    return pdvc_cap_value_grad_ranged_f32(value_pad_mask, level_T, num_levels, batch, num_heads, head_dim, num_point,
                                          rows, steps, max_rows_per_video, video_row_start, video_rows, nullptr,
                                          save_loc, grad_samples, grad_value, grad_value_level_sums, stream);
}

static int cap_value_grad_impl(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels, int batch,
                               int num_heads, int head_dim, int num_point, int rows, int steps,
                               int max_rows_per_video, const int32_t* video_row_start, const int32_t* video_rows,
                               const int32_t* step_rows, const float* save_loc, const float* grad_samples,
                               const float* grad_rows, const float* grad_scale, float* grad_value,
                               float* grad_value_level_sums, uint16_t* gv16, void* stream) {
    float* level_sums = grad_value_level_sums;
    CapLevels lv;
    int S = 0;
    PDVC_CHECK_ARG(level_T != nullptr && num_levels == cL && num_point == cP, "caption value gradient needs %d x %d",
                   cL, cP);
    for (int l = 0; l < cL; ++l) {
        PDVC_CHECK_ARG(level_T[l] > 0, "level %d has non-positive length", l);
        lv.T[l] = level_T[l];
        lv.start[l] = S;
        S += level_T[l];
    }
    PDVC_CHECK_ARG(head_dim > 0 && head_dim <= 512, "head_dim must be in [1, 512], got %d", head_dim);
    PDVC_CHECK_ARG(batch >= 0 && num_heads > 0 && rows >= 0 && steps >= 0 && max_rows_per_video >= 0, "invalid sizes");
    hipStream_t s = (hipStream_t)stream;
    const long nblk = (long)batch * num_heads * cL;
    if (nblk == 0) return PDVC_OK;
    if (steps == 0 || max_rows_per_video == 0) {
        const size_t nv = (size_t)batch * S * num_heads * head_dim;
        hipError_t e = zero_async(grad_value, nv, s);
        if (e == hipSuccess && gv16) e = zero_async(reinterpret_cast<float*>(gv16), nv / 2, s);  // (nv even: checked)
        if (e == hipSuccess && level_sums) e = zero_async(level_sums, (size_t)batch * cL * num_heads * head_dim, s);
        return e == hipSuccess ? PDVC_OK : pdvc_set_error(PDVC_ERR_LAUNCH, "memset: %s", hipGetErrorString(e));
    }
    int Tmax = 0;
    for (int l = 0; l < cL; ++l) Tmax = lv.T[l] > Tmax ? lv.T[l] : Tmax;
    const long budget = 96 * 1024 - 8L * (Tmax + 2);
    const long per_step = 12L * max_rows_per_video * cP;  // LDS bytes per step of samples
    PDVC_CHECK_ARG(budget >= per_step, "too many caption rows per video (%d) for one step in LDS", max_rows_per_video);
    const int chunk = (int)(budget / per_step);
    static std::atomic<int> done[kMaxDevices];
    if (const int rc = lds_optin(done, {{(const void*)cap_value_grad_kernel<1>, 96 * 1024},
                                        {(const void*)cap_value_grad_kernel<2>, 96 * 1024},
                                        {(const void*)cap_value_grad_kernel<4>, 96 * 1024},
                                        {(const void*)cap_value_grad_kernel<8>, 96 * 1024}},
                                 "cap_value_grad_kernel"))
        return rc;
    const int cw = head_dim <= 64 ? 1 : head_dim <= 128 ? 2 : head_dim <= 256 ? 4 : 8;
    for (int s0 = 0; s0 < steps; s0 += chunk) {
        const int ns = steps - s0 < chunk ? steps - s0 : chunk;
        size_t lds = sizeof(int) * (2 * (size_t)(Tmax + 2) + 3 * (size_t)ns * max_rows_per_video * cP);
        const size_t red = sizeof(float) * kCVW * 64 * cw;  // the level-sum reduction
        if (level_sums && lds < red) lds = red;
        const int acc = s0 > 0;
        const dim3 grid((unsigned)nblk), block(kCVW * 64);
#define CVG(CW) hipLaunchKernelGGL((cap_value_grad_kernel<CW>), grid, block, lds, s, value_pad_mask, lv, S, num_heads, \
                                   head_dim, rows, s0, ns, acc, video_row_start, video_rows, save_loc, grad_samples,     \
                                   grad_value, level_sums, step_rows, grad_rows, grad_scale, gv16)
        if (cw == 1) CVG(1);
        else if (cw == 2) CVG(2);
        else if (cw == 4) CVG(4);
        else CVG(8);
#undef CVG
        PDVC_CHECK_LAUNCH("cap_value_grad_kernel");
    }
    return PDVC_OK;
}

extern "C" int pdvc_cap_value_grad_ranged_f32(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels,
                                              int batch, int num_heads, int head_dim, int num_point, int rows,
                                              int steps, int max_rows_per_video, const int32_t* video_row_start,
                                              const int32_t* video_rows, const int32_t* step_rows,
                                              const float* save_loc, const float* grad_samples, float* grad_value,
                                              float* grad_value_level_sums, void* stream) {
    PDVC_CHECK_ARG(grad_samples != nullptr, "grad_samples must not be NULL");
    return cap_value_grad_impl(value_pad_mask, level_T, num_levels, batch, num_heads, head_dim, num_point, rows, steps,
                               max_rows_per_video, video_row_start, video_rows, step_rows, save_loc, grad_samples,
                               nullptr, nullptr, grad_value, grad_value_level_sums, nullptr, stream);
}

// The same pass with rank-1 sample gradients: sample s = (step, row, head, k) has gradient grad_scale[s] *
// grad_rows[(step, row, head)] (grad_rows (steps, rows, heads, head_dim), grad_scale (steps, rows, heads, 16)) -- the
// caption step's p_k * dres, which pdvc_cap_softattn_backward_f32 then need not write 16 times per row.
extern "C" int pdvc_cap_value_grad_rank1_f32(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels,
                                             int batch, int num_heads, int head_dim, int num_point, int rows,
                                             int steps, int max_rows_per_video, const int32_t* video_row_start,
                                             const int32_t* video_rows, const int32_t* step_rows,
                                             const float* save_loc, const float* grad_rows, const float* grad_scale,
                                             float* grad_value, float* grad_value_level_sums, void* stream) {
    PDVC_CHECK_ARG(grad_rows != nullptr && grad_scale != nullptr, "grad_rows and grad_scale must not be NULL");
    return cap_value_grad_impl(value_pad_mask, level_T, num_levels, batch, num_heads, head_dim, num_point, rows, steps,
                               max_rows_per_video, video_row_start, video_rows, step_rows, save_loc, nullptr,
                               grad_rows, grad_scale, grad_value, grad_value_level_sums, nullptr, stream);
}

extern "C" int pdvc_cap_value_grad_f32(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels,
                                       int batch, int num_heads, int head_dim, int num_point, int rows, int steps,
                                       int max_rows_per_video, const int32_t* video_row_start,
                                       const int32_t* video_rows, const float* save_loc, const float* grad_samples,
                                       float* grad_value, void* stream) {
    return pdvc_cap_value_grad_ex_f32(value_pad_mask, level_T, num_levels, batch, num_heads, head_dim, num_point, rows,
                                      steps, max_rows_per_video, video_row_start, video_rows, save_loc, grad_samples,
                                      grad_value, nullptr, stream);
}

// One caption step's sampling of the value rows (with value_pad_mask) and of the projected ctx2att rows U (same shape,
// no mask) plus the soft attention over the 16 samples: pdvc_cap_gather_forward_f32 twice and pdvc_softattn_forward_f32
// in one launch, for head_dim = attention width = 512 (every cfg's cap_nheads 1).  Outputs as theirs.
extern "C" int pdvc_cap_softattn_forward_f32(const float* value, const uint8_t* value_pad_mask, const float* U,
                                             const int32_t* row_video, const float* offsets, int off_stride,
                                             int off_col0, const float* off_add, const float* ref, int ref_dim,
                                             int rd1_rows, const int32_t* level_T, int num_levels, int batch,
                                             int rows, int num_heads, int head_dim, int num_point,
                                             const float* att_h, int ld_att_h, const float* alpha_w,
                                             const float* alpha_b, float* samples, float* save_loc, float* att,
                                             float* probs, float* res, void* stream) {
    CapLevels lv;
    int S, lph, wpr;
    int rc = cap_setup(level_T, num_levels, num_point, head_dim, num_heads, ref_dim, lv, S, lph, wpr);
    if (rc) return rc;
    if (head_dim != 512)
        return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "fused caption step needs head_dim 512, got %d", head_dim);
    PDVC_CHECK_ARG(U && att_h && alpha_w && alpha_b && save_loc && probs && res && (!samples) == (!att),
                   "fused caption step: NULL argument");
    PDVC_CHECK_ARG(off_col0 >= 0 && off_col0 + num_heads * cNS <= off_stride, "offset columns out of range");
    PDVC_CHECK_ARG(batch >= 0 && rows >= 0 && ld_att_h >= 512, "invalid sizes");
    const void* al[] = {value, U, att_h, alpha_w, samples, att, res};
    for (const void* q : al)
        if ((uintptr_t)q % 16) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "fused caption step needs 16-B alignment");
    if (ld_att_h % 4) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "fused caption step needs ld_att_h % 4 == 0");
    const long nwg = (long)rows * num_heads;
    if (nwg == 0) return PDVC_OK;
    PDVC_CHECK_ARG(nwg < (1L << 31), "too many rows");
    hipStream_t s = (hipStream_t)stream;
    static const int ch = [] {  // PDVC_CAP_FWD_CH=4: the 4-sample chunks (same-box A/B)
        const char* e = getenv("PDVC_CAP_FWD_CH");
        return e && e[0] == '4' ? 4 : 1;
    }();
    auto kern = ref_dim == 1 ? (ch == 4 ? cap_softattn_fwd_kernel<1, 4> : cap_softattn_fwd_kernel<1, 1>)
                             : (ch == 4 ? cap_softattn_fwd_kernel<2, 4> : cap_softattn_fwd_kernel<2, 1>);
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(kCSA), 0, s, value, value_pad_mask, U, row_video, offsets,
                       off_stride, off_col0, off_add, ref, rd1_rows, lv, S, num_heads, att_h, ld_att_h, alpha_w,
                       alpha_b, samples, save_loc, att, probs, res);
    PDVC_CHECK_LAUNCH("cap_softattn_fwd_kernel");
    return PDVC_OK;
}

// The backward of pdvc_cap_softattn_forward_f32 in the caption decoder's u_grad form (the value and U gradients come
// from the destination-sorted passes after the loop): pdvc_softattn_backward_f32 and pdvc_cap_gather_backward2_f32 in
// one launch, re-forming the samples and att from their corner rows (the forward may then skip writing them).
extern "C" int pdvc_cap_softattn_backward_f32(const float* value, const uint8_t* value_pad_mask, const float* U,
                                              const int32_t* row_video, const float* offsets, int off_stride,
                                              int off_col0, const float* off_add, const float* ref, int ref_dim,
                                              int rd1_rows, const int32_t* level_T, int num_levels, int batch,
                                              int rows, int num_heads, int head_dim, int num_point,
                                              const float* save_loc, const float* probs, const float* grad_res,
                                              const float* att_h, int ld_att_h, const float* alpha_w,
                                              float* grad_att, float* grad_att_h, int ld_grad_att_h,
                                              float* grad_samples, float* grad_alpha_w_part,
                                              float* grad_alpha_b_part, float* grad_offsets, float* grad_ref,
                                              void* stream) {
    CapLevels lv;
    int S, lph, wpr;
    int rc = cap_setup(level_T, num_levels, num_point, head_dim, num_heads, ref_dim, lv, S, lph, wpr);
    if (rc) return rc;
    if (head_dim != 512)
        return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "fused caption step needs head_dim 512, got %d", head_dim);
    PDVC_CHECK_ARG(value && U && row_video && offsets && ref && save_loc && probs && grad_res && att_h && alpha_w &&
                       grad_att && grad_att_h && grad_alpha_w_part && grad_alpha_b_part && grad_offsets,
                   "fused caption step backward: NULL argument");
    PDVC_CHECK_ARG(off_col0 >= 0 && off_col0 + num_heads * cNS <= off_stride, "offset columns out of range");
    PDVC_CHECK_ARG(batch >= 0 && rows >= 0 && ld_att_h >= 512 && ld_grad_att_h >= 512, "invalid sizes");
    const void* al[] = {value, U, grad_res, att_h, alpha_w, grad_att, grad_att_h, grad_samples, grad_alpha_w_part};
    for (const void* q : al)
        if ((uintptr_t)q % 16) return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "fused caption step needs 16-B alignment");
    if (ld_att_h % 4 || ld_grad_att_h % 4)
        return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "fused caption step needs row strides % 4 == 0");
    const long nwg = (long)rows * num_heads;
    if (nwg == 0) return PDVC_OK;
    PDVC_CHECK_ARG(nwg < (1L << 31), "too many rows");
    hipStream_t s = (hipStream_t)stream;
    static const int ch = [] {  // PDVC_CAP_BWD_CH=4: the 4-sample chunks (same-box A/B)
        const char* e = getenv("PDVC_CAP_BWD_CH");
        return e && e[0] == '4' ? 4 : 1;
    }();
    auto kern = ref_dim == 1 ? (ch == 4 ? cap_softattn_bwd_kernel<1, 4> : cap_softattn_bwd_kernel<1, 1>)
                             : (ch == 4 ? cap_softattn_bwd_kernel<2, 4> : cap_softattn_bwd_kernel<2, 1>);
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(kCSA), 0, s, value, value_pad_mask, U, row_video, offsets,
                       off_stride, off_col0, off_add, ref, rd1_rows, lv, S, num_heads, save_loc, probs, grad_res, att_h,
                       ld_att_h, alpha_w, grad_att, grad_att_h, ld_grad_att_h, grad_samples, grad_alpha_w_part,
                       grad_alpha_b_part, grad_offsets, grad_ref);
    PDVC_CHECK_LAUNCH("cap_softattn_bwd_kernel");
    return PDVC_OK;
}

// pdvc_cap_value_grad_ranged_f32 plus the bf16 rounding of grad_value at the same offsets (the bf16 mode: the caption
// head's value-gradient operand of the projections' GEMMs, written by the pass that writes grad_value)
extern "C" int pdvc_cap_value_grad_ranged_f32_bf16out(const uint8_t* value_pad_mask, const int32_t* level_T,
                                                      int num_levels, int batch, int num_heads, int head_dim,
                                                      int num_point, int rows, int steps, int max_rows_per_video,
                                                      const int32_t* video_row_start, const int32_t* video_rows,
                                                      const int32_t* step_rows, const float* save_loc,
                                                      const float* grad_samples, float* grad_value,
                                                      float* grad_value_level_sums, uint16_t* grad_value16,
                                                      void* stream) {
    PDVC_CHECK_ARG(grad_samples != nullptr, "grad_samples must not be NULL");
    PDVC_CHECK_ARG(grad_value16 != nullptr && ((uintptr_t)grad_value16 % 4) == 0 && (num_heads * head_dim) % 2 == 0,
                   "grad_value16: a 4-byte aligned bf16 buffer, num_heads * head_dim even");
    return cap_value_grad_impl(value_pad_mask, level_T, num_levels, batch, num_heads, head_dim, num_point, rows, steps,
                               max_rows_per_video, video_row_start, video_rows, step_rows, save_loc, grad_samples,
                               nullptr, nullptr, grad_value, grad_value_level_sums, grad_value16, stream);
}
