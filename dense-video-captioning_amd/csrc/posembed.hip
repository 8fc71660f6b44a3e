// posembed.hip -- the encoder's positional input lvl_pos (N, S, C), all pyramid levels in one pass
//
// Reference: PositionEmbeddingSine.forward (pdvc/position_encoding.py:20-75) per level -- sine features of
// the level's normalised cumulative position (channels [0, F)) next to the video's duration embedding
// (channels [F, C)) -- then DeformableTransformer's  pos_l + level_embed[l]  and the concatenation over levels
// (deformable_transformer.py:100-112).  torch spends a dozen launches per level on it (div, sin, cos, stack,
// cat with the broadcast duration rows, the level add, the final cat): 2-3 passes over (N, S, C).  Here one
// thread writes one float4 of lvl_pos:
//     lvl_pos[n, s, c] = (c < F ? (c even ? sin : cos)(xe[n, s] / dim_t[c]) : dur[n, c - F]) + level_embed[l(s), c]
// with xe the normalised positions (tiny, computed by the host-side torch ops of the reference) and dim_t the
// reference's frequency table -- the same fp32 division, sin/cos and add, in the reference's order.
// Backward: per (video, level) column sums of dlvl_pos in one read (grid: video x level x 64-column tile);
// the level-embedding gradient and the duration-embedding gradient are sums of those partials.
#include "pdvc_common.h"

namespace pdvc {

constexpr int kPosMaxLevels = 8;

struct PosLevels {
    int start[kPosMaxLevels + 1];
    int n;
};

__device__ __forceinline__ int pos_level(const PosLevels& lv, int s) {
    int l = 0;
#pragma unroll
    for (int k = 1; k < kPosMaxLevels; ++k) l += (k < lv.n && s >= lv.start[k]) ? 1 : 0;
    return l;
}

__global__ __launch_bounds__(256) void level_pos_fwd_kernel(const float* __restrict__ xe,
                                                            const float* __restrict__ dim_t,
                                                            const float* __restrict__ dur,
                                                            const float* __restrict__ lemb, PosLevels lv, int N,
                                                            int S, int F, int Dd, const float* __restrict__ add,
                                                            float* __restrict__ pos, uint16_t* __restrict__ pos16) {
    const int C = F + Dd, c4n = C / 4;
    const long total = (long)N * S * c4n;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long r = i / c4n;
        const int c = (int)(i - r * c4n) * 4;
        const int n = (int)(r / S), s = (int)(r - (long)n * S);
        const int l = pos_level(lv, s);
        const float4 le = *reinterpret_cast<const float4*>(lemb + (size_t)l * C + c);
        float v[4];
        if (c < F) {  // F % 4 == 0: a float4 never straddles the sine / duration boundary
            const float x = xe[r];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float a = x / dim_t[c + k];
                v[k] = ((c + k) & 1) ? cosf(a) : sinf(a);
            }
        } else {
            const float4 d = *reinterpret_cast<const float4*>(dur + (size_t)n * Dd + (c - F));
            v[0] = d.x;
            v[1] = d.y;
            v[2] = d.z;
            v[3] = d.w;
        }
        float4 o = make_float4(v[0] + le.x, v[1] + le.y, v[2] + le.z, v[3] + le.w);
        if (add) {  // q = src + lvl_pos, in that order (deformable_transformer.py:146 with_pos_embed)
            const float4 a = reinterpret_cast<const float4*>(add)[i];
            o = make_float4(a.x + o.x, a.y + o.y, a.z + o.z, a.w + o.w);
        }
        reinterpret_cast<float4*>(pos)[i] = o;
        if (pos16) store_bf16x4(pos16 + i * 4, o.x, o.y, o.z, o.w);
    }
}

// The same values with the row arithmetic hoisted (the grid-stride form above divides 64-bit indices per float4):
// block = rpi rows x c4n float4 lanes (c4n = C/4 divides 256), kPosRows consecutive flattened rows per block,
// (video, row) advanced incrementally.  With C = 512, F = 256 a wave is all-sine or all-duration lanes.
constexpr int kPosRows = 64;
__global__ __launch_bounds__(256) void level_pos_rows_kernel(const float* __restrict__ xe,
                                                             const float* __restrict__ dim_t,
                                                             const float* __restrict__ dur,
                                                             const float* __restrict__ lemb, PosLevels lv, int N,
                                                             int S, int F, int Dd, const float* __restrict__ add,
                                                             float* __restrict__ pos, uint16_t* __restrict__ pos16) {
    const int C = F + Dd, c4n = C / 4, rpi = 256 / c4n;
    const int cg = threadIdx.x % c4n, rr = threadIdx.x / c4n;
    const int c = cg * 4;
    const long rows = (long)N * S;
    long r = (long)blockIdx.x * kPosRows + rr;
    const long rend = min(rows, (long)(blockIdx.x + 1) * kPosRows);
    if (r >= rend) return;
    int n = (int)(r / S), s = (int)(r - (long)n * S);
    float dt[4] = {1.f, 1.f, 1.f, 1.f};
    if (c < F) {
#pragma unroll
        for (int k = 0; k < 4; ++k) dt[k] = dim_t[c + k];
    }
    for (; r < rend; r += rpi) {
        const int l = pos_level(lv, s);
        const float4 le = *reinterpret_cast<const float4*>(lemb + (size_t)l * C + c);
        float v[4];
        if (c < F) {
            const float x = xe[r];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float a = x / dt[k];
                v[k] = ((c + k) & 1) ? cosf(a) : sinf(a);
            }
        } else {
            const float4 d = *reinterpret_cast<const float4*>(dur + (size_t)n * Dd + (c - F));
            v[0] = d.x;
            v[1] = d.y;
            v[2] = d.z;
            v[3] = d.w;
        }
        float4 o = make_float4(v[0] + le.x, v[1] + le.y, v[2] + le.z, v[3] + le.w);
        const size_t i = (size_t)r * c4n + cg;
        if (add) {
            const float4 a = reinterpret_cast<const float4*>(add)[i];
            o = make_float4(a.x + o.x, a.y + o.y, a.z + o.z, a.w + o.w);
        }
        reinterpret_cast<float4*>(pos)[i] = o;
        if (pos16) store_bf16x4(pos16 + i * 4, o.x, o.y, o.z, o.w);
        s += rpi;
        while (s >= S) {
            s -= S;
            ++n;
        }
    }
}

// grid (C / 64, levels, N): 16 float4 column groups x 16 row lanes over the level's rows of one video
__global__ __launch_bounds__(256) void level_pos_bwd_kernel(const float* __restrict__ dpos, PosLevels lv, int S,
                                                            int C, float* __restrict__ part) {
    __shared__ float4 red[16][16];
    const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int c4 = blockIdx.x * 16 + cg, l = blockIdx.y, n = blockIdx.z;
    const int cs = C / 4;
    const int r0 = lv.start[l], r1 = lv.start[l + 1];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < cs) {
        const float4* src = reinterpret_cast<const float4*>(dpos) + (size_t)n * S * cs + c4;
#pragma unroll 4
        for (int r = r0 + rl; r < r1; r += 16) {
            const float4 v = src[(size_t)r * cs];
            a.x += v.x;
            a.y += v.y;
            a.z += v.z;
            a.w += v.w;
        }
    }
    red[rl][cg] = a;
    __syncthreads();
    if (rl == 0 && c4 < cs) {
        float4 t = red[0][cg];
#pragma unroll
        for (int k = 1; k < 16; ++k) {
            t.x += red[k][cg].x;
            t.y += red[k][cg].y;
            t.z += red[k][cg].z;
            t.w += red[k][cg].w;
        }
        reinterpret_cast<float4*>(part + ((size_t)n * lv.n + l) * C)[c4] = t;
    }
}

static int fill_pos_levels(const int32_t* level_T, int L, int S, PosLevels& lv) {
    PDVC_CHECK_ARG(level_T != nullptr && L >= 1 && L <= kPosMaxLevels, "1..%d levels required", kPosMaxLevels);
    lv.n = L;
    int acc = 0;
    for (int l = 0; l < L; ++l) {
        PDVC_CHECK_ARG(level_T[l] > 0, "level %d has non-positive length", l);
        lv.start[l] = acc;
        acc += level_T[l];
    }
    for (int l = L; l <= kPosMaxLevels; ++l) lv.start[l] = acc;
    PDVC_CHECK_ARG(acc == S, "level lengths sum to %d, expected S = %d", acc, S);
    return PDVC_OK;
}

}  // namespace pdvc

using namespace pdvc;

extern "C" int pdvc_level_pos_rows_add_f32_bf16out(const float* xe, const float* dim_t, const float* dur,
                                                   const float* level_embed, const int32_t* level_T, int num_levels,
                                                   int N, int S, int F, int Dd, const float* add, float* out,
                                                   uint16_t* out16, void* stream) {
    float* pos = out;
    PDVC_CHECK_ARG(((uintptr_t)out16 % 8) == 0, "out16 must be 8-byte aligned");
    PDVC_CHECK_ARG(N >= 0 && S > 0 && F > 0 && Dd >= 0 && F % 4 == 0 && Dd % 4 == 0, "invalid sizes");
    PDVC_CHECK_ARG(((uintptr_t)add % 16) == 0, "add must be 16-byte aligned");
    PDVC_CHECK_ARG(((uintptr_t)pos % 16) == 0 && ((uintptr_t)level_embed % 16) == 0 &&
                       (Dd == 0 || ((uintptr_t)dur % 16) == 0),
                   "pos, level_embed and dur must be 16-byte aligned");
    PosLevels lv;
    int rc = fill_pos_levels(level_T, num_levels, S, lv);
    if (rc) return rc;
    const long total = (long)N * S * ((F + Dd) / 4);
    if (total == 0) return PDVC_OK;
    const int c4n = (F + Dd) / 4;
    if (c4n <= 256 && 256 % c4n == 0) {
        const long blocks = ((long)N * S + kPosRows - 1) / kPosRows;
        hipLaunchKernelGGL(level_pos_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, xe, dim_t,
                           dur, level_embed, lv, N, S, F, Dd, add, pos, out16);
        PDVC_CHECK_LAUNCH("level_pos_rows_kernel");
        return PDVC_OK;
    }
    const long want = (total + 255) / 256;
    const unsigned blocks = (unsigned)(want < 16384 ? want : 16384);
    hipLaunchKernelGGL(level_pos_fwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, xe, dim_t, dur,
                       level_embed, lv, N, S, F, Dd, add, pos, out16);
    PDVC_CHECK_LAUNCH("level_pos_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_level_pos_rows_add_f32(const float* xe, const float* dim_t, const float* dur,
                                           const float* level_embed, const int32_t* level_T, int num_levels, int N,
                                           int S, int F, int Dd, const float* add, float* out, void* stream) {
    return pdvc_level_pos_rows_add_f32_bf16out(xe, dim_t, dur, level_embed, level_T, num_levels, N, S, F, Dd, add, out,
                                               nullptr, stream);
}

extern "C" int pdvc_level_pos_rows_forward_f32(const float* xe, const float* dim_t, const float* dur,
                                               const float* level_embed, const int32_t* level_T, int num_levels,
                                               int N, int S, int F, int Dd, float* pos, void* stream) {
    return pdvc_level_pos_rows_add_f32(xe, dim_t, dur, level_embed, level_T, num_levels, N, S, F, Dd, nullptr, pos,
                                       stream);
}

extern "C" int pdvc_level_pos_rows_backward_f32(const float* dpos, const int32_t* level_T, int num_levels, int N,
                                                int S, int C, float* partials, void* stream) {
    PDVC_CHECK_ARG(N >= 0 && S > 0 && C > 0 && C % 4 == 0, "invalid sizes");
    PDVC_CHECK_ARG(((uintptr_t)dpos % 16) == 0 && ((uintptr_t)partials % 16) == 0, "16-byte alignment required");
    PosLevels lv;
    int rc = fill_pos_levels(level_T, num_levels, S, lv);
    if (rc) return rc;
    if (N == 0) return PDVC_OK;
    hipLaunchKernelGGL(level_pos_bwd_kernel, dim3((unsigned)((C / 4 + 15) / 16), (unsigned)num_levels, (unsigned)N),
                       dim3(256), 0, (hipStream_t)stream, dpos, lv, S, C, partials);
    PDVC_CHECK_LAUNCH("level_pos_bwd_kernel");
    return PDVC_OK;
}
