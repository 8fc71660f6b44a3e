// seqattn.hip -- long-sequence multi-head attention core for the dual-modality front-end of cfgs/yc2_newModel_sound
// (reference: NewModel.visual_self_attention / visual_sound_attention, NewModel.py:41-65: nn.MultiheadAttention(768,
// 32 heads, batch_first) over the T clip features, queries = clips or sound features).  T = 512 queries and keys,
// head_dim 24: outside the decoder kernel's range (mha.hip: Q <= 300), and a (T x T) score matrix per head is
// 1 MB, so nothing of size T^2 is ever written (flash-style: running max / sum, P recomputed in the backward).
//
//   forward:  out_i = sum_j softmax_j(scale q_i.k_j) v_j, lse_i saved
//   backward: delta_i = dout_i.out_i;  p_ij = exp(scale q_i.k_j - lse_i);  ds_ij = p_ij (dout_i.v_j - delta_i)
//             dq_i = scale sum_j ds_ij k_j  (query-owner kernel);  dk_j = scale sum_i ds_ij q_i,
//             dv_j = sum_i p_ij dout_i (key-owner kernel) -- every gradient row has exactly one writer, no atomics.
//
// Every product runs on v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulation).  A wave owns 32 rows of
// its side (queries, or keys in the dk/dv kernel) and walks the other side in 32-row sub-blocks staged through
// LDS, 64 rows per tile, double-buffered (the next tile's global loads are issued before the current tile's
// MFMAs).  MFMA operand layout of one k-step: lane l supplies A[l%32][slot l/32] and B[slot l/32][l%32], the
// accumulator register r of lane l holds C[crow(r, l/32)][l%32].  Two choices make the whole step run out of
// registers with no LDS round trip of the probabilities:
//   * scores are computed TRANSPOSED, C = K . Q^T (forward, dq) or Q . K^T (dk/dv), so the owned side indexes the
//     lanes and the other side the accumulator registers.  The row statistics of the owned side (running max,
//     lse, delta) are then one value per lane, and the softmax reduction runs over a lane's own 16 registers plus
//     one exchange between the two 32-lane halves;
//   * the reduction index of the second product is the other side, which the score tile holds in its registers:
//     register r of P^T is directly the B operand of k-step r when the logical reduction slot (r, l/32) is mapped
//     to the physical row crow(r, l/32) -- the matching A operand is that LDS row, read column-wise.
// The head-dim reduction of the score products maps slot (kk, l/32) to channel (l/32) * D/2 + kk, so each lane
// reads a contiguous D/2-channel chunk of its row (ds_read_b128).  Outputs with head_dim below a multiple of 32
// (24 -> 32) carry zero channel rows: the LDS tiles keep columns D..32*NT zero.
// Scores are kept in log2 units (q pre-multiplied by scale * log2(e)): exp2 is the hardware v_exp_f32.
// No dropout and no key padding: the front-end uses neither (nn.MultiheadAttention defaults, all clips valid).
#include <math.h>

#include "pdvc_common.h"
#include "seqattn.h"

namespace pdvc {

typedef float sq_f32x16 __attribute__((ext_vector_type(16)));

constexpr int kSqWaves = 8;            // waves per workgroup, each owning 32 rows
constexpr int kSqThreads = 64 * kSqWaves;
constexpr int kSqOwn = 32 * kSqWaves;  // owned rows per workgroup
constexpr int kSqKT = 64;              // rows of the streamed side per LDS tile
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ sq_f32x16 sq_mfma(float a, float b, sq_f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int sq_crow(int r, int hi) { return (r & 3) + 8 * (r >> 2) + 4 * hi; }
__device__ __forceinline__ float sq_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float sq_swap32(float x) { return __shfl_xor(x, 32, PDVC_WAVE); }

template <int D>
struct SqCfg {
    static constexpr int DH = D / 2;               // score k-steps over the head dim
    static constexpr int NT = (D + 31) / 32;       // 32-channel output tiles
    // LDS row stride D + 4 (= 4 x odd): the 16 rows of a ds_read_b128 lane group land on distinct bank quads.
    // Column walks (A operands of the second products) read lanes l%32 = 0..31 of a row; lanes past D read
    // the next row's first channels -- garbage that only reaches output channel rows >= D, never written.
    static constexpr int LD = D + 4;
    static constexpr int TILE = kSqKT * LD;        // floats per staged matrix tile
    static constexpr int SMEM = 4 * TILE + 64;     // [buf][2 matrices] + slack for the last row's column walk
    static constexpr int EPT = kSqKT * D / kSqThreads;  // staged elements per thread per matrix
    // accumulator registers holding real channels of output tile t (channel rows >= D are padding)
    static constexpr int valid(int t) { return (D - 32 * t) >= 32 ? 16 : (D - 32 * t) / 2; }
    // forward: a spare output channel row D (head_dim not a multiple of 32) carries the softmax denominator,
    // V's column D being held at 1 (accumulator register 12 of the lanes l/32 = 0 for D = 24)
    static constexpr bool ONES = (D % 32) != 0;
    static_assert(D % 8 == 0 && D <= 64, "head_dim must be a multiple of 8, at most 64");
    static_assert((kSqKT * D) % kSqThreads == 0, "tile elements must split evenly over the threads");
};

// Row chunk [hi*D/2, hi*D/2 + D/2) of LDS row `row` -> registers (ds_read_b128)
template <int D>
__device__ __forceinline__ void sq_chunk(const float* tile, int row, int hi, float (&x)[D / 2]) {
    const float4* p = reinterpret_cast<const float4*>(tile + row * SqCfg<D>::LD + hi * (D / 2));
#pragma unroll
    for (int i = 0; i < D / 8; ++i) {
        const float4 f = p[i];
        x[4 * i] = f.x;
        x[4 * i + 1] = f.y;
        x[4 * i + 2] = f.z;
        x[4 * i + 3] = f.w;
    }
}

// Global -> register -> LDS staging of kSqKT-row tiles of two (rows, D) head slices; rows past `nrows` are zero.
template <int D>
struct SqStager {
    static constexpr int EPT = SqCfg<D>::EPT;
    int goff[EPT], soff[EPT];
    float a[EPT], b[EPT];
    __device__ __forceinline__ SqStager(int tid) {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
            const int e = tid + kSqThreads * i, r = e / D, c = e - r * D;
            goff[i] = (r << 8) | c;  // row (< 256) and column, unpacked per tile
            soff[i] = r * SqCfg<D>::LD + c;
        }
    }
    __device__ __forceinline__ void load(const float* __restrict__ A, long lda, const float* __restrict__ B, long ldb,
                                         int r0, int nrows) {
        const float* Ar = A + (long)r0 * lda;
        const float* Br = B + (long)r0 * ldb;
        if (r0 + kSqKT <= nrows) {  // full tile: no row predicate
#pragma unroll
            for (int i = 0; i < EPT; ++i) {
                const int r = goff[i] >> 8, c = goff[i] & 255;
                a[i] = Ar[r * lda + c];
                b[i] = Br[r * ldb + c];
            }
        } else {
#pragma unroll
            for (int i = 0; i < EPT; ++i) {
                const int r = goff[i] >> 8, c = goff[i] & 255;
                const bool ok = r0 + r < nrows;
                a[i] = ok ? Ar[r * lda + c] : 0.f;
                b[i] = ok ? Br[r * ldb + c] : 0.f;
            }
        }
    }
    __device__ __forceinline__ void store(float* ta, float* tb) const {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
            ta[soff[i]] = a[i];
            tb[soff[i]] = b[i];
        }
    }
};

// Workgroup -> (video*head, owned block): consecutive owned blocks of one head on one XCD (shared K/V in its L2)
__device__ __forceinline__ void sq_block(int nblocks_own, int& nh, int& ob) {
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    nh = lb / nblocks_own;
    ob = lb - nh * nblocks_own;
}

// Options of the decoder self-attention route (mha.hip, Q > 128): a key padding mask and dropout on the
// probabilities with mha.hip's counter-hash mask, keep_elem(seed, video*head, query, key, Q), so every route of
// pdvc_mha_* drops the same elements.  The front-end instantiates neither.
struct SqOpts {
    const uint8_t* kpm;  // (N, Tk) nonzero = padded key (KPM)
    uint64_t seed0;
    const uint64_t* seed_dev;
    uint32_t thresh;     // drop_threshold(p) (DROP)
    float keep_scale;    // 1 / (1 - p)
};

// per-tile additive key bias (0, or -inf at padded keys and keys >= Tk), staged with the K / V tile (KPM)
struct SqKeyBias {
    float b = 0.f;
    __device__ __forceinline__ void load(const uint8_t* kpm_row, int r0, int nrows, int tid) {
        if (tid < kSqKT) {
            const int j = r0 + tid;
            b = (j < nrows && !kpm_row[j]) ? 0.f : -INFINITY;
        }
    }
    __device__ __forceinline__ void store(float* dst, int tid) const {
        if (tid < kSqKT) dst[tid] = b;
    }
};

// bias of the 16 keys a lane's score registers hold in 32-key block sb of a tile: rows sb*32 + crow(r, hi)
__device__ __forceinline__ void sq_add_bias(sq_f32x16& s, const float* bias, int sb, int hi) {
    const float4* B4 = reinterpret_cast<const float4*>(bias + sb * 32 + 4 * hi);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 b = B4[2 * g];
        s[4 * g] += b.x;
        s[4 * g + 1] += b.y;
        s[4 * g + 2] += b.z;
        s[4 * g + 3] += b.w;
    }
}

// ---------------------------------------------------------------------------------------------------------------
// forward: wave = 32 queries; per 64-key tile S^T = K . Q^T (two independent 32-key MFMA chains), one online
// softmax update over the key registers, O^T += V^T . P^T.  Measured alternatives (tools/seqattn_bench.py, T=512,
// 32 heads of 24, 64 videos; this kernel 0.62 ms = 83 TFLOP/s): two 32-query blocks per wave sharing the K / V
// operand reads 75-85; a one-tile software pipeline (next tile's score MFMAs before this tile's softmax, two named
// score states, 240 VGPRs) 69; 128-key tiles 65; s_setprio around the MFMA runs, sched_group_barrier
// interleaves and skipping the identity rescale when no row max moved: within noise.  The workgroup is 8 waves
// (256 queries, 2 per (video, head) at T = 512) held to 4 waves per SIMD (<= 128 VGPRs).
// DROP: the denominator sums the undropped p (so no ones-column trick), P.V takes the dropped, rescaled p.
template <int D, bool DROP, bool KPM>
__global__ __launch_bounds__(kSqThreads) __attribute__((amdgpu_waves_per_eu(4))) void seqattn_fwd_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, int H, int Tq, int Tk,
    long ldq, long ldk, long ldv, float qmul, int qblocks, SqOpts opt, float* __restrict__ out,
    float* __restrict__ lse) {
    using C = SqCfg<D>;
    constexpr bool ONES = C::ONES && !DROP;
    constexpr int SB = kSqKT / 32;          // 32-key score blocks per tile
    constexpr int TL = C::NT - 1;           // output tile holding channel row D (ONES)
    constexpr int RL = (D - 32 * TL) / 2;   // its accumulator register in the lanes l/32 = 0
    __shared__ __attribute__((aligned(16))) float smem[C::SMEM];  // [buf][K, V]
    __shared__ __attribute__((aligned(16))) float kbias[KPM ? 2 : 1][KPM ? kSqKT : 4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hi = lane >> 5;
    int nh, qb;
    sq_block(qblocks, nh, qb);
    const int n = nh / H, h = nh - n * H;
    const int qi = qb * kSqOwn + w * 32 + l32;
    const bool qok = qi < Tq;
    const uint64_t seed = DROP ? load_seed(opt.seed0, opt.seed_dev) : 0;
    float qr[C::DH];
    {
        const float* qp = q + ((long)n * Tq + (qok ? qi : 0)) * ldq + h * D + hi * C::DH;
#pragma unroll
        for (int kk = 0; kk < C::DH; ++kk) qr[kk] = qok ? qp[kk] * qmul : 0.f;
    }
    const float* kh = k + (long)n * Tk * ldk + h * D;
    const float* vh = v + (long)n * Tk * ldv + h * D;
    const uint8_t* kpm_row = KPM ? opt.kpm + (long)n * Tk : nullptr;
    if (ONES)
        for (int r = tid; r < 2 * kSqKT; r += kSqThreads)
            smem[(r / kSqKT) * 2 * C::TILE + C::TILE + (r % kSqKT) * C::LD + D] = 1.f;
    SqStager<D> st(tid);
    SqKeyBias kb;
    st.load(kh, ldk, vh, ldv, 0, Tk);
    if (KPM) kb.load(kpm_row, 0, Tk, tid);
    st.store(smem, smem + C::TILE);
    if (KPM) kb.store(kbias[0], tid);
    __syncthreads();
    sq_f32x16 o[C::NT];
#pragma unroll
    for (int t = 0; t < C::NT; ++t) o[t] = sq_f32x16{};
    float m = -INFINITY, l = 0.f;
    const int ntiles = (Tk + kSqKT - 1) / kSqKT;
    for (int it = 0; it < ntiles; ++it) {
        const int t0 = it * kSqKT, buf = it & 1;
        const float* Ks = smem + buf * 2 * C::TILE;
        const float* Vs = Ks + C::TILE;
        if (it + 1 < ntiles) {
            st.load(kh, ldk, vh, ldv, t0 + kSqKT, Tk);
            if (KPM) kb.load(kpm_row, t0 + kSqKT, Tk, tid);
        }
        // the tile's 32-key score blocks (independent MFMA chains), one softmax update over the whole tile
        sq_f32x16 s[SB];
        {
            float kc[SB][C::DH];
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) sq_chunk<D>(Ks, sb * 32 + l32, hi, kc[sb]);
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) s[sb] = sq_mfma(kc[sb][0], qr[0], sq_f32x16{});
#pragma unroll
            for (int kk = 1; kk < C::DH; ++kk)
#pragma unroll
                for (int sb = 0; sb < SB; ++sb) s[sb] = sq_mfma(kc[sb][kk], qr[kk], s[sb]);
        }
        if (KPM) {
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) sq_add_bias(s[sb], kbias[buf], sb, hi);
        } else if (t0 + kSqKT > Tk) {
#pragma unroll
            for (int sb = 0; sb < SB; ++sb)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (t0 + sb * 32 + sq_crow(r, hi) >= Tk) s[sb][r] = -INFINITY;
        }
        float mx = s[0][0];
#pragma unroll
        for (int sb = 0; sb < SB; ++sb)
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[sb][r]);
        mx = fmaxf(mx, sq_swap32(mx));
        const float mn = fmaxf(m, mx);  // finite: the tile holds at least one valid key
        const float corr = sq_exp2(m - mn);
        m = mn;
#pragma unroll
        for (int sb = 0; sb < SB; ++sb)
#pragma unroll
            for (int r = 0; r < 16; ++r) s[sb][r] = sq_exp2(s[sb][r] - mn);
        if (!ONES) {
            l *= corr;
#pragma unroll
            for (int sb = 0; sb < SB; ++sb)
#pragma unroll
                for (int r = 0; r < 16; ++r) l += s[sb][r];
        }
        if (DROP) {
#pragma unroll
            for (int sb = 0; sb < SB; ++sb)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const uint32_t key = (uint32_t)(t0 + sb * 32 + sq_crow(r, hi));
                    s[sb][r] = keep_elem(seed, (uint32_t)nh, (uint32_t)qi, key, (uint32_t)Tq, opt.thresh)
                                   ? s[sb][r] * opt.keep_scale : 0.f;
                }
        }
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
            for (int r = 0; r < C::valid(t) + (ONES && t == TL ? 1 : 0); ++r) o[t][r] *= corr;
#pragma unroll
        for (int sb = 0; sb < SB; ++sb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float* vc = Vs + (sb * 32 + sq_crow(r, hi)) * C::LD + l32;
#pragma unroll
                for (int t = 0; t < C::NT; ++t) o[t] = sq_mfma(vc[32 * t], s[sb][r], o[t]);
            }
        if (it + 1 < ntiles) {
            st.store(smem + (buf ^ 1) * 2 * C::TILE, smem + (buf ^ 1) * 2 * C::TILE + C::TILE);
            if (KPM) kb.store(kbias[buf ^ 1], tid);
        }
        __syncthreads();
    }
    if (ONES) {  // channel row D = sum_j p_j, held by the lanes l/32 = 0
        const float own = o[TL][RL], other = sq_swap32(own);
        l = hi ? other : own;
    } else {
        l += sq_swap32(l);
    }
    if (qok) {
        const float inv = 1.f / l;
        float* orow = out + ((long)n * Tq + qi) * (long)(H * D) + h * D;
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
            for (int g = 0; g < C::valid(t) / 4; ++g)
                *reinterpret_cast<float4*>(orow + 32 * t + 8 * g + 4 * hi) =
                    make_float4(o[t][4 * g] * inv, o[t][4 * g + 1] * inv, o[t][4 * g + 2] * inv, o[t][4 * g + 3] * inv);
        if (hi == 0) lse[(long)nh * Tq + qi] = (m + log2f(l)) * kLn2;
    }
}

// ---------------------------------------------------------------------------------------------------------------
// backward, query owner: S^T = K . Q^T, dP^T = V . dO^T, dS^T = P^T (dP^T - delta), dQ^T += K^T . dS^T.
// Publishes delta_i = dout_i . out_i for the key-owner kernel.  DROP: dP = dP_d * keep / (1 - p) (delta is
// unchanged: sum_j p_ij dP_ij = dout_i . out_i with out the dropped product).
template <int D, bool DROP, bool KPM>
__global__ __launch_bounds__(kSqThreads) void seqattn_bwd_dq_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ out,
    float* __restrict__ delta, int H, int Tq, int Tk, long ldq, long ldk, long ldv, float qmul, float scale,
    int qblocks, SqOpts opt, float* __restrict__ dq, long lddq) {
    using C = SqCfg<D>;
    __shared__ __attribute__((aligned(16))) float smem[C::SMEM];  // [buf][K, V]
    __shared__ __attribute__((aligned(16))) float kbias[KPM ? 2 : 1][KPM ? kSqKT : 4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hi = lane >> 5;
    int nh, qb;
    sq_block(qblocks, nh, qb);
    const int n = nh / H, h = nh - n * H;
    const int E = H * D;
    const int qi = qb * kSqOwn + w * 32 + l32;
    const bool qok = qi < Tq;
    const uint64_t seed = DROP ? load_seed(opt.seed0, opt.seed_dev) : 0;
    float qr[C::DH], gr[C::DH];
    float dl = 0.f, l2 = 0.f;
    {
        const long qrow = (long)n * Tq + (qok ? qi : 0);
        const float* qp = q + qrow * ldq + h * D + hi * C::DH;
        const float* gp = dout + qrow * E + h * D + hi * C::DH;
        const float* op = out + qrow * E + h * D + hi * C::DH;
#pragma unroll
        for (int kk = 0; kk < C::DH; ++kk) {
            qr[kk] = qok ? qp[kk] * qmul : 0.f;
            gr[kk] = qok ? gp[kk] : 0.f;
            dl += qok ? gr[kk] * op[kk] : 0.f;
        }
        dl += sq_swap32(dl);
        if (qok) {
            l2 = lse[(long)nh * Tq + qi] * kLog2e;
            if (hi == 0) delta[(long)nh * Tq + qi] = dl;
        }
    }
    const float* kh = k + (long)n * Tk * ldk + h * D;
    const float* vh = v + (long)n * Tk * ldv + h * D;
    const uint8_t* kpm_row = KPM ? opt.kpm + (long)n * Tk : nullptr;
    SqStager<D> st(tid);
    SqKeyBias kb;
    st.load(kh, ldk, vh, ldv, 0, Tk);
    if (KPM) kb.load(kpm_row, 0, Tk, tid);
    st.store(smem, smem + C::TILE);
    if (KPM) kb.store(kbias[0], tid);
    __syncthreads();
    sq_f32x16 acc[C::NT];
#pragma unroll
    for (int t = 0; t < C::NT; ++t) acc[t] = sq_f32x16{};
    const int ntiles = (Tk + kSqKT - 1) / kSqKT;
    for (int it = 0; it < ntiles; ++it) {
        const int t0 = it * kSqKT, buf = it & 1;
        const float* Ks = smem + buf * 2 * C::TILE;
        const float* Vs = Ks + C::TILE;
        if (it + 1 < ntiles) {
            st.load(kh, ldk, vh, ldv, t0 + kSqKT, Tk);
            if (KPM) kb.load(kpm_row, t0 + kSqKT, Tk, tid);
        }
#pragma unroll
        for (int sb = 0; sb < kSqKT / 32; ++sb) {
            if (t0 + sb * 32 >= Tk) break;  // keys past Tk inside a sub-block are zero rows: ds * 0 adds nothing
            float kc[C::DH], vc[C::DH];
            sq_chunk<D>(Ks, sb * 32 + l32, hi, kc);
            sq_chunk<D>(Vs, sb * 32 + l32, hi, vc);
            sq_f32x16 s = sq_f32x16{}, dp = sq_f32x16{};
#pragma unroll
            for (int kk = 0; kk < C::DH; ++kk) {
                s = sq_mfma(kc[kk], qr[kk], s);
                dp = sq_mfma(vc[kk], gr[kk], dp);
            }
            if (KPM) sq_add_bias(s, kbias[buf], sb, hi);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float d = dp[r];
                if (DROP) {
                    const uint32_t key = (uint32_t)(t0 + sb * 32 + sq_crow(r, hi));
                    d = keep_elem(seed, (uint32_t)nh, (uint32_t)qi, key, (uint32_t)Tq, opt.thresh) ? d * opt.keep_scale
                                                                                                 : 0.f;
                }
                s[r] = sq_exp2(s[r] - l2) * (d - dl);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float* kcol = Ks + (sb * 32 + sq_crow(r, hi)) * C::LD + l32;
#pragma unroll
                for (int t = 0; t < C::NT; ++t) acc[t] = sq_mfma(kcol[32 * t], s[r], acc[t]);
            }
        }
        if (it + 1 < ntiles) {
            st.store(smem + (buf ^ 1) * 2 * C::TILE, smem + (buf ^ 1) * 2 * C::TILE + C::TILE);
            if (KPM) kb.store(kbias[buf ^ 1], tid);
        }
        __syncthreads();
    }
    if (qok) {
        float* row = dq + ((long)n * Tq + qi) * lddq + h * D;
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
            for (int r = 0; r < C::valid(t); ++r) row[32 * t + sq_crow(r, hi)] = acc[t][r] * scale;
    }
}

// ---------------------------------------------------------------------------------------------------------------
// backward, key owner: S = Q . K^T, dP = dO . V^T (key index on the lanes), dV^T += dO^T . P_d, dK^T += Q^T . dS.
template <int D, bool DROP, bool KPM>
__global__ __launch_bounds__(kSqThreads) void seqattn_bwd_dkv_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta, int H, int Tq,
    int Tk, long ldq, long ldk, long ldv, float kmul, float scale, int kblocks, SqOpts opt, float* __restrict__ dk,
    long lddk, float* __restrict__ dv, long lddv) {
    using C = SqCfg<D>;
    __shared__ __attribute__((aligned(16))) float smem[C::SMEM];  // [buf][Q, dO]
    __shared__ __attribute__((aligned(16))) float rowst[2][2][kSqKT];   // [buf][lse2, delta]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l32 = lane & 31, hi = lane >> 5;
    int nh, kb;
    sq_block(kblocks, nh, kb);
    const int n = nh / H, h = nh - n * H;
    const int E = H * D;
    const int kj = kb * kSqOwn + w * 32 + l32;
    const bool kok = kj < Tk;
    const uint64_t seed = DROP ? load_seed(opt.seed0, opt.seed_dev) : 0;
    // this lane's key: padded -> every p of it is 0
    const float kbias = (KPM && kok && opt.kpm[(long)n * Tk + kj]) ? -INFINITY : 0.f;
    float kr[C::DH], vr[C::DH];
    {
        const long krow = (long)n * Tk + (kok ? kj : 0);
        const float* kp = k + krow * ldk + h * D + hi * C::DH;
        const float* vp = v + krow * ldv + h * D + hi * C::DH;
#pragma unroll
        for (int kk = 0; kk < C::DH; ++kk) {
            kr[kk] = kok ? kp[kk] * kmul : 0.f;
            vr[kk] = kok ? vp[kk] : 0.f;
        }
    }
    const float* qh = q + (long)n * Tq * ldq + h * D;
    const float* gh = dout + (long)n * Tq * E + h * D;
    const float* lh = lse + (long)nh * Tq;
    const float* dh = delta + (long)nh * Tq;
    SqStager<D> st(tid);
    float rl = 0.f, rd = 0.f;  // this thread's row statistic (threads < 64)
    auto load_rows = [&](int r0) {
        if (tid < kSqKT) {
            const int i = r0 + tid;
            rl = i < Tq ? lh[i] * kLog2e : INFINITY;  // padded queries: p = exp2(s - inf) = 0
            rd = i < Tq ? dh[i] : 0.f;
        }
    };
    auto store_rows = [&](int buf) {
        if (tid < kSqKT) {
            rowst[buf][0][tid] = rl;
            rowst[buf][1][tid] = rd;
        }
    };
    st.load(qh, ldq, gh, E, 0, Tq);
    load_rows(0);
    st.store(smem, smem + C::TILE);
    store_rows(0);
    __syncthreads();
    sq_f32x16 ak[C::NT], av[C::NT];
#pragma unroll
    for (int t = 0; t < C::NT; ++t) ak[t] = av[t] = sq_f32x16{};
    const int ntiles = (Tq + kSqKT - 1) / kSqKT;
    for (int it = 0; it < ntiles; ++it) {
        const int t0 = it * kSqKT, buf = it & 1;
        const float* Qs = smem + buf * 2 * C::TILE;
        const float* Gs = Qs + C::TILE;
        if (it + 1 < ntiles) {
            st.load(qh, ldq, gh, E, t0 + kSqKT, Tq);
            load_rows(t0 + kSqKT);
        }
#pragma unroll
        for (int sb = 0; sb < kSqKT / 32; ++sb) {
            if (t0 + sb * 32 >= Tq) break;
            float qc[C::DH], gc[C::DH];
            sq_chunk<D>(Qs, sb * 32 + l32, hi, qc);
            sq_chunk<D>(Gs, sb * 32 + l32, hi, gc);
            sq_f32x16 s = sq_f32x16{}, dp = sq_f32x16{};
#pragma unroll
            for (int kk = 0; kk < C::DH; ++kk) {
                s = sq_mfma(qc[kk], kr[kk], s);
                dp = sq_mfma(gc[kk], vr[kk], dp);
            }
            // query rows of the registers: sb*32 + crow(r, hi) -> 4 float4 reads of each statistic
            const float4* L4 = reinterpret_cast<const float4*>(&rowst[buf][0][sb * 32 + 4 * hi]);
            const float4* D4 = reinterpret_cast<const float4*>(&rowst[buf][1][sb * 32 + 4 * hi]);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 lv = L4[2 * g], dv4 = D4[2 * g];
                const float lr[4] = {lv.x, lv.y, lv.z, lv.w}, dr[4] = {dv4.x, dv4.y, dv4.z, dv4.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int r = 4 * g + j;
                    const float p = sq_exp2(s[r] - lr[j] + kbias);
                    float d = dp[r], pd = p;
                    if (DROP) {
                        const uint32_t qq = (uint32_t)(t0 + sb * 32 + sq_crow(r, hi));
                        const bool keep = keep_elem(seed, (uint32_t)nh, qq, (uint32_t)kj, (uint32_t)Tq, opt.thresh);
                        d = keep ? d * opt.keep_scale : 0.f;
                        pd = keep ? p * opt.keep_scale : 0.f;
                    }
                    s[r] = pd;
                    dp[r] = p * (d - dr[j]);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (sb * 32 + sq_crow(r, hi)) * C::LD + l32;
#pragma unroll
                for (int t = 0; t < C::NT; ++t) {
                    av[t] = sq_mfma(Gs[row + 32 * t], s[r], av[t]);
                    ak[t] = sq_mfma(Qs[row + 32 * t], dp[r], ak[t]);
                }
            }
        }
        if (it + 1 < ntiles) {
            st.store(smem + (buf ^ 1) * 2 * C::TILE, smem + (buf ^ 1) * 2 * C::TILE + C::TILE);
            store_rows(buf ^ 1);
        }
        __syncthreads();
    }
    if (kok) {
        float* rk = dk + ((long)n * Tk + kj) * lddk + h * D;
        float* rv = dv + ((long)n * Tk + kj) * lddv + h * D;
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
            for (int r = 0; r < C::valid(t); ++r) {
                rk[32 * t + sq_crow(r, hi)] = ak[t][r] * scale;
                rv[32 * t + sq_crow(r, hi)] = av[t][r];
            }
    }
}

#define PDVC_SQ_DISPATCH(D_, CALL) \
    switch (D_) {                  \
        case 16: CALL(16); break;  \
        case 24: CALL(24); break;  \
        case 32: CALL(32); break;  \
        case 48: CALL(48); break;  \
        case 64: CALL(64); break;  \
        default: break;            \
    }

bool sq_head_dim_ok(int D) { return D == 16 || D == 24 || D == 32 || D == 48 || D == 64; }

template <bool DROP, bool KPM>
static void sq_launch_fwd(dim3 grid, hipStream_t s, const float* q, long ldq, const float* k, long ldk,
                          const float* v, long ldv, int batch, int num_query, int num_key, int num_heads,
                          int head_dim, float qmul, int qblocks, const SqOpts& o, float* out, float* lse) {
#define PDVC_SQ_FWD(DD)                                                                                          \
    hipLaunchKernelGGL((seqattn_fwd_kernel<DD, DROP, KPM>), grid, dim3(kSqThreads), 0, s, q, k, v, num_heads,    \
                       num_query, num_key, ldq, ldk, ldv, qmul, qblocks, o, out, lse)
    PDVC_SQ_DISPATCH(head_dim, PDVC_SQ_FWD)
#undef PDVC_SQ_FWD
}

template <bool DROP, bool KPM>
static void sq_launch_bwd(dim3 gq, dim3 gk, hipStream_t s, const float* q, long ldq, const float* k, long ldk,
                          const float* v, long ldv, const float* out, const float* grad_out, const float* lse,
                          int num_query, int num_key, int num_heads, int head_dim, float qmul, float scale,
                          int qblocks, int kblocks, const SqOpts& o, float* delta, float* grad_q, long ld_grad_q,
                          float* grad_k, long ld_grad_k, float* grad_v, long ld_grad_v) {
#define PDVC_SQ_DQ(DD)                                                                                               \
    hipLaunchKernelGGL((seqattn_bwd_dq_kernel<DD, DROP, KPM>), gq, dim3(kSqThreads), 0, s, q, k, v, grad_out, lse,  \
                       out, delta, num_heads, num_query, num_key, ldq, ldk, ldv, qmul, scale, qblocks, o, grad_q,    \
                       ld_grad_q)
#define PDVC_SQ_DKV(DD)                                                                                              \
    hipLaunchKernelGGL((seqattn_bwd_dkv_kernel<DD, DROP, KPM>), gk, dim3(kSqThreads), 0, s, q, k, v, grad_out, lse, \
                       delta, num_heads, num_query, num_key, ldq, ldk, ldv, qmul, scale, kblocks, o, grad_k,         \
                       ld_grad_k, grad_v, ld_grad_v)
    PDVC_SQ_DISPATCH(head_dim, PDVC_SQ_DQ)
    PDVC_SQ_DISPATCH(head_dim, PDVC_SQ_DKV)
#undef PDVC_SQ_DQ
#undef PDVC_SQ_DKV
}

// Shared by the C ABI below and mha.hip's route for long query sets: scale multiplies q . k (the caller's
// convention: 1/sqrt(D) here, sqrt(1/D) there); kpm / dropout as SqOpts.  Arguments validated by the callers.
int sq_forward(const float* q, long ldq, const float* k, long ldk, const float* v, long ldv, int batch,
               int num_query, int num_key, int num_heads, int head_dim, float scale, const uint8_t* kpm,
               float dropout_p, uint64_t seed, const uint64_t* seed_dev, float* out, float* lse, hipStream_t s) {
    const int qblocks = (num_query + kSqOwn - 1) / kSqOwn;
    const long blocks = (long)qblocks * batch * num_heads;
    PDVC_CHECK_ARG(blocks < (1L << 31), "too many (video, head, query block) workgroups");
    PDVC_CHECK_ARG((long)num_key * ldk < (1L << 31) && (long)num_key * ldv < (1L << 31),
                   "one video's keys must span < 2^31 floats");
    const SqOpts o{kpm, seed, seed_dev, drop_threshold(dropout_p), dropout_p > 0.f ? 1.f / (1.f - dropout_p) : 1.f};
    const dim3 grid((unsigned)blocks);
    const float qmul = scale * kLog2e;
    const bool drop = dropout_p > 0.f;
    if (drop && kpm)
        sq_launch_fwd<true, true>(grid, s, q, ldq, k, ldk, v, ldv, batch, num_query, num_key, num_heads, head_dim,
                                  qmul, qblocks, o, out, lse);
    else if (drop)
        sq_launch_fwd<true, false>(grid, s, q, ldq, k, ldk, v, ldv, batch, num_query, num_key, num_heads, head_dim,
                                   qmul, qblocks, o, out, lse);
    else if (kpm)
        sq_launch_fwd<false, true>(grid, s, q, ldq, k, ldk, v, ldv, batch, num_query, num_key, num_heads, head_dim,
                                   qmul, qblocks, o, out, lse);
    else
        sq_launch_fwd<false, false>(grid, s, q, ldq, k, ldk, v, ldv, batch, num_query, num_key, num_heads, head_dim,
                                    qmul, qblocks, o, out, lse);
    PDVC_CHECK_LAUNCH("seqattn_fwd_kernel");
    return PDVC_OK;
}

int sq_backward(const float* q, long ldq, const float* k, long ldk, const float* v, long ldv, const float* out,
                const float* grad_out, const float* lse, int batch, int num_query, int num_key, int num_heads,
                int head_dim, float scale, const uint8_t* kpm, float dropout_p, uint64_t seed,
                const uint64_t* seed_dev, float* workspace, float* grad_q, long ld_grad_q, float* grad_k,
                long ld_grad_k, float* grad_v, long ld_grad_v, hipStream_t s) {
    const long E = (long)num_heads * head_dim;
    if (num_query == 0) {  // no query: the key and value gradients are zero
        hipError_t e1 = hipMemset2DAsync(grad_k, sizeof(float) * ld_grad_k, 0, sizeof(float) * E,
                                         (size_t)batch * num_key, s);
        hipError_t e2 = hipMemset2DAsync(grad_v, sizeof(float) * ld_grad_v, 0, sizeof(float) * E,
                                         (size_t)batch * num_key, s);
        if (e1 != hipSuccess || e2 != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "memset grad_k/grad_v");
        return PDVC_OK;
    }
    const int qblocks = (num_query + kSqOwn - 1) / kSqOwn, kblocks = (num_key + kSqOwn - 1) / kSqOwn;
    const long gq = (long)qblocks * batch * num_heads, gk = (long)kblocks * batch * num_heads;
    PDVC_CHECK_ARG(gq < (1L << 31) && gk < (1L << 31), "too many (video, head, block) workgroups");
    PDVC_CHECK_ARG((long)num_query * ldq < (1L << 31) && (long)num_query * E < (1L << 31) &&
                       (long)num_key * ldk < (1L << 31) && (long)num_key * ldv < (1L << 31),
                   "one video's rows must span < 2^31 floats");
    const SqOpts o{kpm, seed, seed_dev, drop_threshold(dropout_p), dropout_p > 0.f ? 1.f / (1.f - dropout_p) : 1.f};
    float* delta = workspace;  // (N, H, Tq): written by the dq kernel, read by the dk/dv kernel
    const float qmul = scale * kLog2e;
    const bool drop = dropout_p > 0.f;
#define PDVC_SQ_BWD(DR, KP)                                                                                      \
    sq_launch_bwd<DR, KP>(dim3((unsigned)gq), dim3((unsigned)gk), s, q, ldq, k, ldk, v, ldv, out, grad_out, lse, \
                          num_query, num_key, num_heads, head_dim, qmul, scale, qblocks, kblocks, o, delta, grad_q,   \
                          ld_grad_q, grad_k, ld_grad_k, grad_v, ld_grad_v)
    if (drop && kpm) PDVC_SQ_BWD(true, true);
    else if (drop) PDVC_SQ_BWD(true, false);
    else if (kpm) PDVC_SQ_BWD(false, true);
    else PDVC_SQ_BWD(false, false);
#undef PDVC_SQ_BWD
    PDVC_CHECK_LAUNCH("seqattn_bwd_dq_kernel / seqattn_bwd_dkv_kernel");
    return PDVC_OK;
}

}  // namespace pdvc

using namespace pdvc;

extern "C" int pdvc_seq_attention_forward_f32(const float* q, long ldq, const float* k, long ldk, const float* v,
                                              long ldv, int batch, int num_query, int num_key, int num_heads,
                                              int head_dim, float* out, float* lse, void* stream) {
    PDVC_CHECK_ARG(batch >= 0 && num_query >= 0 && num_key > 0 && num_heads > 0, "invalid sizes");
    PDVC_CHECK_ARG(sq_head_dim_ok(head_dim), "head_dim must be 16, 24, 32, 48 or 64, got %d", head_dim);
    const long E = (long)num_heads * head_dim;
    PDVC_CHECK_ARG(ldq >= E && ldk >= E && ldv >= E, "row strides must be >= num_heads * head_dim");
    if (batch == 0 || num_query == 0) return PDVC_OK;
    return sq_forward(q, ldq, k, ldk, v, ldv, batch, num_query, num_key, num_heads, head_dim,
                      1.f / sqrtf((float)head_dim), nullptr, 0.f, 0, nullptr, out, lse, (hipStream_t)stream);
}

extern "C" int pdvc_seq_attention_backward_f32(const float* q, long ldq, const float* k, long ldk, const float* v,
                                               long ldv, const float* out, const float* grad_out, const float* lse,
                                               int batch, int num_query, int num_key, int num_heads, int head_dim,
                                               float* workspace, float* grad_q, long ld_grad_q, float* grad_k,
                                               long ld_grad_k, float* grad_v, long ld_grad_v, void* stream) {
    PDVC_CHECK_ARG(batch >= 0 && num_query >= 0 && num_key > 0 && num_heads > 0, "invalid sizes");
    PDVC_CHECK_ARG(sq_head_dim_ok(head_dim), "head_dim must be 16, 24, 32, 48 or 64, got %d", head_dim);
    const long E = (long)num_heads * head_dim;
    PDVC_CHECK_ARG(ldq >= E && ldk >= E && ldv >= E && ld_grad_q >= E && ld_grad_k >= E && ld_grad_v >= E,
                   "row strides must be >= num_heads * head_dim");
    if (batch == 0) return PDVC_OK;
    return sq_backward(q, ldq, k, ldk, v, ldv, out, grad_out, lse, batch, num_query, num_key, num_heads, head_dim,
                       1.f / sqrtf((float)head_dim), nullptr, 0.f, 0, nullptr, workspace, grad_q, ld_grad_q, grad_k,
                       ld_grad_k, grad_v, ld_grad_v, (hipStream_t)stream);
}
