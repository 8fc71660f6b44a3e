// gemm3.hip -- fp32 GEMM on the gfx950 bf16 matrix cores by exact three-term splitting.
//
// gfx950 has no xf32: the f32-input MFMA runs at 64 FLOP/clk/SIMD (157 TF/s), 1/16 of the bf16 MFMA rate.  Every
// fp32 operand x is split on its way into LDS into three bf16 terms by round-to-nearest,
//     x0 = bf16(x),  x1 = bf16(x - x0),  x2 = bf16(x - x0 - x1) = x - x0 - x1  (exactly),
// with |x1| <= 2^-8 |x| and |x2| <= 2^-16 |x| -- the split is EXACT for normal fp32 values (24 significant bits in
// three 8-bit pieces; the subtractions are exact in fp32).  The product keeps the six terms whose order is at most
// 2^-16:  a.b = a0b0 + (a0b1 + a1b0) + (a0b2 + a2b0 + a1b1) + drop,  |drop| = |a1b2 + a2b1 + a2b2| <= 2^-23 |a||b|,
// i.e. the same order as the rounding of one fp32 product (2^-24); every bf16 x bf16 product is exact in the fp32
// accumulator of v_mfma_f32_32x32x16_bf16.  Six bf16 MFMAs per 32x32x16 step = 1024 * 16 / 6 / 64 = 2.67x the
// f32-input MFMA's rate in exact arithmetic terms.  tests/test_gpu_gemm3.py measures the error against float64
// next to hipBLASLt's fp32 GEMM on the same operands (GEMMs).
//
//   C[M,N] (op) = sum_k opA[m,k] * opB[n,k]
//   A_KC: A[m*lda + k] (k contiguous) else A[k*lda + m];   B_KC: B[n*ldb + k] else B[k*ldb + n]
//   nn.Linear: forward  y = x W^T       A = x (KC),  B = W (KC)
//              dgrad    dx = dy W       A = dy (KC), B = W (MC: opB[n=in, k=out] = W[k*in + n])
//              wgrad    dW = dy^T x     A = dy (MC), B = x (MC); the reduction (rows) split over gridDim.z
//
// Tiling: a 512-thread workgroup (8 waves) computes a BM x BN tile, each wave a 64 x 64 piece as 2 x 2 blocks of
// 32 x 32; K advances in 32-deep stages.  A stage's fp32 slices are loaded into registers one stage ahead (full 128-B
// lines for k-contiguous operands; 4 x 4 micro-blocks transposed in registers for mn-contiguous ones), split, and
// written as three bf16 plane images [row][32 k] (64-B rows; the 16-B k-chunk index XOR-swizzled by (row >> 2) & 3,
// so the 16-lane groups of a fragment read hit 16 distinct 16-B bank slots), double buffered: one barrier a stage.
#include <type_traits>

#include "an_hash.h"
#include "ffn_hash.h"
#include "pdvc_common.h"

namespace pdvc {
namespace g3 {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#ifndef G3_ASPREAD
#define G3_ASPREAD 1  // gemm3p: A pieces split and reloaded one per spread-out MFMA group (0: groups 2-3, reload at 4)
#endif
#ifndef G3_AL2
#define G3_AL2 0
#endif
#ifndef G3_ABLATE
#define G3_ABLATE 0  // measurement-only builds (tools/variant_lib.sh): 1 no staging stores, 2 no staging loads, 4 no MFMA,
                     // 8 no B-plane DMA (gemm3p), 16 no gemm3p epilogue
#endif

constexpr int BK = 32;     // k per stage
constexpr int ROWB = 64;   // bytes per LDS image row (BK bf16)
constexpr int NT = 512;    // threads per workgroup

enum { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_RELU = 2, EPI_ACCUM = 3, EPI_SLAB = 4, EPI_BIAS_RELU_DROP = 5,
       EPI_DMASK = 6, EPI_RESID_DROP = 7 };

// EPI_BIAS_RELU_DROP: the feed-forward block's relu -> dropout in the epilogue of linear1 (ffn.hip's forward pass,
// the same keep mask bit for bit: ffn_hash.h); seed read on the device (graph-safe), scale = 1 / (1 - p)
struct Drop {
    const uint64_t* seed;
    uint32_t thresh;
    float scale;
    const float* hd;  // EPI_DMASK: the forward's relu -> dropout output (C's shape and ldc); C = hd > 0 ? acc * scale : 0
                      // EPI_RESID_DROP: the residual x (C's shape and ldc); C = x + keep ? (acc + bias) * scale : 0
};

__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
    const bf16x2 h = __builtin_convertvector((f32x2){a, b}, bf16x2);  // v_cvt_pk_bf16_f32, round to nearest even
    return __builtin_bit_cast(unsigned, h);
}

// a - b as one v_sub_f32: written plainly, the compiler pairs the two lanes' subtractions into v_pk_add_f32, a
// packed fp32 op that costs more issue cycles beside MFMAs than two plain ones (MI355X_MICROARCH.md, constants)
__device__ __forceinline__ float sub_f32(float a, float b) {
    float r;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// x -> (x0, x1, x2) for two values; packed pairs, element 0 in the low half (the lower k)
__device__ __forceinline__ void split2(float a, float b, unsigned& p0, unsigned& p1, unsigned& p2) {
    p0 = pk_bf16(a, b);
    const float ra = sub_f32(a, __uint_as_float(p0 << 16));
    const float rb = sub_f32(b, __uint_as_float(p0 & 0xffff0000u));
    p1 = pk_bf16(ra, rb);
    const float sa = sub_f32(ra, __uint_as_float(p1 << 16));
    const float sb = sub_f32(rb, __uint_as_float(p1 & 0xffff0000u));
    p2 = pk_bf16(sa, sb);
}

// byte offset of the 4 k values [4*k4, 4*k4 + 4) of image row `row`
__device__ __forceinline__ int unit_off(int row, int k4) {
    return row * ROWB + ((((k4 >> 1) ^ (row >> 2)) & 3) << 4) + ((k4 & 1) << 3);
}
// byte offset of the 8 k values [8*c, 8*c + 8) of image row `row` (a fragment's 16 bytes)
__device__ __forceinline__ int frag_off(int row, int c) { return row * ROWB + (((c ^ (row >> 2)) & 3) << 4); }

// One operand's stage: R rows (m or n) x BK k, staged through registers (NV float4 per thread) as NU pieces: a KC
// piece is 4 k values of one row (threads 8 apart walk a row: full 128-B lines), an MC piece a 4 k x 4 mn block
// transposed in registers (k group fastest across lanes: 8 lanes cover one 128-B line of each of 4 k rows, and the
// 8 lanes of one mn group then write a whole 64-B image row -- conflict-free).
template <int R, bool KC>
struct Stage {
    static constexpr int NP = KC ? R * BK / 4 : (R / 4) * (BK / 4);  // pieces per stage
    static constexpr int NU = (NP + NT - 1) / NT;
    static constexpr int NV = KC ? NU : 4 * NU;  // float4 registers
    float4 v[NV];

    __device__ __forceinline__ static bool has(int i) { return NP % NT == 0 || (int)threadIdx.x + NT * i < NP; }

    // unconditional loads (no branch, no per-load wait): K is a multiple of BK, so a stage never leaves the k range;
    // rows (KC) or column groups (MC) past the matrix are clamped to its last one -- they feed only outputs that are
    // never stored
    __device__ __forceinline__ void load(int i, const float* __restrict__ P, long ld, int mn0, int k0, int MN) {
        const int u = has(i) ? threadIdx.x + NT * i : 0;
        if constexpr (KC) {
            const int row = min(mn0 + (u >> 3), MN - 1), k = k0 + ((u & 7) << 2);
            v[i] = *reinterpret_cast<const float4*>(P + (long)row * ld + k);
        } else {
            const int kg = u & 7, mn = min(mn0 + 4 * (u >> 3), MN - 4);
            const float* q = P + (long)(k0 + 4 * kg) * ld + mn;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 * i + j] = *reinterpret_cast<const float4*>(q + j * ld);
        }
    }

    // split piece i and write its three planes (plane p at img + p * R * ROWB)
    __device__ __forceinline__ void store(int i, char* __restrict__ img) const {
        if (!has(i)) return;
        const int u = threadIdx.x + NT * i;
        if constexpr (KC) {
            const int off = unit_off(u >> 3, u & 7);
            uint2 p0, p1, p2;
            split2(v[i].x, v[i].y, p0.x, p1.x, p2.x);
            split2(v[i].z, v[i].w, p0.y, p1.y, p2.y);
            *reinterpret_cast<uint2*>(img + off) = p0;
            *reinterpret_cast<uint2*>(img + R * ROWB + off) = p1;
            *reinterpret_cast<uint2*>(img + 2 * R * ROWB + off) = p2;
        } else {
            const int kg = u & 7, r0 = 4 * (u >> 3);
            const float4* q = v + 4 * i;
            // image row r0 + e takes (q[0].e, q[1].e, q[2].e, q[3].e): k = 4kg .. 4kg + 3.  A ds_write_b64 serves 16
            // lanes (two mn groups) per LDS cycle in 128 B: rows 4m + e and 4m + 4 + e would share one 64-B half (a
            // 2-way conflict), so the odd mn group writes its rows in the order e ^ 1 -- rows 3 or 5 apart
            const bool odd = (u >> 3) & 1;
#define G3_SEL(A, B) (odd ? (B) : (A))
#define G3_COL(E, F, G)                                                                     \
    {                                                                                      \
        const int off = unit_off(r0 + ((E) ^ (int)odd), kg);                               \
        uint2 p0, p1, p2;                                                                  \
        split2(G3_SEL(q[0].F, q[0].G), G3_SEL(q[1].F, q[1].G), p0.x, p1.x, p2.x);          \
        split2(G3_SEL(q[2].F, q[2].G), G3_SEL(q[3].F, q[3].G), p0.y, p1.y, p2.y);          \
        *reinterpret_cast<uint2*>(img + off) = p0;                                         \
        *reinterpret_cast<uint2*>(img + R * ROWB + off) = p1;                              \
        *reinterpret_cast<uint2*>(img + 2 * R * ROWB + off) = p2;                          \
    }
            G3_COL(0, x, y) G3_COL(1, y, x) G3_COL(2, z, w) G3_COL(3, w, z)
#undef G3_COL
#undef G3_SEL
        }
    }
    __device__ __forceinline__ void load_all(const float* P, long ld, int mn0, int k0, int MN) {
#pragma unroll
        for (int i = 0; i < NU; ++i) load(i, P, ld, mn0, k0, MN);
    }
    __device__ __forceinline__ void store_all(char* img) const {
#pragma unroll
        for (int i = 0; i < NU; ++i) store(i, img);
    }
};

// the six products of one 32 x 32 x 16 step, smallest terms first
__device__ __forceinline__ f32x16 mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 x) {
    x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], x, 0, 0, 0);
    return x;
}

// accumulator layouts: SZ = 32, v_mfma_f32_32x32x16_bf16 (register r of lane l: row (r & 3) + 8 (r >> 2) + 4 (l >> 5),
// column l & 31); SZ = 16, v_mfma_f32_16x16x32_bf16 (row r + 4 (l >> 4), column l & 15; a 16 x 16 x 32 form of
// gemm3p / gemm3w measured slower, profiles/r06_gemm3_rejected.txt).  lrow / lcol: the lane's row offset and
// column
template <int SZ> struct Lay;
template <> struct Lay<32> {
    typedef f32x16 acc_t;
    static constexpr int NR = 16;
    __device__ static constexpr int dr(int r) { return (r & 3) + 8 * (r >> 2); }
};
template <> struct Lay<16> {
    typedef f32x4 acc_t;
    static constexpr int NR = 4;
    __device__ static constexpr int dr(int r) { return r; }
};

template <int EPI, bool FULL, int BI = 2, int BJ = 2, int SZ = 32>
__device__ __forceinline__ void store_tile(const typename Lay<SZ>::acc_t (&acc)[BI][BJ], float* __restrict__ C,
                                           long ldc, const float* __restrict__ bias, int r0, int c0, int M, int N,
                                           int lcol, int lrow, Drop drp = Drop{nullptr, 0u, 1.f, nullptr}) {
    constexpr int NR = Lay<SZ>::NR;
    constexpr bool BIASED = EPI == EPI_BIAS || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_RELU_DROP;
    if constexpr (EPI == EPI_RESID_DROP) {
        // the residual sub-layer's sum t = x + dropout(acc + bias) for the add-norm pass that then reads t alone:
        // the keep mask of addnorm.hip's forward (an_hash.h) for element (row, col), its row part once per row;
        // seed == NULL: no dropout (p = 0).  The block row's residual values are loaded before its stores (as the
        // accumulate epilogue: interleaved, every load would wait for the stores before it)
        const bool drop = drp.seed != nullptr;
        const uint64_t seed = drop ? *drp.seed : 0ull;
        uint32_t cterm[BJ];
        float bvs[BJ];
#pragma unroll
        for (int j = 0; j < BJ; ++j) {
            const int col = c0 + SZ * j + lcol;
            cterm[j] = an_col(seed, (uint32_t)col);
            bvs[j] = bias[(FULL || col < N) ? col : 0];
        }
#pragma unroll
        for (int i = 0; i < BI; ++i) {
            const int rbase = r0 + SZ * i + lrow;
            float old[BJ][NR];
#pragma unroll
            for (int j = 0; j < BJ; ++j) {
                const int col = c0 + SZ * j + lcol;
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int row = rbase + Lay<SZ>::dr(r);
                    old[j][r] = (FULL || (col < N && row < M)) ? drp.hd[(long)row * ldc + col] : 0.f;
                }
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int row = rbase + Lay<SZ>::dr(r);
                const uint32_t rm = an_row(seed, (uint32_t)row);
#pragma unroll
                for (int j = 0; j < BJ; ++j) {
                    const int col = c0 + SZ * j + lcol;
                    if (FULL || (col < N && row < M)) {
                        float v = acc[i][j][r] + bvs[j];
                        if (drop) v = (an_mix(rm + cterm[j]) >> 8) >= drp.thresh ? v * drp.scale : 0.f;
                        C[(long)row * ldc + col] = old[j][r] + v;
                    }
                }
            }
        }
        return;
    }
    if constexpr (EPI == EPI_BIAS_RELU_DROP) {
        // ffn_keep's hash split by what it depends on: the inner mix of the row once per row (rows outer, the column
        // blocks inner), the column term once per column block -- the v_mul_lo_u32 of the mask are quarter-rate
        const uint64_t seed = *drp.seed;
        uint32_t cterm[BJ];
        float bvs[BJ];
#pragma unroll
        for (int j = 0; j < BJ; ++j) {
            const int col = c0 + SZ * j + lcol;
            cterm[j] = (uint32_t)col * 0xc2b2ae35U + (uint32_t)(seed >> 32);
            bvs[j] = bias[(FULL || col < N) ? col : 0];
        }
#pragma unroll
        for (int i = 0; i < BI; ++i) {
            const int rbase = r0 + SZ * i + lrow;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int dr = Lay<SZ>::dr(r), row = rbase + dr;
                const uint32_t rm = ffn_mix((uint32_t)row * 0x9e3779b1U ^ (uint32_t)seed);
#pragma unroll
                for (int j = 0; j < BJ; ++j) {
                    const int col = c0 + SZ * j + lcol;
                    if (FULL || (col < N && row < M)) {
                        const float v = fmaxf(acc[i][j][r] + bvs[j], 0.f);
                        const bool keep = (ffn_mix(rm + cterm[j]) >> 8) >= drp.thresh;
                        C[(long)row * ldc + col] = keep ? v * drp.scale : 0.f;
                    }
                }
            }
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
        const int col = c0 + SZ * j + lcol;
        const bool colok = FULL || col < N;
        const float bv = BIASED ? bias[colok ? col : 0] : 0.f;
#pragma unroll
        for (int i = 0; i < BI; ++i) {
            const int rbase = r0 + SZ * i + lrow;
            float* p0 = C + (long)rbase * ldc + col;
            // accumulate: the block's 16 old values loaded before any store -- the rows are distinct (ldc >= N >= 1),
            // but the compiler cannot prove a store leaves the next row's load alone, and interleaved it waited for
            // every load in turn (load, vmcnt(0), add, store: 128 round trips per lane and tile)
            float old[NR];
            if constexpr (EPI == EPI_ACCUM || EPI == EPI_DMASK) {  // (EPI_DMASK: the forward output's values)
                const float* q0 = EPI == EPI_DMASK ? drp.hd + ((long)rbase * ldc + col) : p0;
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int dr = Lay<SZ>::dr(r);
                    old[r] = (FULL || (colok && rbase + dr < M)) ? q0[(long)dr * ldc] : 0.f;
                }
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int dr = Lay<SZ>::dr(r);
                if (FULL || (colok && rbase + dr < M)) {
                    float v = acc[i][j][r] + bv;
                    if (EPI == EPI_BIAS_RELU) v = fmaxf(v, 0.f);
                    float* p = p0 + (long)dr * ldc;
                    if constexpr (EPI == EPI_ACCUM) v += old[r];
                    if constexpr (EPI == EPI_DMASK) v = old[r] > 0.f ? v * drp.scale : 0.f;
                    *p = v;
                }
            }
        }
    }
}

// one k16 step's fragments of a wave's 64 x 64 piece: a[i][p] rows wm + 32 i, b[j][p] rows wn + 32 j, plane p
struct Frags {
    bf16x8 a[2][3], b[2][3];
};

template <int BM, int BN>
__device__ __forceinline__ void read_frags(Frags& f, const char* img, int wm, int wn, int ks, int l32, int h) {
    constexpr int AIMG = 3 * BM * ROWB;
    const int c = 2 * ks + h;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ra = wm + 32 * i + l32, rb = wn + 32 * i + l32;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            f.a[i][p] = *reinterpret_cast<const bf16x8*>(img + p * BM * ROWB + frag_off(ra, c));
            f.b[i][p] = *reinterpret_cast<const bf16x8*>(img + AIMG + p * BN * ROWB + frag_off(rb, c));
        }
    }
}

template <int BM, int BN, bool AKC, bool BKC, int EPI>
__global__ __launch_bounds__(NT, 1) void gemm3_kernel(int M, int N, int K, const float* __restrict__ A, long lda,
                                                      const float* __restrict__ B, long ldb, float* __restrict__ C,
                                                      long ldc, const float* __restrict__ bias, int k_per_split,
                                                      int tiles_n, long slab) {
    static_assert((BM / 64) * (BN / 64) == NT / 64, "one 64 x 64 piece per wave");
    constexpr int AIMG = 3 * BM * ROWB, BIMG = 3 * BN * ROWB, STAGE = AIMG + BIMG;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);  // the tiles of one row block run on one XCD (A from its L2)
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kb = blockIdx.z * k_per_split;
    const int nst = (min(K, kb + k_per_split) - kb) / BK;
    const int wm = (wid / (BN / 64)) * 64, wn = (wid % (BN / 64)) * 64;
    const int l32 = lane & 31, h = lane >> 5;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // register ring one stage deep: the registers hold stage s + 1 while stage s computes; they are split into the
    // other LDS buffer among the first k16 step's MFMAs and reloaded with stage s + 2 after them.  The second k16
    // step's fragments (f1) are consumed after the stage's barrier, covering the next stage's first reads (gemm3p).
    Stage<BM, AKC> sa;
    Stage<BN, BKC> sb;
    Frags f0, f1;
    if (nst > 0) {
        sa.load_all(A, lda, m0, kb, M);
        sb.load_all(B, ldb, n0, kb, N);
        sa.store_all(lds);
        sb.store_all(lds + AIMG);
        if (nst > 1) {
            sa.load_all(A, lda, m0, kb + BK, M);
            sb.load_all(B, ldb, n0, kb + BK, N);
        }
    }
    __syncthreads();
    if (nst > 0) read_frags<BM, BN>(f0, lds, wm, wn, 0, l32, h);
    for (int s = 0; s < nst; ++s) {
        const char* cur = lds + (s & 1) * STAGE;
        char* nxt = lds + ((s + 1) & 1) * STAGE;
        const bool more = s + 1 < nst, more2 = s + 2 < nst;
        read_frags<BM, BN>(f1, cur, wm, wn, 1, l32, h);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = q >> 1, j = q & 1;
            if constexpr ((G3_ABLATE & 4) == 0) acc[i][j] = mfma6(f0.a[i], f0.b[j], acc[i][j]);
            else {
#pragma unroll
                for (int p = 0; p < 3; ++p) asm volatile("" ::"v"(f0.a[i][p]), "v"(f0.b[j][p]));
            }
            if (more && (G3_ABLATE & 1) == 0) {
                // staging work between the MFMA groups: A pieces, then B pieces, spread over the four groups
#pragma unroll
                for (int u = 0; u < Stage<BM, AKC>::NU; ++u)
                    if (u * 4 / (Stage<BM, AKC>::NU + Stage<BN, BKC>::NU) == q) sa.store(u, nxt);
#pragma unroll
                for (int u = 0; u < Stage<BN, BKC>::NU; ++u)
                    if ((Stage<BM, AKC>::NU + u) * 4 / (Stage<BM, AKC>::NU + Stage<BN, BKC>::NU) == q)
                        sb.store(u, nxt + AIMG);
            }
            if (q == 3 && more2 && (G3_ABLATE & 2) == 0) {
                sa.load_all(A, lda, m0, kb + (s + 2) * BK, M);
                sb.load_all(B, ldb, n0, kb + (s + 2) * BK, N);
            }
        }
        __syncthreads();
        if (more) read_frags<BM, BN>(f0, nxt, wm, wn, 0, l32, h);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr ((G3_ABLATE & 4) == 0)
                acc[q >> 1][q & 1] = mfma6(f1.a[q >> 1], f1.b[q & 1], acc[q >> 1][q & 1]);
            else {
#pragma unroll
                for (int p = 0; p < 3; ++p) asm volatile("" ::"v"(f1.a[q >> 1][p]), "v"(f1.b[q & 1][p]));
            }
        }
    }

    // epilogue: acc[i][j] register r of lane l is C[row][col], col = l % 32, row = (r & 3) + 8 (r >> 2) + 4 (l / 32)
    float* Cz = C + (EPI == EPI_SLAB ? (long)blockIdx.z * slab : 0);
    const bool full = m0 + BM <= M && n0 + BN <= N;  // whole tile inside C: no per-element checks
    if (full) {
        store_tile<EPI, true>(acc, Cz, ldc, bias, m0 + wm, n0 + wn, M, N, l32, 4 * h);
    } else {
        store_tile<EPI, false>(acc, Cz, ldc, bias, m0 + wm, n0 + wn, M, N, l32, 4 * h);
    }
}

// ---- opB pre-split: the weight operand's three planes made once per call (split_planes_kernel) and streamed into
// LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no VALU), so the in-loop split work is the A operand's
// alone.  Tile BM = 128 (A, split in registers) x BN = 256 (B planes), 8 waves of 64 x 64.

typedef __attribute__((address_space(3))) void g3_lds_t;

// planes[p][n][k] (bf16 bits) of opB[n][k]; b_kc 1: B[n*ldb + k], 0: B[k*ldb + n].  One thread per 4 k of a row.
// NP = 1: plane 0 only (the bf16 rounding, for the bf16 mode's product)
template <int NP>
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ B, long ldb, int b_kc, int N,
                                                           int K, uint16_t* __restrict__ planes) {
    const long n4 = (long)N * (K / 4);
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const int n = (int)(i / (K / 4)), k = (int)(i % (K / 4)) * 4;
        float v[4];
        if (b_kc) {
            const float4 x = *reinterpret_cast<const float4*>(B + (long)n * ldb + k);
            v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = B[(long)(k + j) * ldb + n];
        }
        const long o = (long)n * K + k;
        if constexpr (NP == 1) {
            *reinterpret_cast<uint2*>(planes + o) = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
            continue;
        }
        uint2 p0, p1, p2;
        split2(v[0], v[1], p0.x, p1.x, p2.x);
        split2(v[2], v[3], p0.y, p1.y, p2.y);
        *reinterpret_cast<uint2*>(planes + o) = p0;
        *reinterpret_cast<uint2*>(planes + (long)N * K + o) = p1;
        *reinterpret_cast<uint2*>(planes + 2L * N * K + o) = p2;
    }
}

// one LDS-DMA wave-instruction: 16 image rows x 64 B of one plane.  Lane l lands at dst + 16 l = row l / 4, slot
// l % 4; the slot holds k chunk (l % 4) ^ ((row >> 2) & 3) (the image's swizzle, applied on the source address).
// Issued by inline assembly: the compiler neither sees nor waits for it (its own waits only over-count, never
// under-count, since these DMAs only add to vmcnt); the kernel retires them with an explicit vmcnt before the barrier.
__device__ __forceinline__ void planes_dma(char* dst, const uint16_t* __restrict__ plane, int K, int row0, int N,
                                           int k0, int lane) {
    const int row = row0 + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 2) & 3);
    const uint16_t* src = plane + (long)min(row, N - 1) * K + k0 + 8 * c;
    const uint32_t d = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(g3_lds_t*)dst);
    int keep;
    __asm__ volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(d)
                     : "memory");
}

// gemm3p geometry: a 256 x 256 tile, K in 16-deep stages through a ring of three LDS stages (3 x 48 KiB), 8 waves of
// 128 x 64 (4 x 2 blocks of 32 x 32: 48 MFMAs a stage, 18 fragment reads).  Against a 128 x 256 tile of 32-deep
// stages this halves the L2 -> LDS bytes and the fragment reads per MFMA, and the ring keeps the DMAs and row loads two
// stages ahead of their use.  Image rows are 32 B (16 bf16); the 16-B half of row r holding k chunk c is
// c ^ ((r >> 3) & 1), so the 16-lane groups of a fragment read and the DMA / A-row writes are conflict-free.
namespace p3 {
constexpr int BM = 256, BN = 256, KS = 16, RB = 32, NSTAGE = 3;
constexpr int NUA = BM * KS / 4 / NT;  // A pieces (4 k of a row) per thread: 2
// NP planes per operand: 3 = the exact fp32 product (six MFMA terms; images 24 + 24 KiB, 3 1-KiB DMAs per wave per
// stage); 1 = the bf16 mode's product (operands rounded to bf16, one MFMA term; 8 + 8 KiB, one DMA)
template <int NP> struct Geo {
    static constexpr int AIMG = NP * BM * RB, BIMG = NP * BN * RB, STAGE = AIMG + BIMG;
    static constexpr int BDMA = NP * BN * RB / 1024 / (NT / 64);
};

__device__ __forceinline__ int unit_off16(int row, int k4) {
    return row * RB + ((((k4 >> 1) ^ (row >> 3)) & 1) << 4) + ((k4 & 1) << 3);
}
__device__ __forceinline__ int frag_off16(int row, int h) { return row * RB + (((h ^ (row >> 3)) & 1) << 4); }

struct ARegs {
    float4 v[NUA];
    __device__ __forceinline__ void load(const float* __restrict__ A, long lda, int m0, int k0, int M) {
#pragma unroll
        for (int i = 0; i < NUA; ++i) load1(i, A, lda, m0, k0, M);
    }
    __device__ __forceinline__ void load1(int i, const float* __restrict__ A, long lda, int m0, int k0, int M) {
        {
            const int u = threadIdx.x + NT * i;
#if G3_AL2  // measurement only: every tile reads the first 256 rows (L2-resident A)
            const int row = (u >> 2) + 0 * m0;
#else
            const int row = min(m0 + (u >> 2), M - 1);
#endif
            v[i] = *reinterpret_cast<const float4*>(A + (long)row * lda + k0 + ((u & 3) << 2));
        }
    }
    template <int NP = 3>
    __device__ __forceinline__ void store(int i, char* __restrict__ img) const {
        const int u = threadIdx.x + NT * i;
        const int off = unit_off16(u >> 2, u & 3);
        if constexpr (NP == 1) {  // the bf16 rounding only (v_cvt_pk_bf16_f32: RNE, torch's .to(bfloat16))
            *reinterpret_cast<uint2*>(img + off) = make_uint2(pk_bf16(v[i].x, v[i].y), pk_bf16(v[i].z, v[i].w));
            return;
        }
        uint2 q0, q1, q2;
        split2(v[i].x, v[i].y, q0.x, q1.x, q2.x);
        split2(v[i].z, v[i].w, q0.y, q1.y, q2.y);
        *reinterpret_cast<uint2*>(img + off) = q0;
        *reinterpret_cast<uint2*>(img + BM * RB + off) = q1;
        *reinterpret_cast<uint2*>(img + 2 * BM * RB + off) = q2;
    }
};

// one 1-KiB LDS-DMA wave-instruction: 32 image rows x 32 B of one plane; lane l lands at dst + 16 l = row l / 2,
// half l % 2, which holds k chunk (l % 2) ^ ((row >> 3) & 1)
__device__ __forceinline__ void dma32(char* dst, const uint16_t* __restrict__ plane, int K, int row0, int N, int k0,
                                      int lane) {
    const int row = row0 + (lane >> 1);
    const int c = (lane & 1) ^ ((row >> 3) & 1);
    const uint16_t* src = plane + (long)min(row, N - 1) * K + k0 + 8 * c;
    const uint32_t d = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(g3_lds_t*)dst);
    int keep;
    __asm__ volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(d)
                     : "memory");
}
}  // namespace p3

template <int EPI, int NP = 3>
__global__ __launch_bounds__(NT, 1) void gemm3p_kernel(int M, int N, int K, const float* __restrict__ A, long lda,
                                                       const uint16_t* __restrict__ planes, float* __restrict__ C,
                                                       long ldc, const float* __restrict__ bias, int tiles_n,
                                                       Drop drp) {
    using namespace p3;
    constexpr int AIMG = Geo<NP>::AIMG, STAGE = Geo<NP>::STAGE, BDMA = Geo<NP>::BDMA;
    __shared__ __attribute__((aligned(16))) char lds[NSTAGE * STAGE];

    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);  // the column tiles of one row block share an XCD's L2
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int nst = K / KS;
    const int wm = (wid >> 2) * 128, wn = (wid & 3) * 64;
    const int l32 = lane & 31, h = lane >> 5;
    const long pstride = (long)N * K;

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto b_dma = [&](char* img, int k0) {
#pragma unroll
        for (int q = 0; q < BDMA; ++q) {
            const int g = wid * BDMA + q;  // 8 NP instructions: plane g / 8, rows 32 (g % 8) ..
            const int p = g / (BN / 32), r0 = (g % (BN / 32)) * 32;
            dma32(img + AIMG + p * BN * RB + r0 * RB, planes + p * pstride, K, n0 + r0, N, k0, lane);
        }
    };

    // prologue: stage 0 complete in LDS, stage 1's DMAs issued and its A rows in registers
    ARegs ra;
    if (nst > 0) {
        ra.load(A, lda, m0, 0, M);
#pragma unroll
        for (int i = 0; i < NUA; ++i) ra.template store<NP>(i, lds);  // (waits for the rows; nothing else is in flight)
        b_dma(lds, 0);
        if (nst > 1) {
            b_dma(lds + STAGE, KS);
            ra.load(A, lda, m0, KS, M);
        }
        // stage 0's DMAs are older than stage 1's DMAs and rows: leave those in flight
        if (nst > 1) __builtin_amdgcn_s_waitcnt(0x0F70 | ((BDMA + NUA) & 15));
        else __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    __syncthreads();
    // one stage; the staging work is compile-time unconditional in the main loop (MORE, MORE2 = true), so the split /
    // store / DMA / load instructions share one basic block with the MFMAs and the scheduler can interleave them (as
    // runtime branches they were separate blocks, each run with the matrix pipe idle); the last two stages are peeled
    auto stage = [&](int s, auto MORE_, auto MORE2_) {
        constexpr bool more = decltype(MORE_)::value, more2 = decltype(MORE2_)::value;
        const char* cur = lds + (s % NSTAGE) * STAGE;
        char* nx1 = lds + ((s + 1) % NSTAGE) * STAGE;
        char* nx2 = lds + ((s + 2) % NSTAGE) * STAGE;
        bf16x8 fa[4][NP], fb[2][NP];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int p = 0; p < NP; ++p)
                fb[j][p] = *reinterpret_cast<const bf16x8*>(cur + AIMG + p * BN * RB + frag_off16(wn + 32 * j + l32, h));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int p = 0; p < NP; ++p)
                fa[i][p] = *reinterpret_cast<const bf16x8*>(cur + p * BM * RB + frag_off16(wm + 32 * i + l32, h));
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int i = q >> 1, j = q & 1;
            if constexpr ((G3_ABLATE & 4) != 0) {
#pragma unroll
                for (int p = 0; p < NP; ++p) asm volatile("" ::"v"(fa[i][p]), "v"(fb[j][p]));
            } else if constexpr (NP == 1) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], acc[i][j], 0, 0, 0);
            } else {
                acc[i][j] = mfma6(fa[i], fb[j], acc[i][j]);
            }
            // stage s + 1's A rows: piece i is split into its buffer at group QA(i) (the compiler waits for it: loaded
            // one whole stage ago) and its register reloaded at once with stage s + 2's piece -- each piece gets a full
            // stage to arrive and the split VALU spreads over the groups; stage s + 2's DMAs at group 4
#if G3_ASPREAD
            constexpr int QA0 = 1, QAS = 8 / NUA;  // pieces at groups 1, 5
            if constexpr (more && (G3_ABLATE & 1) == 0)
                if (q >= QA0 && (q - QA0) % QAS == 0 && (q - QA0) / QAS < NUA) ra.template store<NP>((q - QA0) / QAS, nx1);
            if constexpr (more2 && (G3_ABLATE & 2) == 0)
                if (q >= QA0 && (q - QA0) % QAS == 0 && (q - QA0) / QAS < NUA)
                    ra.load1((q - QA0) / QAS, A, lda, m0, (s + 2) * KS, M);
            if constexpr (more2 && (G3_ABLATE & 8) == 0)
                if (q == 4) b_dma(nx2, (s + 2) * KS);
#else
            if constexpr (more && (G3_ABLATE & 1) == 0)
                if (q >= 2 && q < 2 + NUA) ra.template store<NP>(q - 2, nx1);
            if constexpr (more2 && (G3_ABLATE & 8) == 0)
                if (q == 2 + NUA) b_dma(nx2, (s + 2) * KS);
            if constexpr (more2 && (G3_ABLATE & 2) == 0)
                if (q == 2 + NUA) ra.load(A, lda, m0, (s + 2) * KS, M);
#endif
        }
        if constexpr (more && !more2) __builtin_amdgcn_s_waitcnt(0x0F70);  // the last stage's DMAs (nothing later)
        __syncthreads();
    };
    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;
    int s = 0;
    for (; s + 2 < nst; ++s) stage(s, T_{}, T_{});
    if (s + 1 < nst) stage(s++, T_{}, F_{});
    if (s < nst) stage(s, F_{}, F_{});

    if constexpr ((G3_ABLATE & 16) != 0) {  // measurement only: no epilogue, the accumulators kept live
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[i][j]));
        return;
    }
    const bool full = m0 + BM <= M && n0 + BN <= N;
    if (full) store_tile<EPI, true, 4, 2>(acc, C, ldc, bias, m0 + wm, n0 + wn, M, N, l32, 4 * h, drp);
    else store_tile<EPI, false, 4, 2>(acc, C, ldc, bias, m0 + wm, n0 + wn, M, N, l32, 4 * h, drp);
}

// ---- both operands mn-contiguous (the weight gradient dW = dy^T x: the reduction runs over the rows of both) ----
// gemm3w: a 256 x 256 tile, 16 reduction rows per stage, two LDS stages (2 x 48 KiB), 8 waves of 128 x 64.  The
// images are k-major, [k][256 mn] per plane (512-B rows; the 8-B chunk holding mn 4c .. 4c + 3 of row k sits at chunk
// (c + 8 (k & 3)) & 63): a thread's float4 of 4 consecutive mn is split and stored as it was loaded (16 lanes write
// 128 contiguous bytes, no register transpose), and each 32 x 32 x 16 fragment is two ds_read_b64_tr_b16 (4 k x 16
// mn blocks delivered transposed: lane i of a 16-lane group gets mn i of the block's 4 k rows) -- the row rotation
// puts a half-wave's 4 rows x 8 chunks on 32 distinct 8-B slots.
namespace w3 {
constexpr int BM = 256, BN = 256, KS = 16, ROW = 512, PL = KS * ROW;  // a plane: 16 k rows of 256 mn (8 KiB)
constexpr int AIMG = 3 * PL, STAGE = 6 * PL;                          // 24 + 24 KiB
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int chunk_off(int k, int c) { return k * ROW + (((c + 8 * (k & 3)) & 63) << 3); }

// the 32 x 32 x 16 fragment of plane image `img` at mn base mb: lanes hold mn = mb + (l & 31), k = 8 (l >> 5) + j
__device__ __forceinline__ bf16x8 frag_tr(const char* img, int mb, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int c = ((mb + ((g & 1) << 4)) >> 2) + pp;
    const int k = 8 * (g >> 1) + q;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + chunk_off(k, c)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + chunk_off(k + 4, c)));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    return __builtin_bit_cast(bf16x8, v);
}

struct Regs {  // one stage of both operands: float4 u = t + 512 i (i = 0, 1) is row k = u / 64, mn chunk u % 64
    float4 a[2], b[2];
    __device__ __forceinline__ void load(const float* __restrict__ A, long lda, int m0, int M,
                                         const float* __restrict__ B, long ldb, int n0, int N, int k0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int u = threadIdx.x + NT * i, k = k0 + (u >> 6), c = u & 63;
            a[i] = *reinterpret_cast<const float4*>(A + (long)k * lda + min(m0 + 4 * c, M - 4));
            b[i] = *reinterpret_cast<const float4*>(B + (long)k * ldb + min(n0 + 4 * c, N - 4));
        }
    }
    __device__ __forceinline__ static void put(const float4& v, char* img, int u) {
        const int off = chunk_off(u >> 6, u & 63);
        uint2 q0, q1, q2;
        split2(v.x, v.y, q0.x, q1.x, q2.x);
        split2(v.z, v.w, q0.y, q1.y, q2.y);
        *reinterpret_cast<uint2*>(img + off) = q0;
        *reinterpret_cast<uint2*>(img + PL + off) = q1;
        *reinterpret_cast<uint2*>(img + 2 * PL + off) = q2;
    }
    __device__ __forceinline__ void store(int piece, char* img) const {  // pieces 0, 1: A; 2, 3: B
        const int i = piece & 1, u = threadIdx.x + NT * i;
        if (piece < 2) put(a[i], img, u);
        else put(b[i], img + AIMG, u);
    }
};
}  // namespace w3

// CS: also the column sums of A over this split's reduction rows (the bias gradient sum_k dy[k][m] of the layer whose
// weight gradient this is), taken from the float4s each thread loads anyway: colpart[z * M + m] for split z, written by
// the tiles of column block 0 (deterministic: fixed per-thread order, then the 8 waves summed in order through LDS)
template <int EPI, bool CS = false>
__global__ __launch_bounds__(NT, 1) void gemm3w_kernel(int M, int N, int K, const float* __restrict__ A, long lda,
                                                       const float* __restrict__ B, long ldb, float* __restrict__ C,
                                                       long ldc, int k_per_split, int tiles_n, long slab, int nsplit,
                                                       float* __restrict__ colpart) {
    using namespace w3;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // one 1-D grid over (split, tile): the output tiles of one row chunk are consecutive logical blocks, so they run
    // together on one XCD and read the chunk's rows of both operands from its L2 (a (tile, split) grid dealt them
    // to different XCDs: every tile fetched its rows from HBM -- 7.0 GB per 512 x 512 launch for 4.0 of operands)
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int tiles = gridDim.x / nsplit;
    const int zz = lid / tiles, tile = lid - zz * tiles;
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kb = zz * k_per_split;
    const int nst = (min(K, kb + k_per_split) - kb) / KS;
    const int wm = (wid >> 2) * 128, wn = (wid & 3) * 64;
    const int l32 = lane & 31, h = lane >> 5;

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    Regs rg;
    float4 csum = make_float4(0.f, 0.f, 0.f, 0.f);  // CS: this thread's A column chunk summed over its rows
    const bool csb = CS && tn == 0;                  // (only column block 0's tiles write the sums)
    auto cadd = [&](int i) {
        if (csb) {
            csum.x += rg.a[i].x;
            csum.y += rg.a[i].y;
            csum.z += rg.a[i].z;
            csum.w += rg.a[i].w;
        }
    };
    if (nst > 0) {
        rg.load(A, lda, m0, M, B, ldb, n0, N, kb);
        cadd(0);
        cadd(1);
#pragma unroll
        for (int q = 0; q < 4; ++q) rg.store(q, lds);
        if (nst > 1) rg.load(A, lda, m0, M, B, ldb, n0, N, kb + KS);
    }
    __syncthreads();
    // the main loop's stages are branch-free (compile-time MORE / MORE2), the last two peeled (gemm3p)
    auto stage = [&](int s, auto MORE_, auto MORE2_) {
        constexpr bool more = decltype(MORE_)::value, more2 = decltype(MORE2_)::value;
        const char* cur = lds + (s & 1) * STAGE;
        char* nxt = lds + ((s + 1) & 1) * STAGE;
        bf16x8 fa[4][3], fb[2][3];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int p = 0; p < 3; ++p) fb[j][p] = frag_tr(cur + AIMG + p * PL, wn + 32 * j, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int p = 0; p < 3; ++p) fa[i][p] = frag_tr(cur + p * PL, wm + 32 * i, lane);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int i = q >> 1, j = q & 1;
            acc[i][j] = mfma6(fa[i], fb[j], acc[i][j]);
            if constexpr (more) {
                if (q >= 1 && q <= 4) rg.store(q - 1, nxt);  // stage s + 1 into the other buffer
                if (q == 1 || q == 2) cadd(q - 1);
            }
            if constexpr (more2)
                if (q == 5) rg.load(A, lda, m0, M, B, ldb, n0, N, kb + (s + 2) * KS);
        }
        __syncthreads();
    };
    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;
    int s = 0;
    for (; s + 2 < nst; ++s) stage(s, T_{}, T_{});
    if (s + 1 < nst) stage(s++, T_{}, F_{});
    if (s < nst) stage(s, F_{}, F_{});
    (void)l32;
    if constexpr (CS) {
        if (csb) {  // (block-uniform) LDS is free: the last stage ended with a barrier
            float4* red = reinterpret_cast<float4*>(lds);
            red[threadIdx.x] = csum;  // [wave][column chunk]: the chunk is threadIdx.x % 64 in every stage
            __syncthreads();
            if (threadIdx.x < 64) {
                float4 t = red[threadIdx.x];
#pragma unroll
                for (int w = 1; w < NT / 64; ++w) {
                    const float4 v = red[w * 64 + threadIdx.x];
                    t.x += v.x;
                    t.y += v.y;
                    t.z += v.z;
                    t.w += v.w;
                }
                const int m = m0 + 4 * threadIdx.x;
                if (m < M) *reinterpret_cast<float4*>(colpart + (long)zz * M + m) = t;  // (the clamped loads beyond M dropped)
            }
        }
    }
    float* Cz = C + (EPI == EPI_SLAB ? (long)zz * slab : 0);
    const bool full = m0 + BM <= M && n0 + BN <= N;
    if (full) store_tile<EPI, true, 4, 2>(acc, Cz, ldc, nullptr, m0 + wm, n0 + wn, M, N, l32, 4 * h);
    else store_tile<EPI, false, 4, 2>(acc, Cz, ldc, nullptr, m0 + wm, n0 + wn, M, N, l32, 4 * h);
}

// out[i] (=|+=) sum_z ws[z * n + i], float4 lanes (n % 4 == 0); then, in the same launch, out2[i] = sum_z ws2[z * n2 + i]
// over a second region (the bias-gradient partials of gemm3w<CS>; n2 = 0: none)
template <bool ACC>
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ ws, int splits, long n4,
                                                       float* __restrict__ out, const float* __restrict__ ws2,
                                                       long n42, float* __restrict__ out2) {
    for (long t = blockIdx.x * 256L + threadIdx.x; t < n4 + n42; t += (long)gridDim.x * 256) {
        const bool first = t < n4;
        const long i = first ? t : t - n4, n = first ? n4 : n42;
        const float4* src = reinterpret_cast<const float4*>(first ? ws : ws2);
        float4 s = ACC && first ? reinterpret_cast<const float4*>(out)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        for (int z = 0; z < splits; ++z) {
            const float4 v = src[(long)z * n + i];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        reinterpret_cast<float4*>(first ? out : out2)[i] = s;
    }
}

}  // namespace g3
}  // namespace pdvc

using namespace pdvc;
using namespace pdvc::g3;

namespace {

template <int BM, int BN, bool AKC, bool BKC>
void launch_epi(int epi, dim3 grid, hipStream_t s, int M, int N, int K, const float* A, long lda, const float* B,
                long ldb, float* C, long ldc, const float* bias, int kps, int tiles_n, long slab) {
#define G3_L(E) \
    hipLaunchKernelGGL((gemm3_kernel<BM, BN, AKC, BKC, E>), grid, dim3(NT), 0, s, M, N, K, A, lda, B, ldb, C, ldc, bias, kps, tiles_n, slab)
    switch (epi) {
        case EPI_STORE: G3_L(EPI_STORE); break;
        case EPI_BIAS: G3_L(EPI_BIAS); break;
        case EPI_BIAS_RELU: G3_L(EPI_BIAS_RELU); break;
        case EPI_ACCUM: G3_L(EPI_ACCUM); break;
        default: G3_L(EPI_SLAB); break;
    }
#undef G3_L
}

}  // namespace

namespace {

// gemm3w over the reduction split into ceil(K / kpw) slabs (summed by slab_sum_kernel), optionally with the column
// sums of A (db[m] = sum_k A[k][m]; per-slab partials in db_ws when there is more than one slab)
int wgrad_launch(int M, int N, int K, const float* A, long lda, const float* B, long ldb, float* C, long ldc,
                 int epilogue, int splits, float* workspace, float* db, float* db_ws, hipStream_t s) {
    const long wm_ = (M + w3::BM - 1) / w3::BM, wn_ = (N + w3::BN - 1) / w3::BN;
    int kpw = (K + splits - 1) / splits;
    kpw = (kpw + w3::KS - 1) / w3::KS * w3::KS;
    const int nzw = K == 0 ? 1 : (K + kpw - 1) / kpw;
    PDVC_CHECK_ARG(wm_ * wn_ * nzw < (1L << 31), "too many tiles");
    const dim3 gw((unsigned)(wm_ * wn_ * nzw));
    float* dw = nzw > 1 ? workspace : C;
    const long ldw = nzw > 1 ? N : ldc;
    const long slab_n = (long)M * N;
    float* cp = nzw > 1 ? db_ws : db;
    if (db != nullptr) {
        if (nzw > 1) hipLaunchKernelGGL((gemm3w_kernel<EPI_SLAB, true>), gw, dim3(NT), 0, s, M, N, K, A, lda, B, ldb, dw, ldw, kpw, (int)wn_, slab_n, nzw, cp);
        else hipLaunchKernelGGL((gemm3w_kernel<EPI_STORE, true>), gw, dim3(NT), 0, s, M, N, K, A, lda, B, ldb, dw, ldw, kpw, (int)wn_, slab_n, nzw, cp);
    } else {
        if (nzw > 1) hipLaunchKernelGGL(gemm3w_kernel<EPI_SLAB>, gw, dim3(NT), 0, s, M, N, K, A, lda, B, ldb, dw, ldw, kpw, (int)wn_, slab_n, nzw, nullptr);
        else hipLaunchKernelGGL(gemm3w_kernel<EPI_STORE>, gw, dim3(NT), 0, s, M, N, K, A, lda, B, ldb, dw, ldw, kpw, (int)wn_, slab_n, nzw, nullptr);
    }
    PDVC_CHECK_LAUNCH("gemm3w_kernel");
    if (nzw > 1) {  // dW's slabs, and db's partials in the same launch
        const long n4 = slab_n / 4, m4 = db != nullptr ? M / 4 : 0;
        const int blocks = (int)std::min<long>((n4 + m4 + 255) / 256, 2048);
        if (epilogue == 3) hipLaunchKernelGGL(slab_sum_kernel<true>, dim3(blocks), dim3(256), 0, s, workspace, nzw, n4, C, db_ws, m4, db);
        else hipLaunchKernelGGL(slab_sum_kernel<false>, dim3(blocks), dim3(256), 0, s, workspace, nzw, n4, C, db_ws, m4, db);
        PDVC_CHECK_LAUNCH("slab_sum_kernel");
    }
    return PDVC_OK;
}

}  // namespace

// C-ABI: see include/pdvc_msda.h ("fp32 GEMM on the bf16 matrix cores")
extern "C" int pdvc_gemm3_f32(int M, int N, int K, const float* A, long lda, int a_kc, const float* B, long ldb,
                              int b_kc, float* C, long ldc, const float* bias, int epilogue, int splits,
                              float* workspace, void* stream) {
    PDVC_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative sizes");
    PDVC_CHECK_ARG((a_kc == 0 || a_kc == 1) && (b_kc == 0 || b_kc == 1), "a_kc / b_kc must be 0 or 1");
    PDVC_CHECK_ARG(epilogue >= 0 && epilogue <= 3, "epilogue must be 0..3");
    PDVC_CHECK_ARG(epilogue != 1 && epilogue != 2 ? true : bias != nullptr, "bias epilogue needs a bias");
    PDVC_CHECK_ARG(splits >= 1 && (splits == 1 || (epilogue == 0 || epilogue == 3)), "splits > 1: store or accumulate only");
    PDVC_CHECK_ARG(splits == 1 || workspace != nullptr, "splits > 1 needs a workspace of splits * M * N floats");
    PDVC_CHECK_ARG(lda >= (a_kc ? K : M) && ldb >= (b_kc ? K : N) && ldc >= N, "leading dimensions too small");
    // float4 operand loads: 16-B aligned bases, leading dimensions and the contiguous extents multiples of 4
    PDVC_CHECK_ARG((uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0 && lda % 4 == 0 && ldb % 4 == 0,
                   "operands must be 16-byte aligned with leading dimensions divisible by 4");
    PDVC_CHECK_ARG(K % BK == 0, "K must be a multiple of 32");
    PDVC_CHECK_ARG((a_kc ? 4 : M) % 4 == 0 && (b_kc ? 4 : N) % 4 == 0 && (a_kc || M >= 4) && (b_kc || N >= 4),
                   "mn-contiguous operands need M (N) divisible by 4");
    PDVC_CHECK_ARG(splits == 1 || (ldc == N && N % 4 == 0 && (uintptr_t)C % 16 == 0),
                   "split reduction needs a dense, 16-byte aligned C with N divisible by 4");
    if (M == 0 || N == 0) return PDVC_OK;
    hipStream_t s = (hipStream_t)stream;
    constexpr int BM = 256, BN = 128;
    const long tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    PDVC_CHECK_ARG(tiles_m * tiles_n < (1L << 31), "too many tiles");
    int kps = (K + splits - 1) / splits;
    kps = (kps + BK - 1) / BK * BK;
    const int nz = K == 0 ? 1 : (K + kps - 1) / kps;
    PDVC_CHECK_ARG(nz <= 65535, "too many splits");
    const dim3 grid((unsigned)(tiles_m * tiles_n), 1, (unsigned)nz);
    const bool slab = nz > 1;
    float* dst = slab ? workspace : C;
    const long ld = slab ? N : ldc;
    const int epi = slab ? (int)EPI_SLAB : epilogue;
    const long slab_n = (long)M * N;
    if (!a_kc && !b_kc && (epi == EPI_STORE || epi == EPI_SLAB))  // the weight-gradient form: gemm3w's tile
        return wgrad_launch(M, N, K, A, lda, B, ldb, C, ldc, epilogue, splits, workspace, nullptr, nullptr, s);
    if (a_kc && b_kc) launch_epi<BM, BN, true, true>(epi, grid, s, M, N, K, A, lda, B, ldb, dst, ld, bias, kps, (int)tiles_n, slab_n);
    else if (a_kc) launch_epi<BM, BN, true, false>(epi, grid, s, M, N, K, A, lda, B, ldb, dst, ld, bias, kps, (int)tiles_n, slab_n);
    else if (b_kc) launch_epi<BM, BN, false, true>(epi, grid, s, M, N, K, A, lda, B, ldb, dst, ld, bias, kps, (int)tiles_n, slab_n);
    else launch_epi<BM, BN, false, false>(epi, grid, s, M, N, K, A, lda, B, ldb, dst, ld, bias, kps, (int)tiles_n, slab_n);
    PDVC_CHECK_LAUNCH("gemm3_kernel");
    if (slab) {
        const long n4 = slab_n / 4;
        const int blocks = (int)std::min<long>((n4 + 255) / 256, 2048);
        if (epilogue == 3) hipLaunchKernelGGL(slab_sum_kernel<true>, dim3(blocks), dim3(256), 0, s, workspace, nz, n4, C, nullptr, 0L, nullptr);
        else hipLaunchKernelGGL(slab_sum_kernel<false>, dim3(blocks), dim3(256), 0, s, workspace, nz, n4, C, nullptr, 0L, nullptr);
        PDVC_CHECK_LAUNCH("slab_sum_kernel");
    }
    return PDVC_OK;
}

// C-ABI: see include/pdvc_msda.h -- the weight gradient C = A^T B of pdvc_gemm3_f32 (a_kc = b_kc = 0, epilogue 0) and
// the bias gradient db = the column sums of A, from one pass over A
extern "C" int pdvc_gemm3_wgrad_bias_f32(int M, int N, int K, const float* A, long lda, const float* B, long ldb,
                                         float* C, long ldc, int epilogue, int splits, float* workspace, float* db,
                                         float* db_ws, void* stream) {
    PDVC_CHECK_ARG(M >= 4 && N >= 4 && K >= 0 && M % 4 == 0 && N % 4 == 0, "M, N: multiples of 4, at least 4");
    PDVC_CHECK_ARG(epilogue == 0, "epilogue must be 0 (store)");
    PDVC_CHECK_ARG(splits >= 1 && splits <= 65535, "splits out of range");
    PDVC_CHECK_ARG(lda >= M && ldb >= N && ldc >= N, "leading dimensions too small");
    PDVC_CHECK_ARG((uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0 && lda % 4 == 0 && ldb % 4 == 0,
                   "operands must be 16-byte aligned with leading dimensions divisible by 4");
    PDVC_CHECK_ARG(K % BK == 0, "K must be a multiple of 32");
    PDVC_CHECK_ARG(db != nullptr && (uintptr_t)db % 16 == 0, "db: a 16-byte aligned (M,) destination");
    PDVC_CHECK_ARG(splits == 1 || (workspace != nullptr && db_ws != nullptr && (uintptr_t)db_ws % 16 == 0 &&
                                   ldc == N && (uintptr_t)C % 16 == 0),
                   "splits > 1: a workspace of splits * M * N floats, a 16-byte aligned db_ws of splits * M floats "
                   "and a dense, 16-byte aligned C");
    return wgrad_launch(M, N, K, A, lda, B, ldb, C, ldc, epilogue, splits, workspace, db, db_ws, (hipStream_t)stream);
}

namespace {
int split_planes_impl(int np, const float* B, long ldb, int b_kc, int N, int K, uint16_t* planes, void* stream) {
    PDVC_CHECK_ARG(N > 0 && K > 0 && K % BK == 0, "N > 0 and K a positive multiple of 32");
    PDVC_CHECK_ARG(ldb >= (b_kc ? K : N), "leading dimension too small");
    PDVC_CHECK_ARG(!b_kc || ((uintptr_t)B % 16 == 0 && ldb % 4 == 0), "k-contiguous B: 16-byte aligned rows");
    PDVC_CHECK_ARG((uintptr_t)planes % 16 == 0, "planes must be 16-byte aligned");
    const long n4 = (long)N * (K / 4);
    const int blocks = (int)std::min<long>((n4 + 255) / 256, 4096);
    if (np == 1) hipLaunchKernelGGL(split_planes_kernel<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, B, ldb, b_kc, N, K, planes);
    else hipLaunchKernelGGL(split_planes_kernel<3>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, B, ldb, b_kc, N, K, planes);
    PDVC_CHECK_LAUNCH("split_planes_kernel");
    return PDVC_OK;
}

template <int NP>
int gemmp_impl(int M, int N, int K, const float* A, long lda, const uint16_t* planes, float* C, long ldc,
               const float* bias, int epilogue, void* stream, Drop drp = Drop{nullptr, 0u, 1.f, nullptr}) {
    PDVC_CHECK_ARG(M >= 0 && N > 0 && K >= 0 && K % BK == 0, "sizes: N > 0, K a multiple of 32");
    PDVC_CHECK_ARG((epilogue >= 0 && epilogue <= 3) || (epilogue == EPI_BIAS_RELU_DROP && drp.seed != nullptr) ||
                       ((epilogue == EPI_DMASK || epilogue == EPI_RESID_DROP) && drp.hd != nullptr),
                   "epilogue must be 0..3 (5, 6: through pdvc_gemm3p_relu_dropout_f32 / _dmask_f32)");
    PDVC_CHECK_ARG(epilogue == 0 || epilogue == 3 || epilogue == EPI_DMASK || bias != nullptr,
                   "bias epilogue needs a bias");
    PDVC_CHECK_ARG(lda >= K && ldc >= N, "leading dimensions too small");
    PDVC_CHECK_ARG((uintptr_t)A % 16 == 0 && lda % 4 == 0 && (uintptr_t)planes % 16 == 0,
                   "A rows and the planes must be 16-byte aligned");
    if (M == 0) return PDVC_OK;
    const long tiles_m = (M + p3::BM - 1) / p3::BM, tiles_n = (N + p3::BN - 1) / p3::BN;
    PDVC_CHECK_ARG(tiles_m * tiles_n < (1L << 31), "too many tiles");
    const dim3 grid((unsigned)(tiles_m * tiles_n));
    hipStream_t s = (hipStream_t)stream;
#define G3P_L(E) hipLaunchKernelGGL((gemm3p_kernel<E, NP>), grid, dim3(NT), 0, s, M, N, K, A, lda, planes, C, ldc, bias, (int)tiles_n, drp)
    switch (epilogue) {
        case 0: G3P_L(EPI_STORE); break;
        case 1: G3P_L(EPI_BIAS); break;
        case 2: G3P_L(EPI_BIAS_RELU); break;
        case 3: G3P_L(EPI_ACCUM); break;
        case EPI_BIAS_RELU_DROP:
            if constexpr (NP == 3) G3P_L(EPI_BIAS_RELU_DROP);
            break;
        case EPI_RESID_DROP:
            if constexpr (NP == 3) G3P_L(EPI_RESID_DROP);
            break;
        default:
            if constexpr (NP == 3) G3P_L(EPI_DMASK);
            break;
    }
#undef G3P_L
    PDVC_CHECK_LAUNCH("gemm3p_kernel");
    return PDVC_OK;
}
}  // namespace

// C-ABI: see include/pdvc_msda.h
extern "C" int pdvc_split3_planes_f32(const float* B, long ldb, int b_kc, int N, int K, uint16_t* planes,
                                      void* stream) {
    return split_planes_impl(3, B, ldb, b_kc, N, K, planes, stream);
}

extern "C" int pdvc_gemm3p_f32(int M, int N, int K, const float* A, long lda, const uint16_t* planes, float* C,
                               long ldc, const float* bias, int epilogue, void* stream) {
    return gemmp_impl<3>(M, N, K, A, lda, planes, C, ldc, bias, epilogue, stream);
}

// linear1 of the feed-forward block with its relu -> dropout in the epilogue (C = dropout(relu(A opB^T + bias)), the
// keep mask of pdvc_relu_dropout_forward_f32 for element (row, col) of C and the same seed: bit-identical to the GEMM
// followed by that pass)
extern "C" int pdvc_gemm3p_relu_dropout_f32(int M, int N, int K, const float* A, long lda, const uint16_t* planes,
                                            float* C, long ldc, const float* bias, float p, const uint64_t* seed_dev,
                                            void* stream) {
    PDVC_CHECK_ARG(p > 0.f && p < 1.f, "dropout p must be in (0, 1) (p = 0: the bias + ReLU epilogue)");
    PDVC_CHECK_ARG(seed_dev != nullptr && bias != nullptr, "a device seed and a bias are required");
    const Drop drp{seed_dev, ffn_threshold(p), 1.f / (1.f - p), nullptr};
    return gemmp_impl<3>(M, N, K, A, lda, planes, C, ldc, bias, EPI_BIAS_RELU_DROP, stream, drp);
}

// the feed-forward block's backward through relu -> dropout in the data gradient of linear2's input: C = hd > 0 ?
// (A opB^T) / (1 - p) : 0 with hd the forward's output (C's shape and ldc) -- pdvc_relu_dropout_backward_f32's
// arithmetic on the GEMM's result, without its pass over the (rows x d_ffn) gradient
extern "C" int pdvc_gemm3p_dmask_f32(int M, int N, int K, const float* A, long lda, const uint16_t* planes, float* C,
                                     long ldc, const float* hd, float p, void* stream) {
    PDVC_CHECK_ARG(p >= 0.f && p < 1.f && hd != nullptr, "dropout p in [0, 1) and the forward output required");
    const Drop drp{nullptr, 0u, p > 0.f ? 1.f / (1.f - p) : 1.f, hd};
    return gemmp_impl<3>(M, N, K, A, lda, planes, C, ldc, nullptr, EPI_DMASK, stream, drp);
}

// the residual sub-layer's sum before its LayerNorm: C = R + dropout(A opB^T + bias) with the keep mask of
// pdvc_add_dropout_layernorm_forward_f32 (an_hash.h) for element (row, col) of C and the same seed (p = 0: no
// dropout, seed_dev may be NULL); R has C's shape and ldc.  The add-norm pass then reads C alone (s = NULL): its
// forward and backward are those of the unfused pair, bit for bit
extern "C" int pdvc_gemm3p_resid_dropout_f32(int M, int N, int K, const float* A, long lda, const uint16_t* planes,
                                             float* C, long ldc, const float* bias, const float* R, float p,
                                             const uint64_t* seed_dev, void* stream) {
    PDVC_CHECK_ARG(p >= 0.f && p < 1.f, "dropout p must be in [0, 1)");
    PDVC_CHECK_ARG(p == 0.f || seed_dev != nullptr, "p > 0 needs a device seed");
    PDVC_CHECK_ARG(bias != nullptr && R != nullptr, "a bias and the residual R are required");
    const Drop drp{p > 0.f ? seed_dev : nullptr, an_threshold(p), p > 0.f ? 1.f / (1.f - p) : 1.f, R};
    return gemmp_impl<3>(M, N, K, A, lda, planes, C, ldc, bias, EPI_RESID_DROP, stream, drp);
}

// the bf16 mode's product: opB rounded to bf16 (one plane), A rounded in the kernel, one MFMA term, fp32 result
extern "C" int pdvc_round_plane_f32(const float* B, long ldb, int b_kc, int N, int K, uint16_t* plane, void* stream) {
    return split_planes_impl(1, B, ldb, b_kc, N, K, plane, stream);
}

extern "C" int pdvc_gemm1p_f32(int M, int N, int K, const float* A, long lda, const uint16_t* plane, float* C,
                               long ldc, const float* bias, int epilogue, void* stream) {
    return gemmp_impl<1>(M, N, K, A, lda, plane, C, ldc, bias, epilogue, stream);
}

