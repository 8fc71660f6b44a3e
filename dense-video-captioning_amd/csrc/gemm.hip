// gemm.hip -- fp32 GEMM on the gfx950 f32-input matrix cores (v_mfma_f32_32x32x2_f32), exact f32.
//
// The dense projections of the PDVC step (value/offset/output projections and FFN of the transformer over
// N*S = 30720 rows, their data- and weight-gradients, the caption head's projections) in fp32 -- gfx950 has
// no xf32/TF32 path, so the f32-input MFMA at 64 FLOP/clk/SIMD (157 TF/s dense) is the ceiling.
//
//   C[M,N] (=|+=) op(A)[M,K] . op(B)[K,N] (+ bias[N]) (ReLU)
//   op(A): TA = 0 -> A[m*lda + k] (k contiguous), TA = 1 -> A[k*lda + m] (m contiguous)
//   op(B): TB = 0 -> B[k*ldb + n] (n contiguous), TB = 1 -> B[n*ldb + k] (k contiguous)
//
// Tiling: a 256-thread workgroup computes a 128x128 tile, each wave a 64x64 quarter as 2x2 MFMA 32x32
// blocks; K advances in 32-deep slices staged through LDS images [k][mn] (mn contiguous, +4 pad), double
// buffered with the next slice prefetched into registers while the current one feeds the MFMAs.  Fragments
// are single ds_read_b32 per operand per MFMA (lane l reads [k = 2s + l/32][mn = l%32], consecutive lanes on
// consecutive banks); an fp32 MFMA takes 16 cycles per CU, so LDS traffic is far from the bound.
// Operands that are k-contiguous in HBM are transposed on their way into LDS (4 ds_write_b32 per float4).
// Split-K (gridDim.z > 1) accumulates with float atomics: every atomic wave-instruction covers two 128-B
// row segments (the full-rate shape, MI355X_MICROARCH.md "Global float atomics"); the caller zeroes C.
#include "pdvc_common.h"

namespace pdvc {

constexpr int GT = 128;        // tile edge (M and N)
constexpr int GK = 32;         // K slice
constexpr int GLD = GT + 4;    // LDS row stride (floats)
constexpr int GIMG = GK * GLD; // one operand image

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_RELU = 2, EPI_ATOMIC = 3 };

// Loads one operand's 128 x 32 slice into 4 float4 registers per thread (zero outside the matrix).
// KC = true: k contiguous in HBM (rows are mn), else mn contiguous (rows are k).
template <bool KC>
__device__ __forceinline__ void g_load(float4 (&r)[4], const float* __restrict__ P, int ld, int mn0, int k0,
                                       int MN, int K, bool vec) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int mn, k;
        if (KC) {
            mn = t / 8 + 32 * i;
            k = (t % 8) * 4;
        } else {
            k = t / 32 + 8 * i;
            mn = (t % 32) * 4;
        }
        const int gm = mn0 + mn, gk = k0 + k;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (KC) {
            if (gm < MN) {
                const float* p = P + (size_t)gm * ld + gk;
                if (vec && gk + 3 < K) v = *reinterpret_cast<const float4*>(p);
                else {
                    if (gk < K) v.x = p[0];
                    if (gk + 1 < K) v.y = p[1];
                    if (gk + 2 < K) v.z = p[2];
                    if (gk + 3 < K) v.w = p[3];
                }
            }
        } else {
            if (gk < K) {
                const float* p = P + (size_t)gk * ld + gm;
                if (vec && gm + 3 < MN) v = *reinterpret_cast<const float4*>(p);
                else {
                    if (gm < MN) v.x = p[0];
                    if (gm + 1 < MN) v.y = p[1];
                    if (gm + 2 < MN) v.z = p[2];
                    if (gm + 3 < MN) v.w = p[3];
                }
            }
        }
        r[i] = v;
    }
}

template <bool KC>
__device__ __forceinline__ void s_store(const float4 (&r)[4], float* __restrict__ img) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (KC) {
            const int mn = t / 8 + 32 * i, k = (t % 8) * 4;
            img[(k + 0) * GLD + mn] = r[i].x;
            img[(k + 1) * GLD + mn] = r[i].y;
            img[(k + 2) * GLD + mn] = r[i].z;
            img[(k + 3) * GLD + mn] = r[i].w;
        } else {
            const int k = t / 32 + 8 * i, mn = (t % 32) * 4;
            *reinterpret_cast<float4*>(img + k * GLD + mn) = r[i];
        }
    }
}

template <int TA, int TB, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(int M, int N, int K, const float* __restrict__ A, int lda,
                                                          const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                          int ldc, const float* __restrict__ bias, int k_per_split,
                                                          int tiles_n, int vecA, int vecB) {
    __shared__ __attribute__((aligned(16))) float lds[2 * 2 * GIMG];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int tiles = gridDim.x;
    const int tile = xcd_remap(blockIdx.x, tiles);  // consecutive tiles (same A rows) share an XCD's L2
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int m0 = tm * GT, n0 = tn * GT;
    const int kb = blockIdx.z * k_per_split;
    const int ke = min(K, kb + k_per_split);
    const int nslices = (ke - kb + GK - 1) / GK;
    const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
    const int l32 = lane & 31, h = lane >> 5;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 ra[4], rb[4];
    g_load<TA == 0>(ra, A, lda, m0, kb, M, ke, vecA);
    g_load<TB == 1>(rb, B, ldb, n0, kb, N, ke, vecB);
    s_store<TA == 0>(ra, lds);
    s_store<TB == 1>(rb, lds + GIMG);
    __syncthreads();
    for (int s = 0; s < nslices; ++s) {
        const float* As = lds + (s & 1) * 2 * GIMG;
        const float* Bs = As + GIMG;
        const bool more = s + 1 < nslices;
        if (more) {
            g_load<TA == 0>(ra, A, lda, m0, kb + (s + 1) * GK, M, ke, vecA);
            g_load<TB == 1>(rb, B, ldb, n0, kb + (s + 1) * GK, N, ke, vecB);
        }
#pragma unroll
        for (int kk = 0; kk < GK / 2; ++kk) {
            const int row = (2 * kk + h) * GLD;
            const float a0 = As[row + wm + l32], a1 = As[row + wm + 32 + l32];
            const float b0 = Bs[row + wn + l32], b1 = Bs[row + wn + 32 + l32];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (more) {
            float* nxt = lds + ((s + 1) & 1) * 2 * GIMG;
            s_store<TA == 0>(ra, nxt);
            s_store<TB == 1>(rb, nxt + GIMG);
        }
        __syncthreads();
    }

    // epilogue: acc[i][j] register r of lane l is C[row][col], col = l%32, row = (r&3) + 8*(r>>2) + 4*(l/32)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn + 32 * j + l32;
        if (col >= N) continue;
        const float bv = (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (row < M) {
                    float v = acc[i][j][r] + bv;
                    if (EPI == EPI_BIAS_RELU) v = fmaxf(v, 0.f);
                    float* p = C + (size_t)row * ldc + col;
                    if (EPI == EPI_ATOMIC) atomicAdd(p, v);
                    else *p = v;
                }
            }
        }
    }
}

}  // namespace pdvc

using namespace pdvc;

#define GEMM_LAUNCH(TA_, TB_, EPI_)                                                                              \
    hipLaunchKernelGGL((gemm_f32_kernel<TA_, TB_, EPI_>), grid, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc, \
                       bias, kps, tiles_n, vecA, vecB)

template <int EPI_>
static void gemm_dispatch(int ta, int tb, dim3 grid, hipStream_t s, int M, int N, int K, const float* A, int lda,
                          const float* B, int ldb, float* C, int ldc, const float* bias, int kps, int tiles_n,
                          int vecA, int vecB) {
    if (ta == 0 && tb == 0) GEMM_LAUNCH(0, 0, EPI_);
    else if (ta == 0 && tb == 1) GEMM_LAUNCH(0, 1, EPI_);
    else if (ta == 1 && tb == 0) GEMM_LAUNCH(1, 0, EPI_);
    else GEMM_LAUNCH(1, 1, EPI_);
}

extern "C" int pdvc_gemm_f32(int M, int N, int K, const float* A, int lda, int trans_a, const float* B, int ldb,
                             int trans_b, float* C, int ldc, const float* bias, int epilogue, int split_k,
                             void* stream) {
    PDVC_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative sizes");
    PDVC_CHECK_ARG(trans_a == 0 || trans_a == 1, "trans_a must be 0 or 1");
    PDVC_CHECK_ARG(trans_b == 0 || trans_b == 1, "trans_b must be 0 or 1");
    PDVC_CHECK_ARG(epilogue >= 0 && epilogue <= 3, "epilogue must be 0..3");
    PDVC_CHECK_ARG(epilogue == 0 || epilogue == 3 || bias != nullptr, "bias epilogue needs a bias");
    PDVC_CHECK_ARG(split_k >= 1 && (split_k == 1 || epilogue == 3), "split_k > 1 needs the atomic epilogue");
    PDVC_CHECK_ARG(lda >= (trans_a ? M : K) && ldb >= (trans_b ? K : N) && ldc >= N, "leading dimensions too small");
    if (M == 0 || N == 0) return PDVC_OK;
    hipStream_t s = (hipStream_t)stream;
    if (K == 0) {
        if (epilogue == 3) return PDVC_OK;
        return pdvc_set_error(PDVC_ERR_UNSUPPORTED, "K == 0 with a storing epilogue");
    }
    const int tiles_m = (M + GT - 1) / GT, tiles_n = (N + GT - 1) / GT;
    const long tiles = (long)tiles_m * tiles_n;
    PDVC_CHECK_ARG(tiles < (1L << 31), "too many tiles");
    int kps = (K + split_k - 1) / split_k;
    kps = (kps + GK - 1) / GK * GK;
    const int splits = (K + kps - 1) / kps;
    // float4 loads need 16-B aligned rows
    const int vecA = ((uintptr_t)A % 16 == 0) && (lda % 4 == 0);
    const int vecB = ((uintptr_t)B % 16 == 0) && (ldb % 4 == 0);
    dim3 grid((unsigned)tiles, 1, (unsigned)splits);
    switch (epilogue) {
        case 0: gemm_dispatch<EPI_STORE>(trans_a, trans_b, grid, s, M, N, K, A, lda, B, ldb, C, ldc, bias, kps, tiles_n, vecA, vecB); break;
        case 1: gemm_dispatch<EPI_BIAS>(trans_a, trans_b, grid, s, M, N, K, A, lda, B, ldb, C, ldc, bias, kps, tiles_n, vecA, vecB); break;
        case 2: gemm_dispatch<EPI_BIAS_RELU>(trans_a, trans_b, grid, s, M, N, K, A, lda, B, ldb, C, ldc, bias, kps, tiles_n, vecA, vecB); break;
        default: gemm_dispatch<EPI_ATOMIC>(trans_a, trans_b, grid, s, M, N, K, A, lda, B, ldb, C, ldc, bias, kps, tiles_n, vecA, vecB); break;
    }
    PDVC_CHECK_LAUNCH("gemm_f32_kernel");
    return PDVC_OK;
}
