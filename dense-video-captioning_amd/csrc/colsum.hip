// colsum.hip -- column sums of a row-major fp32 matrix: the bias gradients of the projection layers
// (db = sum over rows of dY; nn.Linear's backward in every MSDeformAttn / FFN / MHA layer of the step,
// pdvc/ops/modules/ms_deform_attn.py:55-58, pdvc/deformable_transformer.py:162-165,236-240).
//
// torch's generic reduction reads dY (30720 x 512, 63 MB) at ~2.2 TB/s and a 3200 x 512 decoder gradient in
// ~18 us.  Here pass 1 splits the rows into `parts` slabs (enough workgroups to fill the chip); a workgroup sums
// one slab for 64 consecutive columns (16 lanes own one float4 column group each and 16 row lanes take
// interleaved rows: a wave-instruction reads 4 rows x 256 B) and writes one partial row; pass 2 adds the
// `parts` (<= 256) partial rows over 16 lanes per column group.  Deterministic (fixed order), no atomics, no memset.  HBM-bound: rows*cols*4 bytes read.
#include "pdvc_common.h"

namespace pdvc {

__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ x, int rows, int cols, int parts,
                                                          float* __restrict__ part) {
    __shared__ float4 red[16][16];
    const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;  // float4 column group, row lane
    const int c4 = blockIdx.x * 16 + cg;
    const int p = blockIdx.y;
    const int r0 = (int)(((long)rows * p) / parts), r1 = (int)(((long)rows * (p + 1)) / parts);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    const int cs = cols / 4;
    if (c4 < cs) {
        const float4* src = reinterpret_cast<const float4*>(x) + c4;
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
        reinterpret_cast<float4*>(part + (size_t)p * cols)[c4] = t;
    }
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int parts, int cols,
                                                           float* __restrict__ out) {
    // 16 float4 column groups x 16 lanes over the partial rows, then a fixed-order LDS sum: deterministic
    __shared__ float4 red[16][16];
    const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int c4 = blockIdx.x * 16 + cg, cs = cols / 4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < cs) {
        const float4* src = reinterpret_cast<const float4*>(part) + c4;
        for (int p = rl; p < parts; p += 16) {
            const float4 v = src[(size_t)p * cs];
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
        reinterpret_cast<float4*>(out)[c4] = t;
    }
}

}  // namespace pdvc

using namespace pdvc;

extern "C" int pdvc_colsum_f32(const float* x, int rows, int cols, int parts, float* workspace, float* out,
                               void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && cols > 0 && parts >= 1, "invalid sizes");
    PDVC_CHECK_ARG(cols % 4 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)workspace % 16) == 0 &&
                       ((uintptr_t)out % 16) == 0,
                   "colsum needs 16-byte aligned rows (cols %% 4 == 0)");
    hipStream_t s = (hipStream_t)stream;
    const unsigned cb = (unsigned)((cols / 4 + 15) / 16);
    hipLaunchKernelGGL(colsum_part_kernel, dim3(cb, (unsigned)parts), dim3(256), 0, s, x, rows, cols, parts, workspace);
    PDVC_CHECK_LAUNCH("colsum_part_kernel");
    hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)((cols / 4 + 15) / 16)), dim3(256), 0, s, workspace, parts,
                       cols, out);
    PDVC_CHECK_LAUNCH("colsum_final_kernel");
    return PDVC_OK;
}
