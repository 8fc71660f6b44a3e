// ffn.hip -- the element-wise middle of the transformer feed-forward block, relu -> dropout, both ways
// (reference: DeformableTransformerEncoderLayer.forward_ffn, deformable_transformer.py:140-145, and the decoder's,
// :233-237: linear2(dropout(relu(linear1(x))))).
//
// Forward: one in-place pass over linear1's output h (rows x cols): h_d = relu(h) * keep / (1 - p), the keep mask a
// counter hash of (seed, row, column) -- torch's relu_ + fused_dropout were two passes plus a byte mask.
// Backward needs no mask and no hash: h_d > 0 exactly where relu passed AND dropout kept, so
//     dh = (h_d > 0) ? dh_d / (1 - p) : 0
// in one pass over (dh_d, h_d), in place, which also sums the columns of dh (linear1's bias gradient) into
// per-slab partial rows (the layout of colsum.hip) -- torch's masked_scale + threshold_backward + sum were three.
// HBM-bound: forward 8 bytes / element, backward 12 bytes / element.
#include "ffn_hash.h"
#include "pdvc_common.h"

namespace pdvc {

__global__ __launch_bounds__(256) void relu_dropout_fwd_kernel(float* __restrict__ h, long rows, int cols, float p,
                                                               uint32_t thresh, float scale, uint64_t seed0,
                                                               const uint64_t* __restrict__ seed_dev,
                                                               uint16_t* __restrict__ h16) {
    const uint64_t seed = seed_dev ? *seed_dev : seed0;
    const int c4 = cols / 4;
    const long n4 = rows * c4;
    float4* h4 = reinterpret_cast<float4*>(h);
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const uint32_t row = (uint32_t)(i / c4), col = (uint32_t)(i - (long)row * c4) * 4;
        float4 v = h4[i];
        float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float x = fmaxf(e[k], 0.f);
            if (p > 0.f) x = ffn_keep(seed, row, col + k, thresh) ? x * scale : 0.f;
            e[k] = x;
        }
        h4[i] = make_float4(e[0], e[1], e[2], e[3]);
        if (h16) store_bf16x4(h16 + (size_t)i * 4, e[0], e[1], e[2], e[3]);
    }
}

// grid (ceil(cols/64), parts): 16 float4 column groups x 16 row lanes over one row slab
__global__ __launch_bounds__(256) void relu_dropout_bwd_kernel(const float* __restrict__ hd, float* __restrict__ g,
                                                               int rows, int cols, int parts, float scale,
                                                               float* __restrict__ part,
                                                               uint16_t* __restrict__ g16) {
    __shared__ float4 red[16][16];
    const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const int c4 = blockIdx.x * 16 + cg;
    const int p = blockIdx.y;
    const int r0 = (int)(((long)rows * p) / parts), r1 = (int)(((long)rows * (p + 1)) / parts);
    const int cs = cols / 4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < cs) {
        const float4* h4 = reinterpret_cast<const float4*>(hd) + c4;
        float4* g4 = reinterpret_cast<float4*>(g) + c4;
#pragma unroll 4
        for (int r = r0 + rl; r < r1; r += 16) {
            const size_t o = (size_t)r * cs;
            const float4 x = h4[o];
            float4 d = g4[o];
            d.x = x.x > 0.f ? d.x * scale : 0.f;
            d.y = x.y > 0.f ? d.y * scale : 0.f;
            d.z = x.z > 0.f ? d.z * scale : 0.f;
            d.w = x.w > 0.f ? d.w * scale : 0.f;
            g4[o] = d;
            if (g16) store_bf16x4(g16 + ((size_t)r * cs + c4) * 4, d.x, d.y, d.z, d.w);
            a.x += d.x;
            a.y += d.y;
            a.z += d.z;
            a.w += d.w;
        }
    }
    if (part == nullptr) return;  // block-uniform
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

__global__ __launch_bounds__(256) void ffn_colsum_final_kernel(const float* __restrict__ part, int parts, int cols,
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

static int relu_dropout_forward(float* h, long rows, int cols, float p, uint64_t seed, const uint64_t* seed_dev,
                                uint16_t* h16, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && cols > 0 && cols % 4 == 0 && ((uintptr_t)h % 16) == 0,
                   "relu_dropout needs 16-byte aligned rows (cols %% 4 == 0)");
    PDVC_CHECK_ARG(rows <= 0xffffffffL, "too many rows");
    PDVC_CHECK_ARG(p >= 0.f && p < 1.f, "dropout p must be in [0,1)");
    const long n4 = rows * (cols / 4);
    if (n4 == 0) return PDVC_OK;
    const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
    const long want = (n4 + 255) / 256;
    const unsigned blocks = (unsigned)(want < 8192 ? want : 8192);
    hipLaunchKernelGGL(relu_dropout_fwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, h, rows, cols, p,
                       ffn_threshold(p), scale, seed, seed_dev, h16);
    PDVC_CHECK_LAUNCH("relu_dropout_fwd_kernel");
    return PDVC_OK;
}

static int relu_dropout_backward(const float* hd, float* grad, int rows, int cols, float p, int parts,
                                 float* workspace, float* dbias, uint16_t* g16, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && cols > 0 && cols % 4 == 0 && parts >= 1, "invalid sizes");
    PDVC_CHECK_ARG(((uintptr_t)hd % 16) == 0 && ((uintptr_t)grad % 16) == 0, "16-byte aligned rows required");
    PDVC_CHECK_ARG((dbias == nullptr) == (workspace == nullptr), "dbias needs a workspace of parts*cols floats");
    PDVC_CHECK_ARG(workspace == nullptr || (((uintptr_t)workspace % 16) == 0 && ((uintptr_t)dbias % 16) == 0),
                   "workspace and dbias must be 16-byte aligned");
    PDVC_CHECK_ARG(p >= 0.f && p < 1.f, "dropout p must be in [0,1)");
    hipStream_t s = (hipStream_t)stream;
    const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
    const unsigned cb = (unsigned)((cols / 4 + 15) / 16);
    hipLaunchKernelGGL(relu_dropout_bwd_kernel, dim3(cb, (unsigned)parts), dim3(256), 0, s, hd, grad, rows, cols,
                       parts, scale, workspace, g16);
    PDVC_CHECK_LAUNCH("relu_dropout_bwd_kernel");
    if (dbias) {
        hipLaunchKernelGGL(ffn_colsum_final_kernel, dim3((unsigned)((cols / 4 + 15) / 16)), dim3(256), 0, s, workspace,
                           parts, cols, dbias);
        PDVC_CHECK_LAUNCH("ffn_colsum_final_kernel");
    }
    return PDVC_OK;
}

extern "C" int pdvc_relu_dropout_forward_f32(float* h, long rows, int cols, float p, uint64_t seed,
                                             const uint64_t* seed_dev, void* stream) {
    return relu_dropout_forward(h, rows, cols, p, seed, seed_dev, nullptr, stream);
}

extern "C" int pdvc_relu_dropout_backward_f32(const float* hd, float* grad, int rows, int cols, float p, int parts,
                                              float* workspace, float* dbias, void* stream) {
    return relu_dropout_backward(hd, grad, rows, cols, p, parts, workspace, dbias, nullptr, stream);
}

// The bf16 mode's forms (pdvc/precision.py): the same passes, also writing the bf16 rounding of the result (h / dh,
// the next GEMM's operand) into h16 / g16.
extern "C" int pdvc_relu_dropout_forward_f32_bf16out(float* h, long rows, int cols, float p, uint64_t seed,
                                                     const uint64_t* seed_dev, uint16_t* h16, void* stream) {
    PDVC_CHECK_ARG(h16 != nullptr && ((uintptr_t)h16 % 8) == 0, "h16 must be an 8-byte aligned bf16 buffer");
    return relu_dropout_forward(h, rows, cols, p, seed, seed_dev, h16, stream);
}

extern "C" int pdvc_relu_dropout_backward_f32_bf16out(const float* hd, float* grad, int rows, int cols, float p,
                                                      int parts, float* workspace, float* dbias, uint16_t* g16,
                                                      void* stream) {
    PDVC_CHECK_ARG(g16 != nullptr && ((uintptr_t)g16 % 8) == 0, "g16 must be an 8-byte aligned bf16 buffer");
    return relu_dropout_backward(hd, grad, rows, cols, p, parts, workspace, dbias, g16, stream);
}
