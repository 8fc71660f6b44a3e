// msda_op.hip -- the drop-in MultiScaleDeformableAttention operator for MI355X (general 2-D pyramids).
//
// Semantics: the reference CUDA op (zero padding), pdvc/ops/src/cuda/ms_deform_im2col_cuda.cuh
//   forward  :238-300 (+ bilinear :34-85), backward :88-160 reduced over channels (:407-511),
// and the raw-sample (return_value=True) mode of ms_deform_attn_core_pytorch
//   (pdvc/ops/functions/ms_deform_attn_func.py:41-68) in both paddings (grid_sample border semantics).
//
// MI355X design: one wave64 per (batch, query, head) -- the lanes stride over the head's channels, so a
// corner read is one coalesced D*sizeof(T) row segment, the per-sample channel reductions of the
// backward are wave butterflies (no LDS, no __syncthreads), and the grid is N*Lq*M waves instead of the
// reference's N*Lq*M*D/1024 blocks (480 blocks of 1024 threads at PDVC's encoder shape).  The whole batch
// is one launch (no im2col_step chunk loop: 288 GB of HBM makes chunking pointless).  This general path
// keeps atomics for grad_value; PDVC's modules use the fused 1-D kernels in msda1d.hip instead.
#include <algorithm>

#include "pdvc_common.h"

namespace pdvc {

// the drop-in operator's 1-D fast path (msda1d.hip)
bool dropin1d_applies(int S, int M, int D, int L, int Lq, int P);
int dropin1d_forward(const float* value, const int64_t* shapes, const int64_t* lsi, const float* loc,
                     const float* attn, int N, int S, int M, int Lq, float* out, hipStream_t s);
int dropin1d_backward(const float* value, const int64_t* shapes, const int64_t* lsi, const float* loc,
                      const float* attn, const float* gout, int N, int S, int M, int Lq, float* grad_value,
                      float* grad_loc, float* grad_attn, float* workspace, hipStream_t s);

constexpr int kMaxLevels2d = 64;

template <typename T>
struct Corner {
    T val, dw, dh;       // value, d(value)/d(loc_w), d(value)/d(loc_h) (loc units)
    T cw[4];             // corner weights
    int ci[4];           // corner flat index within the level (-1 = outside)
};

template <typename T, int PAD>
__device__ __forceinline__ void sample2d(const T* __restrict__ vb, int H, int W, int MD, int mc, T loc_w,
                                         T loc_h, Corner<T>& r) {
    r.val = 0; r.dw = 0; r.dh = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) { r.cw[k] = 0; r.ci[k] = -1; }
    if (PAD == PDVC_PAD_ZEROS) {
        // h_im = loc_h * H - 0.5 (.cuh:283-284); the double literal is rounded back to T
        const T h_im = (T)((double)(loc_h * (T)H) - 0.5);
        const T w_im = (T)((double)(loc_w * (T)W) - 0.5);
        if (!(h_im > (T)-1 && w_im > (T)-1 && h_im < (T)H && w_im < (T)W)) return;
        const int h_low = (int)floor(h_im), w_low = (int)floor(w_im);
        const int h_high = h_low + 1, w_high = w_low + 1;
        const T lh = h_im - (T)h_low, lw = w_im - (T)w_low;
        const T hh = (T)1 - lh, hw = (T)1 - lw;
        T v1 = 0, v2 = 0, v3 = 0, v4 = 0, gh = 0, gw = 0;
        if (h_low >= 0 && w_low >= 0) { r.ci[0] = h_low * W + w_low; v1 = vb[(size_t)r.ci[0] * MD + mc]; gh -= hw * v1; gw -= hh * v1; }
        if (h_low >= 0 && w_high <= W - 1) { r.ci[1] = h_low * W + w_high; v2 = vb[(size_t)r.ci[1] * MD + mc]; gh -= lw * v2; gw += hh * v2; }
        if (h_high <= H - 1 && w_low >= 0) { r.ci[2] = h_high * W + w_low; v3 = vb[(size_t)r.ci[2] * MD + mc]; gh += hw * v3; gw -= lh * v3; }
        if (h_high <= H - 1 && w_high <= W - 1) { r.ci[3] = h_high * W + w_high; v4 = vb[(size_t)r.ci[3] * MD + mc]; gh += lw * v4; gw += lh * v4; }
        r.cw[0] = hh * hw; r.cw[1] = hh * lw; r.cw[2] = lh * hw; r.cw[3] = lh * lw;
        r.val = (r.cw[0] * v1 + r.cw[1] * v2 + r.cw[2] * v3 + r.cw[3] * v4);
        r.dw = (T)W * gw;
        r.dh = (T)H * gh;
    } else {
        // grid_sampler_2d, bilinear, border, align_corners=False, on grid = 2*loc - 1
        T gmx = (T)W / (T)2, gmy = (T)H / (T)2;
        T ix = (((T)2 * loc_w - (T)1) + (T)1) * (T)W;
        ix = (ix - (T)1) / (T)2;
        T iy = (((T)2 * loc_h - (T)1) + (T)1) * (T)H;
        iy = (iy - (T)1) / (T)2;
        if (ix <= (T)0) { ix = 0; gmx = 0; } else if (ix >= (T)(W - 1)) { ix = (T)(W - 1); gmx = 0; }
        if (iy <= (T)0) { iy = 0; gmy = 0; } else if (iy >= (T)(H - 1)) { iy = (T)(H - 1); gmy = 0; }
        const int x0 = (int)floor(ix), y0 = (int)floor(iy);
        const T nw = ((T)(x0 + 1) - ix) * ((T)(y0 + 1) - iy);
        const T ne = (ix - (T)x0) * ((T)(y0 + 1) - iy);
        const T sw = ((T)(x0 + 1) - ix) * (iy - (T)y0);
        const T se = (ix - (T)x0) * (iy - (T)y0);
        T vnw = 0, vne = 0, vsw = 0, vse = 0;
        const bool x0in = x0 >= 0 && x0 < W, x1in = x0 + 1 >= 0 && x0 + 1 < W;
        const bool y0in = y0 >= 0 && y0 < H, y1in = y0 + 1 >= 0 && y0 + 1 < H;
        if (y0in && x0in) { r.ci[0] = y0 * W + x0; vnw = vb[(size_t)r.ci[0] * MD + mc]; }
        if (y0in && x1in) { r.ci[1] = y0 * W + x0 + 1; vne = vb[(size_t)r.ci[1] * MD + mc]; }
        if (y1in && x0in) { r.ci[2] = (y0 + 1) * W + x0; vsw = vb[(size_t)r.ci[2] * MD + mc]; }
        if (y1in && x1in) { r.ci[3] = (y0 + 1) * W + x0 + 1; vse = vb[(size_t)r.ci[3] * MD + mc]; }
        r.cw[0] = nw; r.cw[1] = ne; r.cw[2] = sw; r.cw[3] = se;
        r.val = vnw * nw + vne * ne + vsw * sw + vse * se;
        const T gix = -vnw * ((T)(y0 + 1) - iy) + vne * ((T)(y0 + 1) - iy) - vsw * (iy - (T)y0) + vse * (iy - (T)y0);
        const T giy = -vnw * ((T)(x0 + 1) - ix) - vne * (ix - (T)x0) + vsw * ((T)(x0 + 1) - ix) + vse * (ix - (T)x0);
        r.dw = (T)2 * gmx * gix;
        r.dh = (T)2 * gmy * giy;
    }
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, PDVC_WAVE);
    return v;
}

// The level table lives in device memory, so the host cannot check it without a sync.  A level whose rows
// fall outside [0, S) (a malformed table; the reference reads out of bounds there) is given H = W = 0: it
// contributes no samples, and no value row outside the tensor is ever read.
__device__ __forceinline__ void load_levels(const int64_t* __restrict__ shapes, const int64_t* __restrict__ lsi,
                                            int L, int S, int* sH, int* sW, int* sStart) {
    for (int i = threadIdx.x; i < L; i += blockDim.x) {
        const int64_t h = shapes[2 * i], w = shapes[2 * i + 1], st = lsi[i];
        const bool ok = h >= 0 && w >= 0 && st >= 0 && st + h * w <= (int64_t)S;
        sH[i] = ok ? (int)h : 0;
        sW[i] = ok ? (int)w : 0;
        sStart[i] = ok ? (int)st : 0;
    }
    __syncthreads();
}

// MODE 0: weighted reduction -> out (N,Lq,M,D);  MODE 1: raw samples -> out (N*M,D,Lq,L,P)
template <typename T, int PAD, int MODE>
__global__ __launch_bounds__(256) void msda2d_fwd_kernel(const T* __restrict__ value, const int64_t* __restrict__ shapes,
                                                          const int64_t* __restrict__ lsi, const T* __restrict__ loc,
                                                          const T* __restrict__ attn, int N, int S, int M, int D, int L,
                                                          int Lq, int P, int gate_1d, T* __restrict__ out) {
    if (gate_1d) {  // a lifted 1-D pyramid is the drop-in fast path's (msda_dropin_fwd_kernel)
        Levels1d lv;
        if (dropin_levels(shapes, lsi, S, lv)) return;
    }
    __shared__ int sH[kMaxLevels2d], sW[kMaxLevels2d], sStart[kMaxLevels2d];
    load_levels(shapes, lsi, L, S, sH, sW, sStart);
    const int lane = threadIdx.x & 63;
    const long nwaves = (long)gridDim.x * (blockDim.x >> 6);
    for (long wave = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); wave < (long)N * Lq * M;
         wave += nwaves) {
    const int m = (int)(wave % M);
    const int q = (int)((wave / M) % Lq);
    const int n = (int)(wave / ((long)M * Lq));
    const int MD = M * D;
    const long sbase = (long)wave * L * P;  // sample index of (n,q,m,0,0)
    for (int c = lane; c < D; c += PDVC_WAVE) {
        T col = 0;
        for (int l = 0; l < L; ++l) {
            const T* vb = value + ((size_t)n * S + sStart[l]) * MD;
            for (int p = 0; p < P; ++p) {
                const long si = sbase + l * P + p;
                Corner<T> r;
                sample2d<T, PAD>(vb, sH[l], sW[l], MD, m * D + c, loc[2 * si], loc[2 * si + 1], r);
                if (MODE == 0) col += r.val * attn[si];
                else out[((((size_t)(n * M + m) * D + c) * Lq + q) * L + l) * P + p] = r.val;
            }
        }
        if (MODE == 0) out[(size_t)wave * D + c] = col;
    }
    }
}

// MODE 0: backward of the weighted op;  MODE 1: backward of the raw-sample mode (no attn)
template <typename T, int PAD, int MODE>
__global__ __launch_bounds__(256) void msda2d_bwd_kernel(const T* __restrict__ value, const int64_t* __restrict__ shapes,
                                                          const int64_t* __restrict__ lsi, const T* __restrict__ loc,
                                                          const T* __restrict__ attn, const T* __restrict__ gout,
                                                          int N, int S, int M, int D, int L, int Lq, int P, int gate_1d,
                                                          T* __restrict__ grad_value, T* __restrict__ grad_loc,
                                                          T* __restrict__ grad_attn) {
    if (gate_1d) {  // a lifted 1-D pyramid is the drop-in fast path's (msda_dropin_bwd_query_kernel + value kernel)
        Levels1d lv;
        if (dropin_levels(shapes, lsi, S, lv)) return;
    }
    __shared__ int sH[kMaxLevels2d], sW[kMaxLevels2d], sStart[kMaxLevels2d];
    load_levels(shapes, lsi, L, S, sH, sW, sStart);
    const int lane = threadIdx.x & 63;
    const long nwaves = (long)gridDim.x * (blockDim.x >> 6);
    for (long wave = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); wave < (long)N * Lq * M;
         wave += nwaves) {
    const int m = (int)(wave % M);
    const int q = (int)((wave / M) % Lq);
    const int n = (int)(wave / ((long)M * Lq));
    const int MD = M * D;
    const long sbase = (long)wave * L * P;
    for (int l = 0; l < L; ++l) {
        const T* vb = value + ((size_t)n * S + sStart[l]) * MD;
        T* gvb = grad_value + ((size_t)n * S + sStart[l]) * MD;
        for (int p = 0; p < P; ++p) {
            const long si = sbase + l * P + p;
            const T lw_ = loc[2 * si], lh_ = loc[2 * si + 1];
            const T a = (MODE == 0) ? attn[si] : (T)1;
            T ga = 0, glw = 0, glh = 0;
            for (int c = lane; c < D; c += PDVC_WAVE) {
                const T g = (MODE == 0) ? gout[(size_t)wave * D + c]
                                        : gout[((((size_t)(n * M + m) * D + c) * Lq + q) * L + l) * P + p];
                Corner<T> r;
                sample2d<T, PAD>(vb, sH[l], sW[l], MD, m * D + c, lw_, lh_, r);
                const T tgv = g * a;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (r.ci[k] >= 0) atomicAdd(gvb + (size_t)r.ci[k] * MD + m * D + c, r.cw[k] * tgv);
                ga += g * r.val;
                glw += r.dw * tgv;
                glh += r.dh * tgv;
            }
            glw = wave_sum(glw);
            glh = wave_sum(glh);
            if (MODE == 0) ga = wave_sum(ga);
            if (lane == 0) {
                grad_loc[2 * si] = glw;
                grad_loc[2 * si + 1] = glh;
                if (MODE == 0) grad_attn[si] = ga;
            }
        }
    }
    }
}

// grad_value's zero fill for the atomics of msda2d_bwd_kernel; skipped (gate_1d) when the table is a lifted 1-D
// pyramid: the fast path's value-gradient kernel writes every row itself
__global__ __launch_bounds__(256) void msda2d_zero_kernel(float* __restrict__ p, size_t n4,
                                                           const int64_t* __restrict__ shapes,
                                                           const int64_t* __restrict__ lsi, int S, int gate_1d) {
    if (gate_1d) {
        Levels1d lv;
        if (dropin_levels(shapes, lsi, S, lv)) return;
    }
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    float4* q = reinterpret_cast<float4*>(p);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
        q[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// grid-stride launches, at most kMaxBlocks2d workgroups: enough to fill the chip, and cheap to retire when the
// 1-D gate sends the work to the fast path
constexpr long kMaxBlocks2d = 8192;

template <typename T, int PAD, int MODE>
static int launch_fwd(const T* value, const int64_t* shapes, const int64_t* lsi, const T* loc, const T* attn, int N,
                      int S, int M, int D, int L, int Lq, int P, T* out, hipStream_t stream, int gate_1d = 0) {
    const long waves = (long)N * Lq * M;
    if (waves == 0) return PDVC_OK;
    const int blocks = (int)std::min((waves + 3) / 4, kMaxBlocks2d);
    hipLaunchKernelGGL((msda2d_fwd_kernel<T, PAD, MODE>), dim3(blocks), dim3(256), 0, stream, value, shapes, lsi, loc,
                       attn, N, S, M, D, L, Lq, P, gate_1d, out);
    PDVC_CHECK_LAUNCH("msda2d_fwd_kernel");
    return PDVC_OK;
}

template <typename T, int PAD, int MODE>
static int launch_bwd(const T* value, const int64_t* shapes, const int64_t* lsi, const T* loc, const T* attn,
                      const T* gout, int N, int S, int M, int D, int L, int Lq, int P, T* gv, T* gl, T* ga,
                      hipStream_t stream, int gate_1d = 0) {
    const size_t nf = sizeof(T) / sizeof(float) * (size_t)N * S * M * D;
    if (nf > 0) {
        if (gate_1d) {  // D = 64 on this path: float4 stores, aligned (a torch allocation)
            const unsigned zb = (unsigned)std::min<size_t>(nf / 4 / 256 + 1, 8192);
            hipLaunchKernelGGL(msda2d_zero_kernel, dim3(zb), dim3(256), 0, stream, reinterpret_cast<float*>(gv), nf / 4,
                               shapes, lsi, S, gate_1d);
            PDVC_CHECK_LAUNCH("msda2d_zero_kernel");
        } else {
            hipError_t e = zero_async(reinterpret_cast<float*>(gv), nf, stream);
            if (e != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "memset grad_value: %s", hipGetErrorString(e));
        }
    }
    const long waves = (long)N * Lq * M;
    if (waves == 0) return PDVC_OK;
    const int blocks = (int)std::min((waves + 3) / 4, kMaxBlocks2d);
    hipLaunchKernelGGL((msda2d_bwd_kernel<T, PAD, MODE>), dim3(blocks), dim3(256), 0, stream, value, shapes, lsi, loc,
                       attn, gout, N, S, M, D, L, Lq, P, gate_1d, gv, gl, ga);
    PDVC_CHECK_LAUNCH("msda2d_bwd_kernel");
    return PDVC_OK;
}

static int check_common(int batch, int spatial_size, int num_heads, int channels, int num_levels, int num_query,
                        int num_point) {
    PDVC_CHECK_ARG(batch >= 0 && spatial_size >= 0 && num_heads > 0 && channels > 0 && num_query >= 0 &&
                       num_point > 0,
                   "invalid sizes (batch=%d S=%d M=%d D=%d Lq=%d P=%d)", batch, spatial_size, num_heads, channels,
                   num_query, num_point);
    PDVC_CHECK_ARG(num_levels > 0 && num_levels <= kMaxLevels2d, "num_levels must be in [1,%d], got %d", kMaxLevels2d,
                   num_levels);
    return PDVC_OK;
}

static int check_step(int batch, int im2col_step) {
    // ms_deform_attn_cuda.cu:50-52: im2col_step_ = min(batch, im2col_step); batch % im2col_step_ == 0
    if (batch == 0) return PDVC_OK;
    PDVC_CHECK_ARG(im2col_step > 0, "im2col_step must be positive, got %d", im2col_step);
    const int step = batch < im2col_step ? batch : im2col_step;
    PDVC_CHECK_ARG(batch % step == 0, "batch(%d) must divide im2col_step(%d)", batch, step);
    return PDVC_OK;
}

}  // namespace pdvc

using namespace pdvc;

#define PDVC_DEFINE_OP(T, SFX)                                                                                     \
    extern "C" int pdvc_ms_deform_attn_forward_##SFX(const T* value, const int64_t* spatial_shapes,                 \
                                                     const int64_t* level_start_index, const T* sampling_loc,       \
                                                     const T* attn_weight, int batch, int spatial_size,             \
                                                     int num_heads, int channels, int num_levels, int num_query,    \
                                                     int num_point, int im2col_step, T* output, void* stream) {     \
        int rc = check_common(batch, spatial_size, num_heads, channels, num_levels, num_query, num_point);          \
        if (rc) return rc;                                                                                          \
        if ((rc = check_step(batch, im2col_step))) return rc;                                                       \
        return launch_fwd<T, PDVC_PAD_ZEROS, 0>(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, \
                                                batch, spatial_size, num_heads, channels, num_levels, num_query,    \
                                                num_point, output, (hipStream_t)stream);                            \
    }                                                                                                               \
    extern "C" int pdvc_ms_deform_attn_backward_##SFX(                                                              \
        const T* value, const int64_t* spatial_shapes, const int64_t* level_start_index, const T* sampling_loc,     \
        const T* attn_weight, const T* grad_output, int batch, int spatial_size, int num_heads, int channels,       \
        int num_levels, int num_query, int num_point, int im2col_step, T* grad_value, T* grad_sampling_loc,        \
        T* grad_attn_weight, void* stream) {                                                                        \
        int rc = check_common(batch, spatial_size, num_heads, channels, num_levels, num_query, num_point);          \
        if (rc) return rc;                                                                                          \
        if ((rc = check_step(batch, im2col_step))) return rc;                                                       \
        return launch_bwd<T, PDVC_PAD_ZEROS, 0>(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, \
                                                grad_output, batch, spatial_size, num_heads, channels, num_levels,  \
                                                num_query, num_point, grad_value, grad_sampling_loc,                \
                                                grad_attn_weight, (hipStream_t)stream);                             \
    }

PDVC_DEFINE_OP(double, f64)

// f32: the same entry points, plus the 1-D fast path for a lifted pyramid (device-side dispatch, dropin_levels)
extern "C" int pdvc_ms_deform_attn_forward_f32(const float* value, const int64_t* spatial_shapes,
                                               const int64_t* level_start_index, const float* sampling_loc,
                                               const float* attn_weight, int batch, int spatial_size, int num_heads,
                                               int channels, int num_levels, int num_query, int num_point,
                                               int im2col_step, float* output, void* stream) {
    int rc = check_common(batch, spatial_size, num_heads, channels, num_levels, num_query, num_point);
    if (rc) return rc;
    if ((rc = check_step(batch, im2col_step))) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int fast = dropin1d_applies(spatial_size, num_heads, channels, num_levels, num_query, num_point);
    if (fast && (rc = dropin1d_forward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, batch,
                                       spatial_size, num_heads, num_query, output, s)))
        return rc;
    return launch_fwd<float, PDVC_PAD_ZEROS, 0>(value, spatial_shapes, level_start_index, sampling_loc, attn_weight,
                                                batch, spatial_size, num_heads, channels, num_levels, num_query,
                                                num_point, output, s, fast);
}

extern "C" size_t pdvc_ms_deform_attn_workspace_floats(int batch, int num_heads, int num_levels, int num_query,
                                                       int num_point) {
    return 2 * (size_t)batch * num_query * num_heads * num_levels * num_point;
}

extern "C" int pdvc_ms_deform_attn_backward_ws_f32(const float* value, const int64_t* spatial_shapes,
                                                   const int64_t* level_start_index, const float* sampling_loc,
                                                   const float* attn_weight, const float* grad_output, int batch,
                                                   int spatial_size, int num_heads, int channels, int num_levels,
                                                   int num_query, int num_point, int im2col_step, float* grad_value,
                                                   float* grad_sampling_loc, float* grad_attn_weight, float* workspace,
                                                   size_t workspace_floats, void* stream) {
    int rc = check_common(batch, spatial_size, num_heads, channels, num_levels, num_query, num_point);
    if (rc) return rc;
    if ((rc = check_step(batch, im2col_step))) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int fast = workspace != nullptr &&
                     workspace_floats >= pdvc_ms_deform_attn_workspace_floats(batch, num_heads, num_levels, num_query,
                                                                              num_point) &&
                     dropin1d_applies(spatial_size, num_heads, channels, num_levels, num_query, num_point);
    // the general path first: with the gate its zero fill and kernel retire at once for a 1-D pyramid
    if ((rc = launch_bwd<float, PDVC_PAD_ZEROS, 0>(value, spatial_shapes, level_start_index, sampling_loc, attn_weight,
                                                   grad_output, batch, spatial_size, num_heads, channels, num_levels,
                                                   num_query, num_point, grad_value, grad_sampling_loc,
                                                   grad_attn_weight, s, fast)))
        return rc;
    if (fast)
        return dropin1d_backward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output,
                                 batch, spatial_size, num_heads, num_query, grad_value, grad_sampling_loc,
                                 grad_attn_weight, workspace, s);
    return PDVC_OK;
}

extern "C" int pdvc_ms_deform_attn_backward_f32(const float* value, const int64_t* spatial_shapes,
                                                const int64_t* level_start_index, const float* sampling_loc,
                                                const float* attn_weight, const float* grad_output, int batch,
                                                int spatial_size, int num_heads, int channels, int num_levels,
                                                int num_query, int num_point, int im2col_step, float* grad_value,
                                                float* grad_sampling_loc, float* grad_attn_weight, void* stream) {
    return pdvc_ms_deform_attn_backward_ws_f32(value, spatial_shapes, level_start_index, sampling_loc, attn_weight,
                                               grad_output, batch, spatial_size, num_heads, channels, num_levels,
                                               num_query, num_point, im2col_step, grad_value, grad_sampling_loc,
                                               grad_attn_weight, nullptr, 0, stream);
}

extern "C" int pdvc_ms_deform_sample_f32(const float* value, const int64_t* spatial_shapes,
                                         const int64_t* level_start_index, const float* sampling_loc, int batch,
                                         int spatial_size, int num_heads, int channels, int num_levels,
                                         int num_query, int num_point, int padding, float* samples, void* stream) {
    int rc = check_common(batch, spatial_size, num_heads, channels, num_levels, num_query, num_point);
    if (rc) return rc;
    if (padding == PDVC_PAD_ZEROS)
        return launch_fwd<float, PDVC_PAD_ZEROS, 1>(value, spatial_shapes, level_start_index, sampling_loc, nullptr,
                                                    batch, spatial_size, num_heads, channels, num_levels, num_query,
                                                    num_point, samples, (hipStream_t)stream);
    if (padding == PDVC_PAD_BORDER)
        return launch_fwd<float, PDVC_PAD_BORDER, 1>(value, spatial_shapes, level_start_index, sampling_loc, nullptr,
                                                     batch, spatial_size, num_heads, channels, num_levels, num_query,
                                                     num_point, samples, (hipStream_t)stream);
    return pdvc_set_error(PDVC_ERR_INVALID_ARG, "padding must be PDVC_PAD_ZEROS or PDVC_PAD_BORDER, got %d", padding);
}

extern "C" int pdvc_ms_deform_sample_backward_f32(const float* value, const int64_t* spatial_shapes,
                                                  const int64_t* level_start_index, const float* sampling_loc,
                                                  const float* grad_samples, int batch, int spatial_size,
                                                  int num_heads, int channels, int num_levels, int num_query,
                                                  int num_point, int padding, float* grad_value,
                                                  float* grad_sampling_loc, void* stream) {
    int rc = check_common(batch, spatial_size, num_heads, channels, num_levels, num_query, num_point);
    if (rc) return rc;
    if (padding == PDVC_PAD_ZEROS)
        return launch_bwd<float, PDVC_PAD_ZEROS, 1>(value, spatial_shapes, level_start_index, sampling_loc, nullptr,
                                                    grad_samples, batch, spatial_size, num_heads, channels,
                                                    num_levels, num_query, num_point, grad_value, grad_sampling_loc,
                                                    nullptr, (hipStream_t)stream);
    if (padding == PDVC_PAD_BORDER)
        return launch_bwd<float, PDVC_PAD_BORDER, 1>(value, spatial_shapes, level_start_index, sampling_loc, nullptr,
                                                     grad_samples, batch, spatial_size, num_heads, channels,
                                                     num_levels, num_query, num_point, grad_value, grad_sampling_loc,
                                                     nullptr, (hipStream_t)stream);
    return pdvc_set_error(PDVC_ERR_INVALID_ARG, "padding must be PDVC_PAD_ZEROS or PDVC_PAD_BORDER, got %d", padding);
}
