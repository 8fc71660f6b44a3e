// boxref.hip -- iterative box refinement, out = sigmoid(tmp + inverse_sigmoid(reference)), as one pass each way.
//
// Reference: the decoder's refinement (pdvc/deformable_transformer.py:~300-318: new_reference_points =
// (tmp + inverse_sigmoid(reference_points)).sigmoid(), or only the centre refined when the references are 1-d) and
// the per-layer box heads of PDVC.forward (pdvc/pdvc.py:245-253); inverse_sigmoid is misc/detr_utils/misc.py:540-544
// (clamp to [0, 1], then log(max(x, eps) / max(1 - x, eps))).  In torch each is ~9 elementwise launches forward and
// as many backward per layer.  Rows of 2 channels (centre, length); the reference has rd = 1 (centre only) or 2.
#include "pdvc_common.h"

namespace pdvc {

__device__ __forceinline__ float inv_sigmoid(float r, float eps) {
    const float x = fminf(fmaxf(r, 0.f), 1.f);
    const float x1 = fmaxf(x, eps), x2 = fmaxf(1.f - x, eps);
    return logf(x1 / x2);
}

__global__ __launch_bounds__(256) void box_refine_fwd_kernel(const float* __restrict__ tmp, const float* __restrict__ ref,
                                                             long rows, int rd, float eps, float* __restrict__ out) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < rows * 2; i += (long)gridDim.x * blockDim.x) {
        const long r = i >> 1;
        const int c = (int)(i & 1);
        float z = tmp[i];
        if (c < rd) z = z + inv_sigmoid(ref[r * rd + c], eps);
        out[i] = 1.f / (1.f + expf(-z));
    }
}

// gtmp = g s (1 - s); gref (optional) = gtmp * d inverse_sigmoid / d ref, torch's clamp convention (the gradient
// passes where min <= x <= max)
__global__ __launch_bounds__(256) void box_refine_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ out,
                                                             const float* __restrict__ ref, long rows, int rd, float eps,
                                                             float* __restrict__ gtmp, float* __restrict__ gref) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < rows * 2; i += (long)gridDim.x * blockDim.x) {
        const long r = i >> 1;
        const int c = (int)(i & 1);
        const float s = out[i];
        const float gz = gout[i] * (s * (1.f - s));
        gtmp[i] = gz;
        if (gref != nullptr && c < rd) {
            const float rv = ref[r * rd + c];
            const float x = fminf(fmaxf(rv, 0.f), 1.f);
            const float x1 = fmaxf(x, eps), x2 = fmaxf(1.f - x, eps);
            // log(x1 / x2): d/dx1 = 1 / x1, d/dx2 = -1 / x2; x1 = max(x, eps), x2 = max(1 - x, eps)
            float gx = (x >= eps ? gz / x1 : 0.f) + ((1.f - x) >= eps ? gz / x2 : 0.f);
            gref[r * rd + c] = (rv >= 0.f && rv <= 1.f) ? gx : 0.f;
        }
    }
}

}  // namespace pdvc

using namespace pdvc;

static unsigned box_blocks(long n) {
    const long b = (n + 255) / 256;
    return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

extern "C" int pdvc_box_refine_forward_f32(const float* tmp, const float* ref, long rows, int rd, float eps,
                                           float* out, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && (rd == 1 || rd == 2), "box refine: rows >= 0 and rd in {1, 2}, got %ld, %d", rows, rd);
    if (rows == 0) return PDVC_OK;
    hipLaunchKernelGGL(box_refine_fwd_kernel, dim3(box_blocks(rows * 2)), dim3(256), 0, (hipStream_t)stream, tmp, ref,
                       rows, rd, eps, out);
    PDVC_CHECK_LAUNCH("box_refine_fwd_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_box_refine_backward_f32(const float* grad_out, const float* out, const float* ref, long rows,
                                            int rd, float eps, float* grad_tmp, float* grad_ref, void* stream) {
    PDVC_CHECK_ARG(rows >= 0 && (rd == 1 || rd == 2), "box refine: rows >= 0 and rd in {1, 2}, got %ld, %d", rows, rd);
    if (rows == 0) return PDVC_OK;
    hipLaunchKernelGGL(box_refine_bwd_kernel, dim3(box_blocks(rows * 2)), dim3(256), 0, (hipStream_t)stream, grad_out,
                       out, ref, rows, rd, eps, grad_tmp, grad_ref);
    PDVC_CHECK_LAUNCH("box_refine_bwd_kernel");
    return PDVC_OK;
}
