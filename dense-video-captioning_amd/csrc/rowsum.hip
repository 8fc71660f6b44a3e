// rowsum.hip -- destination-sorted row sums: dst[v] = sum of the src rows whose key is v, in a fixed order.
//
// The backward of a gather out = table[idx] (the caption head's word gates as rows of the per-batch vocabulary
// table W_x embed^T, LSTM_DSA.py:229-231 in the reference: xt = embed(it), then W_ih over [xt, ...]): the table's
// gradient sums the gathered rows' gradients per vocabulary entry.  torch's index_add_ does that with float atomics
// (order-dependent, contended on frequent words); here the positions arrive sorted by key (a stable sort, so the
// order inside a key is the positions' order) and one workgroup owns one key's output row chunk: no atomics,
// deterministic.  Each workgroup finds its key's run in the sorted keys by binary search.  HBM-bound: every src row
// is read once and every dst row written once.
#include "pdvc_common.h"

namespace pdvc {

constexpr int kRsLanes = 64;  // float4 column lanes per workgroup (256 columns)
constexpr int kRsRows = 4;    // row lanes (interleaved positions of the key's run)

__device__ __forceinline__ long lower_bound_key(const int64_t* __restrict__ keys, long n, int64_t v) {
    long lo = 0, hi = n;
    while (lo < hi) {
        const long mid = (lo + hi) >> 1;
        if (keys[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kRsLanes * kRsRows) void sorted_row_sums_kernel(const float* __restrict__ src, long ld,
                                                                             int cols, const int64_t* __restrict__ keys,
                                                                             const int64_t* __restrict__ order, long n,
                                                                             float* __restrict__ dst, long ldd) {
    __shared__ float4 red[kRsRows][kRsLanes];
    __shared__ long run[2];
    const int v = blockIdx.x;
    const int cl = threadIdx.x % kRsLanes, rl = threadIdx.x / kRsLanes;
    if (threadIdx.x < 2) run[threadIdx.x] = lower_bound_key(keys, n, (int64_t)v + threadIdx.x);
    __syncthreads();
    const long b = run[0], e = run[1];
    const int c4 = blockIdx.y * kRsLanes + cl;
    const bool live = c4 * 4 < cols;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (live) {
        for (long j = b + rl; j < e; j += kRsRows) {
            const float4 x = *reinterpret_cast<const float4*>(src + order[j] * ld + 4 * c4);
            a.x += x.x;
            a.y += x.y;
            a.z += x.z;
            a.w += x.w;
        }
    }
    red[rl][cl] = a;
    __syncthreads();
    if (rl == 0 && live) {
        float4 t = red[0][cl];
#pragma unroll
        for (int k = 1; k < kRsRows; ++k) {
            t.x += red[k][cl].x;
            t.y += red[k][cl].y;
            t.z += red[k][cl].z;
            t.w += red[k][cl].w;
        }
        *reinterpret_cast<float4*>(dst + (long)v * ldd + 4 * c4) = t;
    }
}

}  // namespace pdvc

using namespace pdvc;

// C-ABI: see include/pdvc_msda.h
extern "C" int pdvc_sorted_row_sums_f32(const float* src, long ld, int cols, const int64_t* sorted_keys,
                                        const int64_t* order, long n, int n_dst, float* dst, long ldd, void* stream) {
    PDVC_CHECK_ARG(cols > 0 && cols % 4 == 0 && n >= 0 && n_dst >= 0, "cols a positive multiple of 4, n, n_dst >= 0");
    PDVC_CHECK_ARG(ld >= cols && ld % 4 == 0 && ldd >= cols && ldd % 4 == 0, "leading dimensions: >= cols, multiples of 4");
    PDVC_CHECK_ARG(n_dst == 0 || (dst && (n == 0 || (src && sorted_keys && order))), "null pointer");
    PDVC_CHECK_ARG((uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0, "src and dst must be 16-byte aligned");
    if (n_dst == 0) return PDVC_OK;
    const dim3 grid((unsigned)n_dst, (unsigned)((cols / 4 + kRsLanes - 1) / kRsLanes));
    hipLaunchKernelGGL(sorted_row_sums_kernel, grid, dim3(kRsLanes * kRsRows), 0, (hipStream_t)stream, src, ld, cols,
                       sorted_keys, order, n, dst, ldd);
    PDVC_CHECK_LAUNCH("sorted_row_sums_kernel");
    return PDVC_OK;
}
