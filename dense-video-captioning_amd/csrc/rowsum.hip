// rowsum.hip -- destination-sorted row sums: dst[v] = sum of the src rows whose key is v, in a fixed order.
//
// The backward of a gather out = table[idx] (the caption head's word gates as rows of the per-batch vocabulary
// table W_x embed^T, LSTM_DSA.py:229-231 in the reference: xt = embed(it), then W_ih over [xt, ...]): the table's
// gradient sums the gathered rows' gradients per vocabulary entry.  torch's index_add_ does that with float atomics
// (order-dependent, contended on frequent words); here the positions arrive sorted by key (a stable sort, so the
// order inside a key is the positions' order) and are summed as a reduce-by-key over fixed chunks of kRsChunk
// sorted positions, so a frequent key (every caption's start token, the end token, common words: thousands of
// positions) is spread over many workgroups instead of one:
//   1. rows_zero_kernel: the destination rows of keys with no position are zeros;
//   2. rows_chunk_kernel: one workgroup per (chunk, 256 columns) walks its chunk in order; a key whose run lies
//      inside the chunk is written to dst at once, the pieces of a run that crosses a chunk edge go to the
//      workspace (the run's opening piece: `open[c]`; a piece that starts at the chunk's first position: `head[c]`);
//   3. rows_join_kernel: one workgroup per chunk whose last run opens in it sums that run's pieces in chunk order.
// No atomics; every sum in a fixed order, so the result is deterministic.  HBM: each src row read once, each dst row
// written once, plus the pieces (2 x chunks x cols floats).
#include "pdvc_common.h"

namespace pdvc {

constexpr int kRsChunk = 64;  // sorted positions per chunk (the C-ABI's workspace unit)
constexpr int kRsLanes = 64;  // float4 column lanes per workgroup (256 columns)

__device__ __forceinline__ long lower_bound_key(const int64_t* __restrict__ keys, long n, int64_t v) {
    long lo = 0, hi = n;
    while (lo < hi) {
        const long mid = (lo + hi) >> 1;
        if (keys[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ void add4(float4& a, const float4& x) {
    a.x += x.x;
    a.y += x.y;
    a.z += x.z;
    a.w += x.w;
}

// 1. zeros for the destination rows of keys that have no position
__global__ __launch_bounds__(kRsLanes) void rows_zero_kernel(const int64_t* __restrict__ keys, long n, int cols,
                                                            float* __restrict__ dst, long ldd) {
    const int v = blockIdx.x, c4 = blockIdx.y * kRsLanes + threadIdx.x;
    const long b = lower_bound_key(keys, n, v);
    if ((b < n && keys[b] == v) || 4 * c4 >= cols) return;
    *reinterpret_cast<float4*>(dst + (long)v * ldd + 4 * c4) = make_float4(0.f, 0.f, 0.f, 0.f);
}

// 2. the chunk's runs in order; a run inside the chunk straight to dst, the pieces of runs crossing an edge to ws
__global__ __launch_bounds__(kRsLanes) void rows_chunk_kernel(const float* __restrict__ src, long ld, int cols,
                                                             const int64_t* __restrict__ keys,
                                                             const int64_t* __restrict__ order, long n, int n_dst,
                                                             float* __restrict__ dst, long ldd,
                                                             float* __restrict__ open, float* __restrict__ head) {
    __shared__ int64_t sk[kRsChunk + 2];  // keys[j0 - 1 .. j1] (ends past the list as INT64_MIN, never a key)
    __shared__ int64_t so[kRsChunk];
    const long c = blockIdx.x, j0 = c * kRsChunk, j1 = min(j0 + kRsChunk, n);
    const int m = (int)(j1 - j0);
    const int t = threadIdx.x;
    if (t < m) {
        sk[t + 1] = keys[j0 + t];
        so[t] = order[j0 + t];
    }
    if (t == 0) sk[0] = j0 > 0 ? keys[j0 - 1] : INT64_MIN;
    if (t == 1) sk[m + 1] = j1 < n ? keys[j1] : INT64_MIN;
    __syncthreads();
    const int c4 = blockIdx.y * kRsLanes + t;
    if (4 * c4 >= cols) return;
    const long cb = (long)c * cols + 4 * c4;  // this lane's float4 in the chunk's workspace rows
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = 0;  // first position of the current segment (chunk-relative)
    // rows loaded kRsPre ahead of their add: the loads do not wait on the previous add
    constexpr int kRsPre = 8;
    float4 pre[kRsPre];
#pragma unroll
    for (int q = 0; q < kRsPre; ++q)
        pre[q] = q < m ? *reinterpret_cast<const float4*>(src + so[q] * ld + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j = 0; j < m; j += kRsPre) {
#pragma unroll
        for (int q = 0; q < kRsPre; ++q) {
            const int jj = j + q;
            if (jj < m) {
                add4(acc, pre[q]);
                const int jn = jj + kRsPre;
                if (jn < m) pre[q] = *reinterpret_cast<const float4*>(src + so[jn] * ld + 4 * c4);
                const int64_t k = sk[jj + 1];
                if (jj + 1 == m || sk[jj + 2] != k) {  // the segment [s, jj] ends here (or at the chunk's end)
                    const bool starts = sk[s] != k;             // the key's run starts inside this chunk
                    const bool ends = jj + 1 < m || sk[m + 1] != k;  // ... and ends inside it
                    if (starts && ends) {
                        if (k >= 0 && k < n_dst) *reinterpret_cast<float4*>(dst + k * ldd + 4 * c4) = acc;
                    } else if (starts) {
                        *reinterpret_cast<float4*>(open + cb) = acc;  // the run's opening piece
                    } else {
                        *reinterpret_cast<float4*>(head + cb) = acc;  // a piece at the chunk's first position
                    }
                    acc = make_float4(0.f, 0.f, 0.f, 0.f);
                    s = jj + 1;
                }
            }
        }
    }
}

// 3. the runs that open in chunk c and end in a later chunk: open[c] + head[c + 1] + ... in chunk order
__global__ __launch_bounds__(kRsLanes) void rows_join_kernel(const int64_t* __restrict__ keys, long n, int cols,
                                                            int n_dst, float* __restrict__ dst, long ldd,
                                                            const float* __restrict__ open,
                                                            const float* __restrict__ head) {
    const long c = blockIdx.x, j0 = c * kRsChunk, j1 = min(j0 + kRsChunk, n);
    if (j1 >= n) return;
    const int64_t k = keys[j1 - 1];
    if (keys[j1] != k) return;  // the chunk's last run does not cross its end
    // ... and it must open here: its first position inside the chunk
    const long b = lower_bound_key(keys, n, k);
    if (b < j0) return;
    const int c4 = blockIdx.y * kRsLanes + threadIdx.x;
    if (4 * c4 >= cols || k < 0 || k >= n_dst) return;
    const long e = lower_bound_key(keys, n, k + 1);  // one past the run's last position
    const long c_last = (e - 1) / kRsChunk;
    float4 acc = *reinterpret_cast<const float4*>(open + c * cols + 4 * c4);
    long q = c + 1;
    for (; q + 4 <= c_last + 1; q += 4) {  // four pieces in flight, added in order
        const float4 x0 = *reinterpret_cast<const float4*>(head + q * cols + 4 * c4);
        const float4 x1 = *reinterpret_cast<const float4*>(head + (q + 1) * cols + 4 * c4);
        const float4 x2 = *reinterpret_cast<const float4*>(head + (q + 2) * cols + 4 * c4);
        const float4 x3 = *reinterpret_cast<const float4*>(head + (q + 3) * cols + 4 * c4);
        add4(acc, x0);
        add4(acc, x1);
        add4(acc, x2);
        add4(acc, x3);
    }
    for (; q <= c_last; ++q) add4(acc, *reinterpret_cast<const float4*>(head + q * cols + 4 * c4));
    *reinterpret_cast<float4*>(dst + k * ldd + 4 * c4) = acc;
}

}  // namespace pdvc

using namespace pdvc;

// C-ABI: see include/pdvc_msda.h
extern "C" long pdvc_sorted_row_sums_workspace(long n, int cols) {
    return n <= 0 ? 0 : 2 * ((n + kRsChunk - 1) / kRsChunk) * (long)cols;
}

extern "C" int pdvc_sorted_row_sums_f32(const float* src, long ld, int cols, const int64_t* sorted_keys,
                                        const int64_t* order, long n, int n_dst, float* dst, long ldd,
                                        float* workspace, void* stream) {
    PDVC_CHECK_ARG(cols > 0 && cols % 4 == 0 && n >= 0 && n_dst >= 0, "cols a positive multiple of 4, n, n_dst >= 0");
    PDVC_CHECK_ARG(ld >= cols && ld % 4 == 0 && ldd >= cols && ldd % 4 == 0, "leading dimensions: >= cols, multiples of 4");
    PDVC_CHECK_ARG(n_dst == 0 || (dst && (n == 0 || (src && sorted_keys && order && workspace))), "null pointer");
    PDVC_CHECK_ARG((uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0 && (uintptr_t)workspace % 16 == 0,
                   "src, dst and workspace must be 16-byte aligned");
    if (n_dst == 0) return PDVC_OK;
    hipStream_t s = (hipStream_t)stream;
    const unsigned cch = (unsigned)((cols / 4 + kRsLanes - 1) / kRsLanes);
    hipLaunchKernelGGL(rows_zero_kernel, dim3((unsigned)n_dst, cch), dim3(kRsLanes), 0, s, sorted_keys, n, cols, dst,
                       ldd);
    PDVC_CHECK_LAUNCH("rows_zero_kernel");
    if (n == 0) return PDVC_OK;
    const long chunks = (n + kRsChunk - 1) / kRsChunk;
    PDVC_CHECK_ARG(chunks < (1L << 31), "too many positions");
    float* open = workspace;
    float* head = workspace + chunks * (long)cols;
    hipLaunchKernelGGL(rows_chunk_kernel, dim3((unsigned)chunks, cch), dim3(kRsLanes), 0, s, src, ld, cols,
                       sorted_keys, order, n, n_dst, dst, ldd, open, head);
    PDVC_CHECK_LAUNCH("rows_chunk_kernel");
    hipLaunchKernelGGL(rows_join_kernel, dim3((unsigned)chunks, cch), dim3(kRsLanes), 0, s, sorted_keys, n, cols, n_dst,
                       dst, ldd, open, head);
    PDVC_CHECK_LAUNCH("rows_join_kernel");
    return PDVC_OK;
}
