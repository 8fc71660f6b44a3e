// pdvc_common.h -- shared device helpers for the PDVC HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdlib>
#include <initializer_list>
#include <utility>
#include <stdint.h>

#include "pdvc_msda.h"

#define PDVC_WAVE 64

namespace pdvc {

// Bijective XCD-aware block remap (MI355X: 8 XCDs, blocks dealt round-robin, so hardware blocks b and
// b+8 share an XCD).  Returns a logical block id such that logical ids [k*per, (k+1)*per) all run on one
// XCD: consecutive logical blocks (same video in our orderings) share that XCD's 4 MB L2.  Speed only.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
    const int q = nblocks >> 3, r = nblocks & 7;
    const int xcd = bid & 7, slot = bid >> 3;
    const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + slot;
}

// Packed fp32 lanes: a float4 held as two register pairs (.xy, .zw), each updated by one v_pk_fma_f32 with the
// scalar weight broadcast (op_sel_hi).  Written per component with fmaf on a float4, the compiler pairs (x, z) and
// (y, w) for v_pk_fma_f32 and re-packs every loaded row with three v_mov_b32 (1 798 movs against 1 024 packed FMAs in
// the pyramid forward); on (.xy, .zw) the loaded registers are the operands as they stand.  Same products, same
// order per component as the fmaf form: the same bits.
typedef float pf2 __attribute__((ext_vector_type(2)));
typedef float pf4 __attribute__((ext_vector_type(4)));

struct PAcc4 {
    pf2 lo, hi;  // (x, y), (z, w)
};

__device__ __forceinline__ PAcc4 pacc_zero() { return PAcc4{pf2{0.f, 0.f}, pf2{0.f, 0.f}}; }

// acc += c * v (4 channels)
__device__ __forceinline__ void pacc_fma(PAcc4& a, float c, const pf4 v) {
    const pf2 cc = {c, c};
    a.lo = __builtin_elementwise_fma(cc, v.xy, a.lo);
    a.hi = __builtin_elementwise_fma(cc, v.zw, a.hi);
}

__device__ __forceinline__ float4 pacc_f4(const PAcc4& a) { return make_float4(a.lo.x, a.lo.y, a.hi.x, a.hi.y); }

// Exact xor-partner exchange for butterfly step d (1, 2, 4, 8) inside aligned 16-lane groups without
// ds_bpermute's lane-index arithmetic: d = 1, 2 on DPP quad_perm, d = 8 on DPP row_ror:8 (VALU operand
// modifiers, no LDS traffic), d = 4 on ds_swizzle's bit mode (gfx9 DPP has no xor-4 pattern; row_half_mirror
// would pair lanes across more than one bit, which is wrong for partial reductions over the higher bits only).
__device__ __forceinline__ float grp_swap(float v, int d) {
    const int x = __float_as_int(v);
    int r;
    switch (d) {
        // every lane has a valid source in these patterns: mov_dpp (no `old` operand) saves the v_mov that would
        // initialise one
        case 1: r = __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true); break;   // quad_perm(1,0,3,2)
        case 2: r = __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true); break;   // quad_perm(2,3,0,1)
        case 4: r = __builtin_amdgcn_ds_swizzle(x, 0x1F | (0x04 << 10)); break;  // lane ^ 4
        default: r = __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, true); break;  // row_ror:8 = lane ^ 8
    }
    return __int_as_float(r);
}

// butterfly partner for any step d of a wave-wide reduction: DPP for d <= 8, ds_swizzle (exact xor inside
// 32-lane halves) for d = 16, ds_bpermute for d = 32
__device__ __forceinline__ float lane_swap(float v, int d) {
    if (d <= 8) return grp_swap(v, d);
    if (d == 16) return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (0x10 << 10)));
    return __shfl_xor(v, d, PDVC_WAVE);
}

// the lane with index k inside each aligned group of G (<= 32) lanes, for every lane of the group
// (ds_swizzle bit mode: lane' = (lane & and_mask) | k within each 32-lane half; k a compile-time constant after
// unrolling, so the pattern is an immediate -- no address arithmetic)
template <int G>
__device__ __forceinline__ int grp_bcast(int v, int k) {
    static_assert(G == 4 || G == 8 || G == 16 || G == 32, "group of 4..32 lanes");
    if constexpr (G == 16) {
        // DPP row_newbcast:k (dpp_ctrl 0x150 + k): lane k of each 16-lane row to the whole row, a VALU operand
        // modifier -- no LDS instruction (tools/probes/dpp_newbcast_probe.hip checks it on gfx950 for every k)
#define PDVC_NB(K) case K: return __builtin_amdgcn_mov_dpp(v, 0x150 + (K), 0xF, 0xF, true);
        switch (k) {
            PDVC_NB(0) PDVC_NB(1) PDVC_NB(2) PDVC_NB(3) PDVC_NB(4) PDVC_NB(5) PDVC_NB(6) PDVC_NB(7)
            PDVC_NB(8) PDVC_NB(9) PDVC_NB(10) PDVC_NB(11) PDVC_NB(12) PDVC_NB(13) PDVC_NB(14) PDVC_NB(15)
            default: return v;
        }
#undef PDVC_NB
    }
    constexpr int and_mask = 0x1F & ~(G - 1);
#define PDVC_SWZ(K) case K: return __builtin_amdgcn_ds_swizzle(v, and_mask | ((K) << 5));
    switch (k) {
        PDVC_SWZ(0) PDVC_SWZ(1) PDVC_SWZ(2) PDVC_SWZ(3) PDVC_SWZ(4) PDVC_SWZ(5) PDVC_SWZ(6) PDVC_SWZ(7)
        PDVC_SWZ(8) PDVC_SWZ(9) PDVC_SWZ(10) PDVC_SWZ(11) PDVC_SWZ(12) PDVC_SWZ(13) PDVC_SWZ(14) PDVC_SWZ(15)
        PDVC_SWZ(16) PDVC_SWZ(17) PDVC_SWZ(18) PDVC_SWZ(19) PDVC_SWZ(20) PDVC_SWZ(21) PDVC_SWZ(22) PDVC_SWZ(23)
        PDVC_SWZ(24) PDVC_SWZ(25) PDVC_SWZ(26) PDVC_SWZ(27) PDVC_SWZ(28) PDVC_SWZ(29) PDVC_SWZ(30) PDVC_SWZ(31)
        default: return v;
    }
#undef PDVC_SWZ
}
template <int G>
__device__ __forceinline__ float grp_bcast(float v, int k) {
    return __int_as_float(grp_bcast<G>(__float_as_int(v), k));
}

// Sum over aligned groups of G lanes (G power of two <= 64) with butterflies (DPP inside 16-lane groups).
template <int G>
__device__ __forceinline__ float group_allreduce(float v) {
#pragma unroll
    for (int d = G >> 1; d > 0; d >>= 1) v += lane_swap(v, d);
    return v;
}

// Transposed (reduce-scatter) butterfly inside aligned groups of G lanes: every lane enters with K
// partial values; after log2(G) halving steps lane r (= lane % G) holds the FULL group sums of the
// K/G consecutive values [r*K/G, (r+1)*K/G).  Costs K/2 + K/4 + ... exchanges instead of K*log2(G).
template <int K, int G>
__device__ __forceinline__ void group_reduce_scatter(float (&v)[K], int lane) {
    static_assert((K % G) == 0, "K must be a multiple of G");
    int keep = K;
#pragma unroll
    for (int d = G >> 1; d > 0; d >>= 1) {
        const bool upper = (lane & d) != 0;
        const int half = keep >> 1;
#pragma unroll
        for (int i = 0; i < K / 2; ++i) {
            if (i < half) {
                // value I send = the half I do not keep; value I receive lands on the half I keep
                const float send = upper ? v[i] : v[i + half];
                const float recv = lane_swap(send, d);
                const float mine = upper ? v[i + half] : v[i];
                v[i] = mine + recv;
            }
        }
        keep = half;
    }
}

template <int CPL>
struct VecF;
template <>
struct VecF<8> {
    float v[8];
    __device__ __forceinline__ void load(const float* p) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
    __device__ __forceinline__ void store(float* p) const {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 0.f;
    }
};
template <>
struct VecF<4> {
    float v[4];
    __device__ __forceinline__ void load(const float* p) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    }
    __device__ __forceinline__ void store(float* p) const {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = 0.f;
    }
};

// Levels of the temporal pyramid, passed by value (host-side constants of the model config), so the
// fused kernels never read spatial shapes from device memory.
struct Levels {
    int n;
    int T[PDVC_MAX_LEVELS];
    int start[PDVC_MAX_LEVELS];
};

// PDVC's temporal pyramid for the fused 1-D kernels (msda1d.hip): 4 levels, lengths and start rows, by value.
constexpr int kL1d = 4;
struct Levels1d {
    int T[kL1d];
    int start[kL1d];
};

// The drop-in operator's level table, read from device memory: true when it is PDVC's lifted 1-D pyramid (see the
// drop-in kernels below).
__device__ __forceinline__ bool dropin_levels(const int64_t* __restrict__ shapes, const int64_t* __restrict__ lsi, int S,
                                              Levels1d& lv) {
    bool ok = true;
    int64_t st = 0;
#pragma unroll
    for (int l = 0; l < kL1d; ++l) {
        const int64_t h = shapes[2 * l], w = shapes[2 * l + 1];
        ok = ok && h == 1 && w > 0 && lsi[l] == st;
        lv.T[l] = (int)w;
        lv.start[l] = (int)st;
        st += w;
    }
    return ok && st == (int64_t)S;
}

// fp32 -> bf16 bits, round to nearest even -- the conversion of torch's Tensor.to(torch.bfloat16) (c10::BFloat16:
// NaN -> 0x7FC0): a producing kernel that also writes the bf16 rounding of its output (the bf16 mode's GEMM operand,
// pdvc/precision.py attach_bf16) writes exactly the bits the cast pass would have
__device__ __forceinline__ uint32_t bf16_bits(float f) {
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ void store_bf16x4(uint16_t* p, float a, float b, float c, float d) {
    *reinterpret_cast<uint2*>(p) = make_uint2(bf16_bits(a) | (bf16_bits(b) << 16), bf16_bits(c) | (bf16_bits(d) << 16));
}

// Attention dropout mask (mha.hip, seqattn.hip): a counter hash of (seed, video*head, query, key), regenerated in
// the backward; keep with probability 1 - p (24-bit uniform against thresh = p * 2^24).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__device__ __forceinline__ bool keep_elem(uint64_t seed, uint32_t head_idx, uint32_t q, uint32_t k, uint32_t Q,
                                          uint32_t thresh) {
    const uint32_t idx = (head_idx * Q + q) * Q + k;
    const uint32_t h = mix32(mix32(idx ^ (uint32_t)seed) + (uint32_t)(seed >> 32) * 0x9e3779b9U);
    return (h >> 8) >= thresh;
}

// the dropout seed from device memory (drawn inside a captured graph) or the host value
__device__ __forceinline__ uint64_t load_seed(uint64_t seed, const uint64_t* seed_dev) {
    return seed_dev ? *seed_dev : seed;
}

static inline uint32_t drop_threshold(float p) {
    double t = (double)p * 16777216.0;
    if (t < 0) t = 0;
    if (t > 16777216.0) t = 16777216.0;
    return (uint32_t)t;
}

// Zero-fill as a kernel (vector stores).  hipMemsetAsync captured into a hipGraph did not re-zero its buffer
// on replays after the first (tools/diag_refgrad.py: the decoder's atomically accumulated grad_ref kept the
// previous replay's contents); a kernel node replays like every other launch.
template <int V>
__global__ __launch_bounds__(256) void zero_fill_kernel(float* __restrict__ p, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (V == 4) {
        float4* q = reinterpret_cast<float4*>(p);
        for (; i < n / 4; i += stride) q[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
        for (; i < n; i += stride) p[i] = 0.f;
    }
}

static inline hipError_t zero_async(float* p, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    static const bool use_memset = [] {  // diagnosis only (tools/diag_memset_graph.py): the hipMemsetAsync form
        const char* e = getenv("PDVC_ZERO_MEMSET");
        return e && e[0] == '1';
    }();
    if (use_memset) return hipMemsetAsync(p, 0, n * sizeof(float), s);
    const bool vec = ((uintptr_t)p % 16 == 0) && (n % 4 == 0);
    const size_t work = vec ? n / 4 : n;
    const unsigned blocks = (unsigned)(work / 256 + 1 < 8192 ? work / 256 + 1 : 8192);
    if (vec)
        hipLaunchKernelGGL(zero_fill_kernel<4>, dim3(blocks), dim3(256), 0, s, p, n);
    else
        hipLaunchKernelGGL(zero_fill_kernel<1>, dim3(blocks), dim3(256), 0, s, p, n);
    return hipGetLastError();
}

}  // namespace pdvc

// Host-side status plumbing (defined in pdvc_status.cpp).
extern "C" int pdvc_set_error(int code, const char* fmt, ...);
#define PDVC_CHECK_ARG(cond, ...)                                             \
    do {                                                                      \
        if (!(cond)) return pdvc_set_error(PDVC_ERR_INVALID_ARG, __VA_ARGS__); \
    } while (0)
#define PDVC_CHECK_LAUNCH(name)                                                                   \
    do {                                                                                          \
        hipError_t _e = hipGetLastError();                                                        \
        if (_e != hipSuccess)                                                                     \
            return pdvc_set_error(PDVC_ERR_LAUNCH, "%s: launch failed: %s", name, hipGetErrorString(_e)); \
    } while (0)

namespace pdvc {
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) applies to the CURRENT device: the opt-in of a kernel set is made
// once per device and remembered per device (`done`: a zero-initialised static array of kMaxDevices flags).  Two
// threads that race on the first call both set the attribute, which is idempotent; a failure is not remembered.
constexpr int kMaxDevices = 64;
inline int lds_optin(std::atomic<int>* done, std::initializer_list<std::pair<const void*, int>> kernels,
                     const char* what) {
    int dev = -1;
    const bool cacheable = hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDevices;
    if (cacheable && done[dev].load(std::memory_order_acquire)) return PDVC_OK;
    for (const auto& k : kernels)
        if (hipFuncSetAttribute(k.first, hipFuncAttributeMaxDynamicSharedMemorySize, k.second) != hipSuccess) {
            (void)hipGetLastError();
            return pdvc_set_error(PDVC_ERR_LAUNCH, "%s: cannot raise the LDS limit", what);
        }
    if (cacheable) done[dev].store(1, std::memory_order_release);
    return PDVC_OK;
}
}  // namespace pdvc
