// pdvc_common.h -- shared device helpers for the PDVC HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
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

// Sum over aligned groups of G lanes (G power of two <= 64) with xor butterflies.
template <int G>
__device__ __forceinline__ float group_allreduce(float v) {
#pragma unroll
    for (int d = G >> 1; d > 0; d >>= 1) v += __shfl_xor(v, d, PDVC_WAVE);
    return v;
}

// Transposed (reduce-scatter) butterfly inside aligned groups of G lanes: every lane enters with K
// partial values; after log2(G) halving steps lane r (= lane % G) holds the FULL group sums of the
// K/G consecutive values [r*K/G, (r+1)*K/G).  Costs K/2 + K/4 + ... shuffles instead of K*log2(G).
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
                const float recv = __shfl_xor(send, d, PDVC_WAVE);
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
