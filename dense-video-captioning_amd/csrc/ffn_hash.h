// ffn_hash.h -- the feed-forward block's dropout keep mask: a counter hash of (seed, row, column), shared by the
// relu + dropout pass (ffn.hip) and the GEMM epilogue that fuses it (gemm3.hip, EPI_BIAS_RELU_DROP), so both
// produce the same mask bit for bit.
#pragma once
#include "pdvc_common.h"

namespace pdvc {

__device__ __forceinline__ uint32_t ffn_mix(uint32_t x) {
    x ^= x >> 16; x *= 0x21f0aaadU; x ^= x >> 15; x *= 0x735a2d97U; x ^= x >> 15;
    return x;
}

// keep with probability 1 - p (24-bit uniform) for element (row, col)
__device__ __forceinline__ bool ffn_keep(uint64_t seed, uint32_t row, uint32_t col, uint32_t thresh) {
    const uint32_t h = ffn_mix(ffn_mix(row * 0x9e3779b1U ^ (uint32_t)seed) + col * 0xc2b2ae35U + (uint32_t)(seed >> 32));
    return (h >> 8) >= thresh;
}

static inline uint32_t ffn_threshold(float p) {
    double t = (double)p * 16777216.0;
    if (t < 0) t = 0;
    if (t > 16777216.0) t = 16777216.0;
    return (uint32_t)t;
}

}  // namespace pdvc
