// an_hash.h -- the residual sub-layers' dropout keep mask: a counter hash of (seed, row, column), shared by the
// add + dropout + LayerNorm passes (addnorm.hip) and the GEMM epilogue that forms x + dropout(y + b) for them
// (gemm3.hip, EPI_RESID_DROP), so both produce the same mask bit for bit.
#pragma once
#include "pdvc_common.h"

namespace pdvc {

__device__ __forceinline__ uint32_t an_mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// the row part of an_keep's hash (once per row where a caller walks a row's columns)
__device__ __forceinline__ uint32_t an_row(uint64_t seed, uint32_t row) { return an_mix(row * 0x9e3779b9U ^ (uint32_t)seed); }
// the column part
__device__ __forceinline__ uint32_t an_col(uint64_t seed, uint32_t col) { return col * 0x85ebca6bU + (uint32_t)(seed >> 32); }

// keep with probability 1 - p: 24-bit uniform from (seed, row, col)
__device__ __forceinline__ bool an_keep(uint64_t seed, uint32_t row, uint32_t col, uint32_t thresh) {
    return (an_mix(an_row(seed, row) + an_col(seed, col)) >> 8) >= thresh;
}

static inline uint32_t an_threshold(float p) {
    double t = (double)p * 16777216.0;
    if (t < 0) t = 0;
    if (t > 16777216.0) t = 16777216.0;
    return (uint32_t)t;
}

}  // namespace pdvc
