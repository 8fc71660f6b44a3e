// seqattn.h -- the flash-style MFMA attention of seqattn.hip, shared with mha.hip (its route for query sets
// longer than the single-workgroup MFMA kernel holds).  Internal: not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdvc {

bool sq_head_dim_ok(int D);

// out = softmax(scale q.k^T [-inf at kpm != 0 keys]) with dropout(p) on the probabilities (keep_elem mask),
// times v; lse (N, H, Tq) natural log-sum-exp of the scaled, masked scores.
int sq_forward(const float* q, long ldq, const float* k, long ldk, const float* v, long ldv, int batch,
               int num_query, int num_key, int num_heads, int head_dim, float scale, const uint8_t* kpm,
               float dropout_p, uint64_t seed, const uint64_t* seed_dev, float* out, float* lse, hipStream_t s);

// workspace: batch * num_heads * num_query floats
int sq_backward(const float* q, long ldq, const float* k, long ldk, const float* v, long ldv, const float* out,
                const float* grad_out, const float* lse, int batch, int num_query, int num_key, int num_heads,
                int head_dim, float scale, const uint8_t* kpm, float dropout_p, uint64_t seed,
                const uint64_t* seed_dev, float* workspace, float* grad_q, long ld_grad_q, float* grad_k,
                long ld_grad_k, float* grad_v, long ld_grad_v, hipStream_t s);

}  // namespace pdvc
