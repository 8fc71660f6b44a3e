// lsap.hip -- the Hungarian matching of SetCriterion on the GPU (MI355X, gfx950).
//
// Replaces the host round trip of HungarianMatcher (pdvc/matcher.py:119-121 in the reference: cost matrix
// .cpu() + scipy.optimize.linear_sum_assignment per video).  Every (decoder layer, video) problem is solved
// by one wave with the same algorithm as scipy -- the rectangular shortest augmenting path of Crouse
// (IEEE TAES 2016), float64 duals and path costs evaluated in the same order, the same tie rule -- so the
// matched indices are the ones scipy returns, bit for bit (tests/test_gpu_lsap.py; the plain restatement
// tests/lsap_ref.py is checked against scipy on CPU).  PDVC matches E targets (rows) to Q >= E queries
// (columns): scipy transposes the (Q, E) matrix the same way.  Output per problem: the E matched queries in
// ascending order and their targets -- scipy's (row_ind, col_ind) of the (Q, E) matrix.
//
// Inside a wave: the augmenting-path scan over the remaining columns is split over lanes; the choice of the
// next column is a wave reduction that reproduces the sequential scan's tie rule ("strictly lower, or equal
// and unassigned": the last unassigned column at the minimum if there is one, else the first column at the
// minimum, in scan order); the scalar bookkeeping (remaining-list swap, augmentation) runs on lane 0.
#include "pdvc_common.h"

namespace pdvc {

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(64) void lsap_kernel(const float* __restrict__ costs, int Q, int Emax,
                                                  const int32_t* __restrict__ sizes, int64_t* __restrict__ q_out,
                                                  int64_t* __restrict__ t_out) {
    extern __shared__ __attribute__((aligned(16))) double lds_d[];
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    const int nr = sizes[p], nc = Q;
    // LDS image: doubles first (alignment), then ints, then bytes
    double* u = lds_d;                     // [Emax]
    double* v = u + Emax;                  // [Q]
    double* spc = v + Q;                   // [Q] shortest path costs
    float* cost = (float*)(spc + Q);       // [Emax][Q] cost(row i = target, col j = query)
    int* path = (int*)(cost + (size_t)Emax * Q);  // [Q]
    int* row4col = path + Q;               // [Q]
    int* remaining = row4col + Q;          // [Q]
    int* col4row = remaining + Q;          // [Emax]
    int* scal = col4row + Emax;            // [4]: sink, index, i, num_rem
    uint8_t* SR = (uint8_t*)(scal + 4);    // [Emax]
    uint8_t* SC = SR + Emax;               // [Q]

    const float* cp = costs + (size_t)p * Q * Emax;
    for (int k = lane; k < nr * nc; k += 64) {
        const int i = k / nc, j = k - i * nc;
        cost[i * nc + j] = cp[(size_t)j * Emax + i];
    }
    for (int j = lane; j < nc; j += 64) {
        v[j] = 0.0;
        row4col[j] = -1;
    }
    for (int i = lane; i < nr; i += 64) {
        u[i] = 0.0;
        col4row[i] = -1;
    }
    wave_sync_lds();

    for (int cur = 0; cur < nr; ++cur) {
        // ---- shortest augmenting path from row `cur`
        double min_val = 0.0;
        for (int it = lane; it < nc; it += 64) {
            remaining[it] = nc - it - 1;
            spc[it] = INFINITY;
            SC[it] = 0;
        }
        for (int i = lane; i < nr; i += 64) SR[i] = 0;
        int num_rem = nc;
        int i = cur;
        int sink = -1;
        wave_sync_lds();
        while (sink == -1) {
            if (lane == 0) SR[i] = 1;
            const double ui = u[i];
            // lane-local candidates: minimum value; first position at it; last unassigned position at it
            double best = INFINITY;
            int first_pos = 0x7fffffff, last_unassigned = -1;
            for (int it = lane; it < num_rem; it += 64) {
                const int j = remaining[it];
                const double r = min_val + (double)cost[i * nc + j] - ui - v[j];
                double s = spc[j];
                if (r < s) {
                    path[j] = i;
                    spc[j] = r;
                    s = r;
                }
                const bool un = row4col[j] == -1;
                if (s < best) {
                    best = s;
                    first_pos = it;
                    last_unassigned = un ? it : -1;
                } else if (s == best) {
                    if (it < first_pos) first_pos = it;
                    if (un && it > last_unassigned) last_unassigned = it;
                }
            }
            // wave reduction of (best, first_pos, last_unassigned) under the same rule
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const double ob = __shfl_xor(best, d, 64);
                const int of = __shfl_xor(first_pos, d, 64);
                const int ou = __shfl_xor(last_unassigned, d, 64);
                if (ob < best) {
                    best = ob;
                    first_pos = of;
                    last_unassigned = ou;
                } else if (ob == best) {
                    first_pos = of < first_pos ? of : first_pos;
                    last_unassigned = ou > last_unassigned ? ou : last_unassigned;
                }
            }
            min_val = best;
            const int index = last_unassigned >= 0 ? last_unassigned : first_pos;
            wave_sync_lds();  // path/spc writes of the scan before lane 0 reads them
            if (lane == 0) {
                const int j = remaining[index];
                if (row4col[j] == -1) scal[0] = j;
                else {
                    scal[0] = -1;
                    scal[2] = row4col[j];
                }
                SC[j] = 1;
                remaining[index] = remaining[num_rem - 1];
            }
            wave_sync_lds();
            sink = scal[0];
            if (sink == -1) i = scal[2];
            num_rem -= 1;
        }
        // ---- dual update (rows of the tree, columns scanned), then augmentation along the path
        for (int r = lane; r < nr; r += 64) {
            if (r == cur) u[r] += min_val;
            else if (SR[r]) u[r] += min_val - spc[col4row[r]];
        }
        for (int j = lane; j < nc; j += 64)
            if (SC[j]) v[j] -= min_val - spc[j];
        wave_sync_lds();
        if (lane == 0) {
            int j = sink;
            while (true) {
                const int ii = path[j];
                row4col[j] = ii;
                const int tmp = col4row[ii];
                col4row[ii] = j;
                j = tmp;
                if (ii == cur) break;
            }
        }
        wave_sync_lds();
    }
    // ---- output sorted by query: rank of each row's query among the matched queries (queries are distinct)
    for (int r = lane; r < nr; r += 64) {
        const int q = col4row[r];
        int rank = 0;
        for (int k = 0; k < nr; ++k) rank += col4row[k] < q;
        q_out[(size_t)p * Emax + rank] = q;
        t_out[(size_t)p * Emax + rank] = r;
    }
}

static size_t lsap_lds(int Q, int Emax) {
    return sizeof(double) * (Emax + 2 * (size_t)Q) + sizeof(float) * (size_t)Emax * Q +
           sizeof(int) * (3 * (size_t)Q + Emax + 4) + (size_t)Emax + Q + 16;
}

}  // namespace pdvc

using namespace pdvc;

extern "C" int pdvc_lsap_f32(const float* costs, int num_problems, int num_query, int max_targets,
                             const int32_t* sizes_host, const int32_t* sizes_dev, int64_t* query_out,
                             int64_t* target_out, void* stream) {
    PDVC_CHECK_ARG(num_problems >= 0 && num_query > 0 && max_targets >= 0, "invalid sizes");
    PDVC_CHECK_ARG(sizes_host != nullptr && sizes_dev != nullptr, "sizes (host and device copies) are required");
    for (int p = 0; p < num_problems; ++p)
        PDVC_CHECK_ARG(sizes_host[p] >= 0 && sizes_host[p] <= max_targets && sizes_host[p] <= num_query,
                       "problem %d: %d targets (max %d, and at most the %d queries)", p, sizes_host[p], max_targets,
                       num_query);
    if (num_problems == 0 || max_targets == 0) return PDVC_OK;
    const size_t lds = lsap_lds(num_query, max_targets);
    PDVC_CHECK_ARG(lds <= 160 * 1024, "matching problem too large for LDS (%d queries x %d targets)", num_query,
                   max_targets);
    static std::atomic<int> done[kMaxDevices];
    if (const int rc = lds_optin(done, {{(const void*)lsap_kernel, 160 * 1024}}, "lsap")) return rc;
    hipLaunchKernelGGL(lsap_kernel, dim3((unsigned)num_problems), dim3(64), lds, (hipStream_t)stream, costs, num_query,
                       max_targets, sizes_dev, query_out, target_out);
    PDVC_CHECK_LAUNCH("lsap_kernel");
    return PDVC_OK;
}
