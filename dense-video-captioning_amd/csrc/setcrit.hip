// setcrit.hip -- the set criterion of the decoder layers as three launches: the matching cost of every (problem,
// query, target) and, after the assignment (lsap.hip), every loss term of every problem with its local gradients,
// combined with the upstream loss gradients by one elementwise pass in the backward.
//
// A problem is one (decoder layer, video) pair; the layers are stacked as Ld * N problems (pdvc/criterion.py).  The
// reference computes each term with a chain of small torch ops per layer (pdvc/criterion.py:46-123 losses,
// pdvc/matcher.py:87-121 cost); here the same per-element arithmetic runs in one workgroup per problem.
//
// The cost kernel repeats the torch expression of HungarianMatcher.cost_padded operation by operation, each rounded to
// fp32 (no FMA contraction); exp, log and the divisions may round differently from torch's kernels, so the costs
// agree to a few ulp and the assignments are the same (tests/test_gpu_setcrit.py checks both; the whole-model
// fixtures check the matched indices against the reference's).  The loss kernel sums in its own order.
#include "pdvc_common.h"

namespace pdvc {

#pragma clang fp contract(off)

__device__ __forceinline__ float sigmoid_t(float x) { return 1.f / (1.f + expf(-x)); }  // torch's sigmoid form

// 1-D generalised IoU of segments (x0, x1) (misc/detr_utils/box_ops.py:21-47), torch's operation order
__device__ __forceinline__ float giou_1d(float a0, float a1, float b0, float b1) {
    const float area1 = a1 - a0, area2 = b1 - b0;
    const float lt = fmaxf(a0, b0), rb = fminf(a1, b1);
    const float inter = fmaxf(rb - lt, 0.f);
    const float uni = (area1 + area2) - inter;
    const float iou = inter / (uni + 1e-5f);
    const float lt2 = fminf(a0, b0), rb2 = fmaxf(a1, b1);
    const float area = fmaxf(rb2 - lt2, 0.f);
    return iou - (area - uni) / (area + 1e-5f);
}

// cost[p, q, e] = w_bbox * L1(box, tbox) + w_class * (pos - neg)[label] + w_giou * (-GIoU)   (matcher.py:87-121)
__global__ __launch_bounds__(256) void match_cost_kernel(const float* __restrict__ logits, const float* __restrict__ boxes,
                                                         const int64_t* __restrict__ labels,
                                                         const float* __restrict__ tboxes, int P, int Q, int C, int E,
                                                         float alpha, float one_m_alpha, float gamma, float w_bbox,
                                                         float w_class, float w_giou, float* __restrict__ cost) {
    const long total = (long)P * Q * E;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int e = (int)(i % E);
        const long pq = i / E;
        const int p = (int)(pq / Q);
        const int lab = (int)labels[(size_t)p * E + e];
        const float prob = sigmoid_t(logits[(size_t)pq * C + lab]);
        // neg = (1 - alpha) * prob ** gamma * (-(1 - prob + 1e-8).log());  pos = alpha * (1 - prob) ** gamma * (-(prob + 1e-8).log())
        const float pg = gamma == 2.f ? prob * prob : powf(prob, gamma);
        const float q1 = 1.f - prob;
        const float qg = gamma == 2.f ? q1 * q1 : powf(q1, gamma);
        const float neg = (one_m_alpha * pg) * (-logf(q1 + 1e-8f));
        const float pos = (alpha * qg) * (-logf(prob + 1e-8f));
        const float c_class = pos - neg;
        const float pc = boxes[(size_t)pq * 2], pl = boxes[(size_t)pq * 2 + 1];
        const float tc = tboxes[((size_t)p * E + e) * 2], tl = tboxes[((size_t)p * E + e) * 2 + 1];
        const float c_bbox = fabsf(pc - tc) + fabsf(pl - tl);
        const float c_giou = -giou_1d(pc - 0.5f * pl, pc + 0.5f * pl, tc - 0.5f * tl, tc + 0.5f * tl);
        cost[i] = (w_bbox * c_bbox + w_class * c_class) + w_giou * c_giou;
    }
}

// d max(a, b) / da, torch's convention: 1 where a > b, 1/2 at a tie
__device__ __forceinline__ float dmax_a(float a, float b) { return a > b ? 1.f : (a == b ? 0.5f : 0.f); }
__device__ __forceinline__ float dmin_a(float a, float b) { return a < b ? 1.f : (a == b ? 0.5f : 0.f); }

// gradient of iou(a, b) (box_iou) with respect to a = (a0, a1) and b = (b0, b1), upstream g
__device__ __forceinline__ void iou_grad(float a0, float a1, float b0, float b1, float g, float& ga0, float& ga1,
                                         float& gb0, float& gb1) {
    const float area1 = a1 - a0, area2 = b1 - b0;
    const float lt = fmaxf(a0, b0), rb = fminf(a1, b1);
    const float w = rb - lt;
    const float inter = fmaxf(w, 0.f);
    const float uni = (area1 + area2) - inter;
    const float d = uni + 1e-5f;
    float g_inter = g / d;
    const float g_u = -g * inter / (d * d);
    g_inter -= g_u;
    const float g_w = w >= 0.f ? g_inter : 0.f;  // clamp(min=0) passes at 0
    ga0 = -g_w * dmax_a(a0, b0) - g_u;
    gb0 = -g_w * dmax_a(b0, a0) - g_u;
    ga1 = g_w * dmin_a(a1, b1) + g_u;
    gb1 = g_w * dmin_a(b1, a1) + g_u;
}

// gradient of giou(a, b) with respect to a, upstream g
__device__ __forceinline__ void giou_grad_a(float a0, float a1, float b0, float b1, float g, float& ga0, float& ga1) {
    const float area1 = a1 - a0, area2 = b1 - b0;
    const float lt = fmaxf(a0, b0), rb = fminf(a1, b1);
    const float w = rb - lt;
    const float inter = fmaxf(w, 0.f);
    const float uni = (area1 + area2) - inter;
    const float d = uni + 1e-5f;
    const float lt2 = fminf(a0, b0), rb2 = fmaxf(a1, b1);
    const float w2 = rb2 - lt2;
    const float area = fmaxf(w2, 0.f);
    const float da = area + 1e-5f;
    // giou = inter / d - (area - uni) / da
    const float g_h = -g;
    const float g_area = g_h * (1.f / da - (area - uni) / (da * da));
    float g_u = g_h * (-1.f / da);
    float g_inter = g / d;
    g_u += g * (-inter / (d * d));
    g_inter -= g_u;
    const float g_w = w >= 0.f ? g_inter : 0.f;
    const float g_w2 = w2 >= 0.f ? g_area : 0.f;
    ga0 = -g_w * dmax_a(a0, b0) - g_w2 * dmin_a(a0, b0) - g_u;
    ga1 = g_w * dmin_a(a1, b1) + g_w2 * dmax_a(a1, b1) + g_u;
}

constexpr int kSetThreads = 256;
constexpr int kSetMaxE = 64;  // matched pairs per problem held in LDS

__device__ __forceinline__ float block_sum(float v, float* red) {
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kSetThreads / 64; ++w) t += red[w];
    return t;
}

// One workgroup per problem p.  losses[p, :] = (ce, counter, bbox, giou, self_iou, cardinality error) as
// SetCriterion.video_losses (criterion.py:46-123, 200-248): focal loss over every (query, class) / num_boxes, the
// Gaussian-masked counter BCE, L1 and 1 - GIoU of the matched pairs / num_boxes, the mean IoU among the matched
// predictions (upper triangle / (n (n - 1) / 2)), |#queries whose argmax is not the last class - n|.
// Local gradients: dlogit (P, Q, C) of ce, dcount (P, K1) of counter, dbox (3, P, Q, 2) of bbox / giou / self_iou.
// mq / mt (P, E): matched query and target of each rank (the device assignment), n = nmatch[p] ranks used (the true
// target count: phantom ranks of a capacity-padded batch are ignored); qmask (P, Q) or null: proposal slots.
__global__ __launch_bounds__(kSetThreads) void set_losses_kernel(
    const float* __restrict__ logits, const float* __restrict__ boxes, const float* __restrict__ count,
    const int64_t* __restrict__ labels, const float* __restrict__ tboxes, const int64_t* __restrict__ nmatch,
    const float* __restrict__ nbox, const int64_t* __restrict__ mq, const int64_t* __restrict__ mt,
    const uint8_t* __restrict__ qmask, const float* __restrict__ rate, int P, int Q, int C, int E, int K1,
    float focal_alpha, float focal_gamma, int gau_mask, float beta, float* __restrict__ losses,
    float* __restrict__ dlogit, float* __restrict__ dcount, float* __restrict__ dbox) {
    extern __shared__ int tcls[];  // [Q] target class of every query (C: none)
    __shared__ float red[kSetThreads / 64];
    __shared__ float sx0[kSetMaxE], sx1[kSetMaxE];
    __shared__ int sq[kSetMaxE];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int n = (int)min((int64_t)min(E, kSetMaxE), nmatch[p]);
    const float nb = nbox[p];
    const float inv_nb = 1.f / nb;
    for (int q = tid; q < Q; q += kSetThreads) tcls[q] = C;
    __syncthreads();
    if (tid < n) {
        const int q = (int)mq[(size_t)p * E + tid];
        tcls[q] = (int)labels[(size_t)p * E + mt[(size_t)p * E + tid]];
    }
    __syncthreads();
    // focal loss and its gradient over every (query, class); the cardinality count
    float ce = 0.f, card = 0.f;
    const float ag = focal_alpha;
    for (int q = tid; q < Q; q += kSetThreads) {
        const bool in = qmask == nullptr || qmask[(size_t)p * Q + q];
        const float* lrow = logits + ((size_t)p * Q + q) * C;
        int am = 0;
        float best = lrow[0];
        for (int c = 0; c < C; ++c) {
            const float x = lrow[c];
            if (x > best) {
                best = x;
                am = c;
            }
            const float t = tcls[q] == c ? 1.f : 0.f;
            const float pr = sigmoid_t(x);
            // binary_cross_entropy_with_logits: max(x, 0) - x t + log(1 + exp(-|x|))
            const float bce = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
            const float pt = pr * t + (1.f - pr) * (1.f - t);
            const float om = 1.f - pt;
            const float m = focal_gamma == 2.f ? om * om : powf(om, focal_gamma);
            const float at = ag >= 0.f ? ag * t + (1.f - ag) * (1.f - t) : 1.f;
            const float l = at * bce * m;
            // d/dx: at (dbce m + bce dm), dbce = pr - t, dm = -gamma om^(gamma-1) dpt, dpt = pr (1 - pr) (2t - 1)
            const float dpt = pr * (1.f - pr) * (2.f * t - 1.f);
            const float dm = -(focal_gamma == 2.f ? 2.f * om : focal_gamma * powf(om, focal_gamma - 1.f)) * dpt;
            const float g = at * ((pr - t) * m + bce * dm);
            if (in) ce += l;
            dlogit[((size_t)p * Q + q) * C + c] = in ? g * inv_nb : 0.f;
        }
        if (in && am != C - 1) card += 1.f;
    }
    // counter (criterion.py:200-220): BCE with weight 1 - rate, Gaussian-masked negatives, mean over K1
    float cnt = 0.f;
    {
        const int ct = (int)min(nmatch[p], (int64_t)(K1 - 1));  // the true event count, capped at max_length
        for (int k = tid; k < K1; k += kSetThreads) {
            const float x = count[(size_t)p * K1 + k];
            const float t = k == ct ? 1.f : 0.f;
            const float w = 1.f - rate[k];
            const float dk = (float)(k - ct);
            const float msk = expf(-(dk * dk) / 8.f);
            const float coef = gau_mask ? t + powf(1.f - msk, beta) * (1.f - t) : t + (1.f - t);
            const float bce = w * (fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x))));
            cnt += bce * coef;
            dcount[(size_t)p * K1 + k] = w * (sigmoid_t(x) - t) * coef / (float)K1;
        }
    }
    // matched pairs: L1 and 1 - GIoU (criterion.py:94-112); box gradients zero for unmatched queries
    float* dl1 = dbox;
    float* dgi = dbox + (size_t)P * Q * 2;
    float* dsi = dbox + 2 * (size_t)P * Q * 2;
    for (int q = tid; q < Q; q += kSetThreads) {
        const size_t o = ((size_t)p * Q + q) * 2;
        dl1[o] = dl1[o + 1] = dgi[o] = dgi[o + 1] = dsi[o] = dsi[o + 1] = 0.f;
    }
    __syncthreads();
    float l1s = 0.f, gis = 0.f;
    if (tid < n) {
        const int q = (int)mq[(size_t)p * E + tid];
        const int e = (int)mt[(size_t)p * E + tid];
        const float sc = boxes[((size_t)p * Q + q) * 2], sl = boxes[((size_t)p * Q + q) * 2 + 1];
        const float tc = tboxes[((size_t)p * E + e) * 2], tl = tboxes[((size_t)p * E + e) * 2 + 1];
        l1s = fabsf(sc - tc) + fabsf(sl - tl);
        const float a0 = sc - 0.5f * sl, a1 = sc + 0.5f * sl, b0 = tc - 0.5f * tl, b1 = tc + 0.5f * tl;
        gis = 1.f - giou_1d(a0, a1, b0, b1);
        const size_t o = ((size_t)p * Q + q) * 2;
        const float sgc = sc > tc ? 1.f : (sc < tc ? -1.f : 0.f), sgl = sl > tl ? 1.f : (sl < tl ? -1.f : 0.f);
        dl1[o] = sgc * inv_nb;
        dl1[o + 1] = sgl * inv_nb;
        float g0, g1;
        giou_grad_a(a0, a1, b0, b1, -inv_nb, g0, g1);  // d(1 - giou) / nb
        dgi[o] = g0 + g1;
        dgi[o + 1] = 0.5f * (g1 - g0);
        sx0[tid] = a0;
        sx1[tid] = a1;
        sq[tid] = q;
    }
    __syncthreads();
    // self-IoU among the matched predictions (criterion.py:113-121): sum over rank pairs i < j / (n (n - 1) / 2)
    float sis = 0.f;
    const float den = 0.5f * (float)n * (float)(n - 1);
    if (tid < n) {
        float g0 = 0.f, g1 = 0.f;
        const float a0 = sx0[tid], a1 = sx1[tid];
        for (int j = 0; j < n; ++j) {
            if (j == tid) continue;
            const float b0 = sx0[j], b1 = sx1[j];
            float ga0, ga1, gb0, gb1;
            if (j > tid) {  // pair (tid, j): this box is the row
                const float area1 = a1 - a0, area2 = b1 - b0;
                const float inter = fmaxf(fminf(a1, b1) - fmaxf(a0, b0), 0.f);
                const float uni = (area1 + area2) - inter;
                sis += inter / (uni + 1e-5f);
                iou_grad(a0, a1, b0, b1, 1.f / den, ga0, ga1, gb0, gb1);
                g0 += ga0;
                g1 += ga1;
            } else {  // pair (j, tid): this box is the column
                iou_grad(b0, b1, a0, a1, 1.f / den, ga0, ga1, gb0, gb1);
                g0 += gb0;
                g1 += gb1;
            }
        }
        const size_t o = ((size_t)p * Q + sq[tid]) * 2;
        dsi[o] = g0 + g1;
        dsi[o + 1] = 0.5f * (g1 - g0);
    }
    ce = block_sum(ce, red);
    card = block_sum(card, red);
    cnt = block_sum(cnt, red);
    l1s = block_sum(l1s, red);
    gis = block_sum(gis, red);
    sis = block_sum(sis, red);
    if (tid == 0) {
        float* lo = losses + (size_t)p * 6;
        lo[0] = ce / nb;
        lo[1] = cnt / (float)K1;
        lo[2] = l1s / nb;
        lo[3] = gis / nb;
        lo[4] = sis / den;
        lo[5] = fabsf(card - (float)nmatch[p]);
    }
}

// backward: dlogits = g[p,0] dlogit, dcount = g[p,1] dcount, dboxes = g[p,2] dl1 + g[p,3] dgiou + g[p,4] dself_iou
__global__ __launch_bounds__(256) void set_losses_bwd_kernel(const float* __restrict__ g, const float* __restrict__ dlogit,
                                                             const float* __restrict__ dcount,
                                                             const float* __restrict__ dbox, int P, int Q, int C, int K1,
                                                             float* __restrict__ glogits, float* __restrict__ gcount,
                                                             float* __restrict__ gboxes) {
    const long nl = (long)P * Q * C, nc = (long)P * K1, nbx = (long)P * Q * 2;
    const long total = nl + nc + nbx;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        if (i < nl) {
            const long p = i / ((long)Q * C);
            glogits[i] = g[p * 6] * dlogit[i];
        } else if (i < nl + nc) {
            const long j = i - nl, p = j / K1;
            gcount[j] = g[p * 6 + 1] * dcount[j];
        } else {
            const long j = i - nl - nc, p = j / ((long)Q * 2);
            gboxes[j] = g[p * 6 + 2] * dbox[j] + g[p * 6 + 3] * dbox[nbx + j] + g[p * 6 + 4] * dbox[2 * nbx + j];
        }
    }
}

}  // namespace pdvc

using namespace pdvc;

extern "C" int pdvc_match_cost_f32(const float* logits, const float* boxes, const int64_t* labels, const float* tboxes,
                                   int P, int Q, int C, int E, float alpha, float one_minus_alpha, float gamma,
                                   float w_bbox, float w_class, float w_giou, float* cost, void* stream) {
    PDVC_CHECK_ARG(P >= 0 && Q > 0 && C > 0 && E >= 0, "match cost: invalid sizes");
    const long total = (long)P * Q * E;
    if (total == 0) return PDVC_OK;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 65535 ? (total + 255) / 256 : 65535);
    hipLaunchKernelGGL(match_cost_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, logits, boxes, labels,
                       tboxes, P, Q, C, E, alpha, one_minus_alpha, gamma, w_bbox, w_class, w_giou, cost);
    PDVC_CHECK_LAUNCH("match_cost_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_set_losses_f32(const float* logits, const float* boxes, const float* count, const int64_t* labels,
                                   const float* tboxes, const int64_t* nmatch, const float* num_boxes,
                                   const int64_t* match_query, const int64_t* match_target, const uint8_t* query_mask,
                                   const float* counter_rate, int P, int Q, int C, int E, int K1, float focal_alpha,
                                   float focal_gamma, int gau_mask, float beta, float* losses, float* dlogit,
                                   float* dcount, float* dbox, void* stream) {
    PDVC_CHECK_ARG(P >= 0 && Q > 0 && C > 0 && E >= 0 && K1 > 0, "set losses: invalid sizes");
    PDVC_CHECK_ARG(E <= kSetMaxE, "set losses: at most %d targets per problem, got %d", kSetMaxE, E);
    if (P == 0) return PDVC_OK;
    hipLaunchKernelGGL(set_losses_kernel, dim3((unsigned)P), dim3(kSetThreads), sizeof(int) * (size_t)Q,
                       (hipStream_t)stream, logits, boxes, count, labels, tboxes, nmatch, num_boxes, match_query,
                       match_target, query_mask, counter_rate, P, Q, C, E, K1, focal_alpha, focal_gamma, gau_mask, beta,
                       losses, dlogit, dcount, dbox);
    PDVC_CHECK_LAUNCH("set_losses_kernel");
    return PDVC_OK;
}

extern "C" int pdvc_set_losses_backward_f32(const float* grad_losses, const float* dlogit, const float* dcount,
                                            const float* dbox, int P, int Q, int C, int K1, float* grad_logits,
                                            float* grad_count, float* grad_boxes, void* stream) {
    const long total = (long)P * (Q * C + K1 + Q * 2);
    if (total == 0) return PDVC_OK;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 65535 ? (total + 255) / 256 : 65535);
    hipLaunchKernelGGL(set_losses_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, grad_losses, dlogit,
                       dcount, dbox, P, Q, C, K1, grad_logits, grad_count, grad_boxes);
    PDVC_CHECK_LAUNCH("set_losses_bwd_kernel");
    return PDVC_OK;
}
