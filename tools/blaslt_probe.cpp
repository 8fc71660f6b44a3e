// Probe: does hipBLASLt on gfx950 run fp32-in / fp32-out GEMMs with bf16 MFMA compute
// (HIPBLAS_COMPUTE_32F_FAST_16BF), and how fast, on the PDVC step's dominant shapes?
//   hipcc --offload-arch=gfx950 -O2 tools/blaslt_probe.cpp -lhipblaslt -o /tmp/blaslt_probe && /tmp/blaslt_probe
// Row-major C[M,N] = A[M,K] * op(B) is issued as column-major C^T = op(B)^T A^T.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { auto _e = (x); if (_e != 0) { printf("error %d at %s:%d\n", (int)_e, __FILE__, __LINE__); exit(1); } } while (0)

struct Shape { const char* name; long M, N, K; bool transB; };

static double run(hipblasLtHandle_t h, hipblasComputeType_t ct, hipDataType ab, const Shape& s, void* A, void* B,
                  float* C, void* ws, size_t wsz, int* n_algo) {
    // column-major view: C^T (N x M) = opB^T (N x K) * A^T (K x M)
    hipblasLtMatmulDesc_t d;
    CK(hipblasLtMatmulDescCreate(&d, ct, HIP_R_32F));
    hipblasOperation_t ta = s.transB ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    hipblasLtMatrixLayout_t la, lb, lc;
    // first operand (B of the row-major product): row-major (K x N) = col-major (N x K) when !transB;
    // row-major (N x K) (a weight, x @ W^T) = col-major (K x N), transposed
    if (s.transB) CK(hipblasLtMatrixLayoutCreate(&la, ab, s.K, s.N, s.K));
    else CK(hipblasLtMatrixLayoutCreate(&la, ab, s.N, s.K, s.N));
    CK(hipblasLtMatrixLayoutCreate(&lb, ab, s.K, s.M, s.K));
    CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, s.N, s.M, s.N));
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz)));
    hipblasLtMatmulHeuristicResult_t res[8];
    int got = 0;
    hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, d, la, lb, lc, lc, pref, 8, res, &got);
    *n_algo = (st == HIPBLAS_STATUS_SUCCESS) ? got : -1;
    double best = -1;
    float alpha = 1.f, beta = 0.f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < got; ++i) {
        if (hipblasLtMatmul(h, d, &alpha, B, la, A, lb, &beta, C, lc, C, lc, &res[i].algo, ws, wsz, 0) != 0) continue;
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r)
            hipblasLtMatmul(h, d, &alpha, B, la, A, lb, &beta, C, lc, C, lc, &res[i].algo, ws, wsz, 0);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double tf = 2.0 * s.M * s.N * s.K / (ms / reps * 1e-3) / 1e12;
        if (tf > best) best = tf;
    }
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtMatmulDescDestroy(d);
    return best;
}

int main() {
    hipblasLtHandle_t h;
    CK(hipblasLtCreate(&h));
    const Shape shapes[] = {
        {"enc fwd x@W^T 245760x512x512", 245760, 512, 512, true},
        {"enc dgrad dY@W 245760x512x512", 245760, 512, 512, false},
        {"wgrad-like 512x512x245760", 512, 512, 245760, false},
        {"logit 53248x5748x512", 53248, 5748, 512, true},
        {"lstm 53248x2048x1536", 53248, 2048, 1536, true},
    };
    size_t maxe = 0;
    for (auto& s : shapes) {
        maxe = std::max(maxe, (size_t)(s.M * s.K));
        maxe = std::max(maxe, (size_t)(s.K * s.N));
        maxe = std::max(maxe, (size_t)(s.M * s.N));
    }
    void *A, *B, *ws;
    float* C;
    CK(hipMalloc(&A, maxe * 4));
    CK(hipMalloc(&B, maxe * 4));
    CK(hipMalloc(&C, maxe * 4));
    size_t wsz = 128 << 20;
    CK(hipMalloc(&ws, wsz));
    CK(hipMemset(A, 0, maxe * 4));
    CK(hipMemset(B, 0, maxe * 4));
    struct Mode { const char* name; hipblasComputeType_t ct; hipDataType ab; } modes[] = {
        {"f32 in, 32F", HIPBLAS_COMPUTE_32F, HIP_R_32F},
        {"f32 in, 32F_FAST_16BF", HIPBLAS_COMPUTE_32F_FAST_16BF, HIP_R_32F},
        {"bf16 in, 32F", HIPBLAS_COMPUTE_32F, HIP_R_16BF},
    };
    for (auto& s : shapes) {
        for (auto& m : modes) {
            int n = 0;
            double tf = run(h, m.ct, m.ab, s, A, B, C, ws, wsz, &n);
            printf("%-34s %-24s algos %2d  best %8.1f TF/s\n", s.name, m.name, n, tf);
            fflush(stdout);
        }
    }
    return 0;
}
