// Probe 2 (round 3): does a captured hipMemsetAsync keep its place in the graph order on every replay?
// tools/diag_memset_graph.py found, in the failing step graph, the memset node correctly ordered by its edges:
// earlier kernels had used the same memory (the caching allocator reuses it) and the accumulating kernel follows the
// memset -- yet from replay 1 the accumulator read the earlier kernels' values.  Capture here, on one stream:
//   `chain` dummy kernels (other memory) -> write(buf, 5) -> memset(buf, 0, 160 B) -> add_one(buf)
// and replay 3 times: 1 every time if the memset runs between the writer and the adder; 6 if it runs before the
// writer (hoisted); 1, 2, 3 if it is skipped.
//   hipcc --offload-arch=gfx950 -O2 tools/memset_graph_probe2.hip -o tools/memset_graph_probe2.bin
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void fill(float* p, int n, float v, int spin) {
    // spin: a slow writer (~spin x 64 cycles of s_sleep) -- if the memset does not wait for it, the write lands last
    for (int k = 0; k < spin; ++k) __builtin_amdgcn_s_sleep(1);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void add_one(float* p, int n) {  // (n elements, one thread each)
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] + 1.f;
}
__global__ void dummy(float* p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.5f + 1.f;
}

int main() {
    const int chains[] = {0, 10, 800};
    const int spins[] = {0, 20000};
    const int sizes[] = {40, 1200, 262144};
    hipStream_t s;
    hipStreamCreate(&s);
    float* other;
    hipMalloc(&other, 4096 * sizeof(float));
    for (int n : sizes)
    for (int spin : spins)
    for (int chain : chains) {
        float* d;
        hipMalloc(&d, n * sizeof(float));
        for (int bytewise = 0; bytewise < 2; ++bytewise) {
            hipMemset(d, 0x7f, n * sizeof(float));
            hipDeviceSynchronize();
            hipGraph_t g;
            hipGraphExec_t ge;
            hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
            for (int c = 0; c < chain; ++c) dummy<<<16, 256, 0, s>>>(other, 4096);
            fill<<<(n + 255) / 256, 256, 0, s>>>(d, n, 5.f, spin);
            if (bytewise)
                hipMemsetAsync(d, 0, n * sizeof(float), s);  // byte memset (elementSize 1 node)
            else
                hipMemsetD32Async((hipDeviceptr_t)d, 0, n, s);
            add_one<<<(n + 255) / 256, 256, 0, s>>>(d, n);
            hipStreamEndCapture(s, &g);
            hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            printf("n %6d spin %5d chain %4d %s:", n, spin, chain, bytewise ? "memset8 " : "memsetD32");
            for (int r = 0; r < 3; ++r) {
                hipGraphLaunch(ge, s);
                hipStreamSynchronize(s);
                float h0, h1;
                hipMemcpy(&h0, d, sizeof(float), hipMemcpyDeviceToHost);
                hipMemcpy(&h1, d + n - 1, sizeof(float), hipMemcpyDeviceToHost);
                printf("  replay %d: %g %g", r, h0, h1);
            }
            printf("\n");
            hipGraphExecDestroy(ge);
            hipGraphDestroy(g);
        }
        hipFree(d);
    }
    hipFree(other);
    return 0;
}
