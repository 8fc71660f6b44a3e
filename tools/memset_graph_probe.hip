// Probe: is a hipMemsetAsync captured into a hipGraph re-applied on every replay?
// Capture: memset(buf, 0) -> kernel adds 1 to each element (vector stores of buf[i] + 1).  Replay 3 times and
// read buf after each: 1, 1, 1 if the memset node replays; 1, 2, 3 if it does not.  Small sizes and large.
//   hipcc --offload-arch=gfx950 -O2 tools/memset_graph_probe.hip -o tools/memset_graph_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void add_one(float* p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] + 1.f;
}

int main() {
    const int sizes[] = {40, 160, 4096, 1 << 20};
    hipStream_t s;
    hipStreamCreate(&s);
    for (int n : sizes) {
        float* d;
        hipMalloc(&d, n * sizeof(float));
        hipMemset(d, 0x7f, n * sizeof(float));  // junk before capture
        hipDeviceSynchronize();
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        hipMemsetAsync(d, 0, n * sizeof(float), s);
        add_one<<<(n + 255) / 256, 256, 0, s>>>(d, n);
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        printf("n=%8d:", n);
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
        hipFree(d);
    }
    return 0;
}
