// Probe 3 (round 3): hipMemsetAsync captured into a graph -- what node does it become, and does it survive EAGER work
// between replays?  tools/diag_memset_graph.py found the failing step graph (PDVC_ZERO_MEMSET=1) holding ONE memset
// node for dozens of captured hipMemsetAsync calls: the others were captured as kernel nodes of HIP's own fill kernels.
// Here: capture  fill(buf, 5) -> hipMemsetAsync(buf, 0) -> add_one(buf), list the graph's node types, then replay 3
// times with eager launches between the replays (hipMemsetAsync on other buffers, a kernel) -- as the training step
// does (optimizer, clipping).  1 after every replay if the captured zero-fill holds; 6 if it did not run.
//   hipcc --offload-arch=gfx950 -O2 tools/memset_graph_probe3.hip -o tools/memset_graph_probe3.bin
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void fill(float* p, int n, float v) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void add_one(float* p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] + 1.f;
}

int main() {
    const int sizes[] = {40, 400, 1200, 4096, 262144};
    hipStream_t s;
    hipStreamCreate(&s);
    float* other;
    const int on = 1 << 22;
    hipMalloc(&other, on * sizeof(float));
    for (int n : sizes)
    for (int eager = 0; eager <= 64; eager += 64) {
        float* d;
        hipMalloc(&d, n * sizeof(float));
        hipMemset(d, 0x7f, n * sizeof(float));
        hipDeviceSynchronize();
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        fill<<<(n + 255) / 256, 256, 0, s>>>(d, n, 5.f);
        hipMemsetAsync(d, 0, n * sizeof(float), s);
        add_one<<<(n + 255) / 256, 256, 0, s>>>(d, n);
        hipStreamEndCapture(s, &g);
        size_t nn = 0;
        hipGraphGetNodes(g, nullptr, &nn);
        hipGraphNode_t nodes[16];
        hipGraphGetNodes(g, nodes, &nn);
        printf("n %6d eager %2d nodes:", n, eager);
        for (size_t k = 0; k < nn && k < 16; ++k) {
            hipGraphNodeType t;
            hipGraphNodeGetType(nodes[k], &t);
            printf(" %d", (int)t);
        }
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        printf(" |");
        for (int r = 0; r < 3; ++r) {
            hipGraphLaunch(ge, s);
            hipStreamSynchronize(s);
            float h0, h1;
            hipMemcpy(&h0, d, sizeof(float), hipMemcpyDeviceToHost);
            hipMemcpy(&h1, d + n - 1, sizeof(float), hipMemcpyDeviceToHost);
            printf(" replay %d: %g %g", r, h0, h1);
            for (int e = 0; e < eager; ++e) {  // eager work between the replays: zero-fills of other sizes, a kernel
                hipMemsetAsync(other, 0, (size_t)(((e * 7919) % 4096) + 1) * 4 * 16, s);
                fill<<<64, 256, 0, s>>>(other, 16384, (float)e);
            }
            hipStreamSynchronize(s);
        }
        printf("\n");
        hipGraphExecDestroy(ge);
        hipGraphDestroy(g);
        hipFree(d);
    }
    hipFree(other);
    return 0;
}
