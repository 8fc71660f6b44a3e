// Probe: does DPP row_newbcast:k (dpp_ctrl 0x150 + k) broadcast lane k of each 16-lane row to the whole row for a
// 32-bit v_mov_b32_dpp on gfx950?  Prints, for k = 0..15, the number of lanes whose result differs from the
// expected value (the source lane's value).  Build: hipcc --offload-arch=gfx950 -O2 dpp_newbcast_probe.hip -o probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__global__ void bcast(const int* in, int* out) {
    const int v = in[threadIdx.x];
    out[threadIdx.x] = __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xF, 0xF, false);
}

int main() {
    int h[64], r[64];
    for (int i = 0; i < 64; ++i) h[i] = 1000 + i * 7;
    int *din, *dout;
    if (hipMalloc(&din, 256) != hipSuccess || hipMalloc(&dout, 256) != hipSuccess) return 1;
    hipMemcpy(din, h, 256, hipMemcpyHostToDevice);
    int bad_total = 0;
#define RUN(K)                                                                         \
    {                                                                                  \
        hipLaunchKernelGGL(bcast<K>, dim3(1), dim3(64), 0, 0, din, dout);              \
        hipMemcpy(r, dout, 256, hipMemcpyDeviceToHost);                                \
        int bad = 0;                                                                   \
        for (int i = 0; i < 64; ++i) bad += r[i] != h[(i & ~15) + K];                  \
        printf("row_newbcast:%d  mismatching lanes %d  (lane 5 got %d, want %d)\n", K, bad, r[5], h[K]); \
        bad_total += bad;                                                              \
    }
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7)
    RUN(8) RUN(9) RUN(10) RUN(11) RUN(12) RUN(13) RUN(14) RUN(15)
    printf("%s\n", bad_total ? "row_newbcast is NOT a 16-lane broadcast here" : "row_newbcast = 16-lane broadcast");
    return 0;
}
