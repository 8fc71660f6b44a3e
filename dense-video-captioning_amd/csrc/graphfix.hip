// graphfix.hip -- rewrites the memset nodes of a captured hipGraph as kernel nodes, before instantiation.
//
// A small captured memset node does not re-apply on every replay on this ROCm stack: tools/memset_torch_probe.py
// captures fill(5) -> hipMemsetAsync(160 B) -> add(1) on torch-allocated memory and finds the first element at 3073
// instead of 1 from the second replay on, after eager work between replays (larger memsets, and hipMalloc'd buffers
// in plain HIP, re-apply: tools/memset_graph_probe2/3.hip).  torch's multi-block reductions zero their semaphores with
// such tiny memsets (4-32 B), and the 1024-video training step graph holds 11 of them: replays after the first
// produced garbage in the gradients those reductions form (tools/check_graph_replays.py).  Every library zero-fill
// of ours is a kernel already (zero_async, pdvc_common.h); this pass gives torch's memsets the same treatment in the
// captured graph: each 1-D memset node becomes a kernel node that writes the same value over the same bytes, with the
// same dependencies.  Pitched (2-D) memsets are rewritten the same way; a node this pass cannot rewrite is an error,
// never a silently kept memset.
#include <vector>

#include "pdvc_common.h"

namespace pdvc {

// width elements of esize bytes per row, `height` rows `pitch` bytes apart (a 1-D memset: height 1)
__global__ __launch_bounds__(256) void memset_node_kernel(char* dst, size_t width, size_t height, size_t pitch,
                                                          uint32_t value, int esize) {
    const size_t count = width * height;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / width, c = i - r * width;
        char* at = dst + r * pitch + c * (size_t)esize;
        if (esize == 4)
            *reinterpret_cast<uint32_t*>(at) = value;
        else if (esize == 2)
            *reinterpret_cast<uint16_t*>(at) = (uint16_t)value;
        else
            *reinterpret_cast<uint8_t*>(at) = (uint8_t)value;
    }
}

}  // namespace pdvc

using namespace pdvc;

extern "C" int pdvc_graph_replace_memsets(void* graph, int* replaced) {
    PDVC_CHECK_ARG(graph != nullptr, "graph is NULL");
    hipGraph_t g = (hipGraph_t)graph;
    size_t n = 0;
    if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "hipGraphGetNodes");
    std::vector<hipGraphNode_t> nodes(n);
    if (n && hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess)
        return pdvc_set_error(PDVC_ERR_LAUNCH, "hipGraphGetNodes");
    int done = 0;
    for (hipGraphNode_t node : nodes) {
        hipGraphNodeType t;
        if (hipGraphNodeGetType(node, &t) != hipSuccess || t != hipGraphNodeTypeMemset) continue;
        hipMemsetParams p;
        if (hipGraphMemsetNodeGetParams(node, &p) != hipSuccess)
            return pdvc_set_error(PDVC_ERR_LAUNCH, "hipGraphMemsetNodeGetParams");
        if (p.elementSize != 1 && p.elementSize != 2 && p.elementSize != 4)
            return pdvc_set_error(PDVC_ERR_INVALID_ARG, "memset node with element size %u: not rewritable",
                                  (unsigned)p.elementSize);
        size_t nd = 0, no = 0;
        (void)hipGraphNodeGetDependencies(node, nullptr, &nd);
        (void)hipGraphNodeGetDependentNodes(node, nullptr, &no);
        std::vector<hipGraphNode_t> deps(nd), outs(no);
        if (nd) (void)hipGraphNodeGetDependencies(node, deps.data(), &nd);
        if (no) (void)hipGraphNodeGetDependentNodes(node, outs.data(), &no);
        char* dst = static_cast<char*>(p.dst);
        size_t width = p.width, height = p.height ? p.height : 1;
        size_t pitch = height > 1 ? p.pitch : width * p.elementSize;
        uint32_t value = p.value;
        int esize = (int)p.elementSize;
        const size_t count = width * height;
        void* args[] = {&dst, &width, &height, &pitch, &value, &esize};
        hipKernelNodeParams kp{};
        kp.func = reinterpret_cast<void*>(memset_node_kernel);
        const size_t blocks = (count + 255) / 256;
        kp.gridDim = dim3((unsigned)(blocks < 4096 ? (blocks ? blocks : 1) : 4096));
        kp.blockDim = dim3(256);
        kp.sharedMemBytes = 0;
        kp.kernelParams = args;
        kp.extra = nullptr;
        hipGraphNode_t kn;
        if (hipGraphAddKernelNode(&kn, g, nd ? deps.data() : nullptr, nd, &kp) != hipSuccess)
            return pdvc_set_error(PDVC_ERR_LAUNCH, "hipGraphAddKernelNode");
        for (hipGraphNode_t o : outs)
            if (hipGraphAddDependencies(g, &kn, &o, 1) != hipSuccess)
                return pdvc_set_error(PDVC_ERR_LAUNCH, "hipGraphAddDependencies");
        if (hipGraphDestroyNode(node) != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "hipGraphDestroyNode");
        ++done;
    }
    if (replaced) *replaced = done;
    return PDVC_OK;
}

// Events a captured graph records for work outside it (pdvc/distributed.py, the data-parallel overlap): torch's ROCm
// build refuses torch.cuda.Event(external=True), so the step graph records these directly.  Recorded with
// hipEventRecordExternal on a capturing stream, the record becomes an event-record node of the graph, and every
// replay records the event when the node's dependencies have run; a stream outside the graph waits on it.
extern "C" int pdvc_event_create(void** event) {
    PDVC_CHECK_ARG(event != nullptr, "event is NULL");
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
        return pdvc_set_error(PDVC_ERR_LAUNCH, "hipEventCreateWithFlags");
    *event = (void*)e;
    return PDVC_OK;
}

extern "C" int pdvc_event_destroy(void* event) {
    PDVC_CHECK_ARG(event != nullptr, "event is NULL");
    return hipEventDestroy((hipEvent_t)event) == hipSuccess ? PDVC_OK
                                                            : pdvc_set_error(PDVC_ERR_LAUNCH, "hipEventDestroy");
}

// On a capturing stream the record is added to the capture's graph as an event-record node after the stream's
// current dependency set (hipStreamGetCaptureInfo_v2), and the stream's later work is made to follow it
// (hipEventRecordWithFlags(.., hipEventRecordExternal) is refused inside a capture on this stack: invalid argument).
// On a stream that is not capturing it is a plain record.
extern "C" int pdvc_event_record_external(void* event, void* stream) {
    PDVC_CHECK_ARG(event != nullptr, "event is NULL");
    hipStream_t s = (hipStream_t)stream;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    hipError_t e = hipStreamGetCaptureInfo_v2(s, &st, &id, &g, &deps, &nd);
    if (e != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "hipStreamGetCaptureInfo_v2: %s", hipGetErrorString(e));
    if (st != hipStreamCaptureStatusActive) {
        e = hipEventRecord((hipEvent_t)event, s);
        return e == hipSuccess ? PDVC_OK : pdvc_set_error(PDVC_ERR_LAUNCH, "hipEventRecord: %s", hipGetErrorString(e));
    }
    std::vector<hipGraphNode_t> dv(deps, deps + nd);  // copied: the stream's array may change with the update below
    hipGraphNode_t node;
    e = hipGraphAddEventRecordNode(&node, g, nd ? dv.data() : nullptr, nd, (hipEvent_t)event);
    if (e != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "hipGraphAddEventRecordNode: %s", hipGetErrorString(e));
    e = hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
    return e == hipSuccess ? PDVC_OK
                           : pdvc_set_error(PDVC_ERR_LAUNCH, "hipStreamUpdateCaptureDependencies: %s", hipGetErrorString(e));
}

extern "C" int pdvc_event_record_captured(void* event, void* stream) {
    PDVC_CHECK_ARG(event != nullptr, "event is NULL");
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    const hipError_t e = hipStreamIsCapturing((hipStream_t)stream, &st);
    if (e != hipSuccess) return pdvc_set_error(PDVC_ERR_LAUNCH, "hipStreamIsCapturing: %s", hipGetErrorString(e));
    PDVC_CHECK_ARG(st == hipStreamCaptureStatusActive,
                   "pdvc_event_record_captured: the stream is not capturing (a bucket event recorded outside the "
                   "captured step would not gate the replays' all-reduces)");
    return pdvc_event_record_external(event, stream);
}

extern "C" int pdvc_stream_wait_event(void* stream, void* event) {
    PDVC_CHECK_ARG(event != nullptr, "event is NULL");
    const hipError_t e = hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0);
    return e == hipSuccess ? PDVC_OK : pdvc_set_error(PDVC_ERR_LAUNCH, "hipStreamWaitEvent: %s", hipGetErrorString(e));
}

// ---- the overlap probe's gate: a host flag the device polls (fine-grained, coherent pinned memory) ----
namespace {
__global__ void spin_until_flag_kernel(const int* flag, int value, unsigned long long ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    // system-scope loads: vector loads past the caches, each one a read of the host's int
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != value) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) return;  // bounded: the grid always drains
        __builtin_amdgcn_s_sleep(32);
    }
}
}  // namespace

extern "C" int pdvc_host_flag_alloc(void** host, void** dev) {
    PDVC_CHECK_ARG(host != nullptr && dev != nullptr, "host / dev is NULL");
    void* h = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
        return pdvc_set_error(PDVC_ERR_LAUNCH, "hipHostMalloc");
    *reinterpret_cast<volatile int*>(h) = 0;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        return pdvc_set_error(PDVC_ERR_LAUNCH, "hipHostGetDevicePointer");
    }
    *host = h;
    *dev = d;
    return PDVC_OK;
}

extern "C" int pdvc_host_flag_free(void* host) {
    PDVC_CHECK_ARG(host != nullptr, "host is NULL");
    return hipHostFree(host) == hipSuccess ? PDVC_OK : pdvc_set_error(PDVC_ERR_LAUNCH, "hipHostFree");
}

extern "C" int pdvc_spin_until_flag(const int* dev_flag, int value, int timeout_ms, void* stream) {
    PDVC_CHECK_ARG(dev_flag != nullptr, "flag is NULL");
    PDVC_CHECK_ARG(timeout_ms > 0 && timeout_ms <= 10000, "timeout_ms must be in (0, 10000]");
    hipLaunchKernelGGL(spin_until_flag_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dev_flag, value,
                       (unsigned long long)timeout_ms * 100000ull);
    PDVC_CHECK_LAUNCH("spin_until_flag_kernel");
    return PDVC_OK;
}
