// Library-level entry points of libdfq_hip.so: version, error strings and the
// last-HIP-error side channel used by the Python host layer for messages.
#include "dfq_common.h"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

namespace dfq {
static thread_local char g_last_hip[256] = "";
void set_last_hip_error(hipError_t e) {
    const char* msg = hipGetErrorString(e);
    size_t i = 0;
    for (; msg && msg[i] && i + 1 < sizeof(g_last_hip); ++i) g_last_hip[i] = msg[i];
    g_last_hip[i] = '\0';
}
// the calling thread's last HIP error text (a worker thread's error, reported by
// the thread that joins it)
void set_last_hip_error_text(const char* msg) {
    size_t i = 0;
    for (; msg && msg[i] && i + 1 < sizeof(g_last_hip); ++i) g_last_hip[i] = msg[i];
    g_last_hip[i] = '\0';
}

// Pinned staging slots for stage_h2d, per device (an event belongs to the device
// it was created on).  A slot is free once the event recorded behind its last DMA
// has completed; with every slot busy the oldest is waited for (bounded memory).
namespace {
struct StageSlot {
    void* host = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    int device = -1;
    uint64_t last_use = 0;
};
constexpr size_t kStageMinBytes = 1 << 20;
constexpr size_t kStageMaxSlots = 32;
std::mutex g_stage_mu;
std::vector<StageSlot> g_stage;
uint64_t g_stage_tick = 0;
}  // namespace

hipError_t stage_h2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    int dev = 0;
    hipError_t e = hipStreamGetDevice(s, &dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(g_stage_mu);
    StageSlot* slot = nullptr;
    StageSlot* oldest = nullptr;
    size_t on_dev = 0;
    for (auto& sl : g_stage) {
        if (sl.device != dev) continue;
        ++on_dev;
        if (sl.cap >= bytes && hipEventQuery(sl.ev) == hipSuccess &&
            (!slot || sl.cap < slot->cap)) slot = &sl;
        if (!oldest || sl.last_use < oldest->last_use) oldest = &sl;
    }
    if (!slot && on_dev >= kStageMaxSlots && oldest) {   // every slot busy: recycle the oldest
        if ((e = hipEventSynchronize(oldest->ev)) != hipSuccess) return e;
        if (oldest->cap < bytes) {
            (void)hipHostFree(oldest->host);
            oldest->host = nullptr;
            oldest->cap = 0;
            size_t cap = std::max(bytes, kStageMinBytes);
            if ((e = hipHostMalloc(&oldest->host, cap, hipHostMallocDefault)) != hipSuccess) return e;
            oldest->cap = cap;
        }
        slot = oldest;
    }
    if (!slot) {
        StageSlot ns;
        ns.device = dev;
        ns.cap = std::max(bytes, kStageMinBytes);
        int cur = 0;
        if ((e = hipGetDevice(&cur)) != hipSuccess) return e;
        if (cur != dev && (e = hipSetDevice(dev)) != hipSuccess) return e;
        e = hipHostMalloc(&ns.host, ns.cap, hipHostMallocDefault);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ns.ev, hipEventDisableTiming);
        if (cur != dev) (void)hipSetDevice(cur);
        if (e != hipSuccess) {
            if (ns.host) (void)hipHostFree(ns.host);
            return e;
        }
        g_stage.push_back(ns);
        slot = &g_stage.back();
    }
    std::memcpy(slot->host, src, bytes);
    if ((e = hipMemcpyAsync(dst, slot->host, bytes, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    slot->last_use = ++g_stage_tick;
    return hipEventRecord(slot->ev, s);
}
}  // namespace dfq

namespace dfq {
// dfq_preload: `n` free staging slots of kStageMinBytes on the current device, so
// the first table uploads of a run (BN folds, absorption, sweep plans, the BC
// chain) do not pay for pinned allocations inside the caller's timed region.
static hipError_t stage_preload(size_t n) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(g_stage_mu);
    size_t on_dev = 0;
    for (const auto& sl : g_stage) on_dev += sl.device == dev ? 1 : 0;
    for (; on_dev < n && on_dev < kStageMaxSlots; ++on_dev) {
        StageSlot ns;
        ns.device = dev;
        ns.cap = kStageMinBytes;
        if ((e = hipHostMalloc(&ns.host, ns.cap, hipHostMallocDefault)) != hipSuccess) return e;
        if ((e = hipEventCreateWithFlags(&ns.ev, hipEventDisableTiming)) != hipSuccess) {
            (void)hipHostFree(ns.host);
            return e;
        }
        g_stage.push_back(ns);
    }
    return hipSuccess;
}
constexpr size_t kStagePreloadSlots = 8;

hipError_t preload_sweep();
hipError_t preload_transform();
hipError_t preload_cle();
}  // namespace dfq

extern "C" int dfq_preload(void) {
    DFQ_HIP_CHECK(dfq::preload_sweep());
    DFQ_HIP_CHECK(dfq::preload_transform());
    DFQ_HIP_CHECK(dfq::preload_cle());
    DFQ_HIP_CHECK(dfq::stage_preload(dfq::kStagePreloadSlots));
    return DFQ_OK;
}

extern "C" int dfq_abi_version(void) { return DFQ_ABI_VERSION; }

extern "C" const char* dfq_last_hip_error(void) { return dfq::g_last_hip; }

extern "C" const char* dfq_error_string(int code) {
    switch (code) {
        case DFQ_OK: return "ok";
        case DFQ_ERR_INVALID: return "invalid argument";
        case DFQ_ERR_HIP: return "HIP runtime error";
        case DFQ_ERR_UNSUPPORTED: return "unsupported request";
        case DFQ_ERR_NOMEM: return "out of memory";
        case DFQ_ERR_SHAPE: return "shape mismatch";
        case DFQ_ERR_WORKSPACE: return "workspace too small";
        default: return "unknown error";
    }
}
