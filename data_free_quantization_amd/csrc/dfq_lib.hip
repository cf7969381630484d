// Library-level entry points of libdfq_hip.so: version, error strings and the
// last-HIP-error side channel used by the Python host layer for messages.
#include "dfq_common.h"

namespace dfq {
static thread_local char g_last_hip[256] = "";
void set_last_hip_error(hipError_t e) {
    const char* msg = hipGetErrorString(e);
    size_t i = 0;
    for (; msg && msg[i] && i + 1 < sizeof(g_last_hip); ++i) g_last_hip[i] = msg[i];
    g_last_hip[i] = '\0';
}
}  // namespace dfq

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
