// Roofline probe (measurement only): a grid-stride stream with the sweep's exact
// per-element traffic mix for 1x1 / Linear layers -- read x (16 B per 4
// elements), write dq (16 B), codes (4 B) and E (16 B) -- and no arithmetic.
// bench.py times it next to the sweep so the roofline fraction can be read
// against an achievable same-mix ceiling as well as against the 8 TB/s spec.
#include "dfq_common.h"

namespace dfq {
__global__ void __launch_bounds__(256) probe_stream_kernel(const float4* __restrict__ x, float4* __restrict__ y,
                                                           uint32_t* __restrict__ c, float4* __restrict__ e,
                                                           int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const float4 v = x[i];
        y[i] = v;
        if (c) c[i] = __float_as_uint(v.x);
        if (e) e[i] = v;
    }
}
// 4 float4 per thread in flight per iteration (all loads before any store).
__global__ void __launch_bounds__(256) probe_stream4_kernel(const float4* __restrict__ x, float4* __restrict__ y,
                                                            uint32_t* __restrict__ c, float4* __restrict__ e,
                                                            int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t n16 = n4 / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = x[i + k * n16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            y[i + k * n16] = v[k];
            if (c) c[i + k * n16] = __float_as_uint(v[k].x);
            if (e) e[i + k * n16] = v[k];
        }
    }
}
}  // namespace dfq

// n: elements (multiple of 4); codes/esum may be NULL (drops that stream).
extern "C" int dfq_probe_stream(const float* x, float* y, void* codes, float* esum, int64_t n, int32_t blocks,
                                void* stream) {
    if (!x || !y || n < 0 || (n & 3) || blocks == 0) return DFQ_ERR_INVALID;
    if (n == 0) return DFQ_OK;
    const int grid = blocks > 0 ? blocks : -blocks;
    if (blocks < 0 && (n % 16) == 0) {   // negative block count: the 4-deep variant
        hipLaunchKernelGGL(dfq::probe_stream4_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                           reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y),
                           static_cast<uint32_t*>(codes), reinterpret_cast<float4*>(esum), n / 4);
        DFQ_LAUNCH_CHECK();
        return DFQ_OK;
    }
    hipLaunchKernelGGL(dfq::probe_stream_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                       reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y),
                       static_cast<uint32_t*>(codes), reinterpret_cast<float4*>(esum), n / 4);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}
