// Roofline probe (measurement only): a grid-stride stream with the sweep's exact
// per-element traffic mix for 1x1 / Linear layers -- read x (16 B per 4
// elements), write dq (16 B), codes (4 B) and E (16 B) -- and no arithmetic.
// bench.py times it next to the sweep so the roofline fraction can be read
// against an achievable same-mix ceiling as well as against the 8 TB/s spec.
#include "dfq_common.h"
#include "dfq_diag.h"

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

// The sweep's exact memory pattern without its arithmetic: 4 waves per block, a
// wave task of 2048 fp32 moved HBM -> LDS by non-temporal LDS-DMA, then dq (16 B),
// codes (4 B) and E (16 B) stored non-temporally from LDS.  copy_only: dq only.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) probe_lds_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                        uint32_t* __restrict__ c, float* __restrict__ e, int64_t n,
                                                        int copy_only) {
    __shared__ __attribute__((aligned(16))) float lds[4 * 2048];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float* wl = lds + w * 2048;
    const int64_t ntask = n / 2048;
    for (int64_t t = (int64_t)blockIdx.x * 4 + w; t < ntask; t += (int64_t)gridDim.x * 4) {
        const float* src = x + t * 2048;
        for (int m = 0; m < 8; ++m)
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 4 * (lane + 64 * m)), (lds_void_t*)(wl + 256 * m), 16,
                                             0, 2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int j = lane; j < 512; j += 64) {
            const f32x4 v = reinterpret_cast<const f32x4*>(wl)[j];
            __builtin_nontemporal_store(v, (__attribute__((address_space(1))) f32x4*)(y + t * 2048) + j);
            if (!copy_only) {
                __builtin_nontemporal_store(__float_as_uint(v.x),
                                            (__attribute__((address_space(1))) uint32_t*)(c + t * 512) + j);
                __builtin_nontemporal_store(v, (__attribute__((address_space(1))) f32x4*)(e + t * 2048) + j);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}
}  // namespace dfq

// Sweep-pattern probe (LDS-DMA in, non-temporal out); n a multiple of 2048.
extern "C" int dfq_probe_lds(const float* x, float* y, void* codes, float* esum, int64_t n, int32_t copy_only,
                             int32_t blocks, void* stream) {
    if (!x || !y || n < 0 || (n % 2048) || blocks <= 0 || (!copy_only && (!codes || !esum))) return DFQ_ERR_INVALID;
    if (n == 0) return DFQ_OK;
    hipLaunchKernelGGL(dfq::probe_lds_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), x, y,
                       static_cast<uint32_t*>(codes), esum, n, (int)copy_only);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

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
