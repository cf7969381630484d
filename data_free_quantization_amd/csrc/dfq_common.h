// Shared device/host helpers for libdfq_hip.so (gfx950 only).
//
// Numerics contract: the library is compiled with
// -ffp-contract=off and the default correctly-rounded fp32 divide/sqrt, so every
// fp32 op below rounds once, exactly like torch's CPU eager ops in the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dfq_hip.h"

namespace dfq {

constexpr int kWave = 64;

// Ordered-uint encoding of fp32: enc is monotone in the float order (with -0 < +0),
// so integer atomicMin/atomicMax give exact, order-independent float min/max.
__device__ __forceinline__ uint32_t enc_ord(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float dec_ord(uint32_t e) {
    uint32_t u = (e & 0x80000000u) ? (e & 0x7fffffffu) : ~e;
    return __uint_as_float(u);
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fminf(v, __shfl_xor(v, off, kWave));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}
__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// LDS ordering between lanes of ONE wave: drain this wave's LDS ops and keep the
// compiler from moving LDS accesses across the point.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Quantizer parameters, exactly as UniformQuantize.forward builds them
// (utils/quantize.py:51-72):  y = rint(clamp((x + negmn) / s, qmin, qmax)) * s + mn.
struct QParams {
    float s;      // (float) scale
    float negmn;  // (float)(-min)   (-0.0f for symmetric)
    float mn;     // (float) min     (+0.0f for symmetric)
    float qmin;
    float qmax;
};

// mn/mx: the fp32 data range; flags/given_*: see dfq_tensor_desc.
__device__ __host__ inline QParams make_qparams(float mn, float mx, int bits, bool sym, int flags,
                                                double given_min, double given_max) {
    QParams p;
    if (sym) {
        const int qmax_i = (1 << (bits - 1)) - 1;
        p.qmin = -(float)(1 << (bits - 1));
        p.qmax = (float)qmax_i;
        if (flags & DFQ_GIVEN_RANGE && flags & DFQ_SCALE_F32) {
            mn = (float)given_min;
            mx = (float)given_max;
        }
        if (flags & DFQ_SCALE_F32) {
            // 0-d fp32 tensors: abs, compare, fp32 divide by the int qmax.
            float a = fabsf(mx), b = fabsf(mn);
            if (a < b) a = b;
            float s = a / (float)qmax_i;
            if (s < (float)1e-8) s = (float)1e-8;
            p.s = s;
        } else {
            double dmx = (flags & DFQ_GIVEN_RANGE) ? given_max : (double)mx;
            double dmn = (flags & DFQ_GIVEN_RANGE) ? given_min : (double)mn;
            double a = fabs(dmx), b = fabs(dmn);
            if (a < b) a = b;
            double d = a / (double)qmax_i;
            if (1e-8 > d) d = 1e-8;   // Python max(scale, 1e-8)
            p.s = (float)d;
        }
        p.negmn = -0.0f;
        p.mn = 0.0f;
    } else {
        const int qmax_i = (1 << bits) - 1;
        p.qmin = 0.0f;
        p.qmax = (float)qmax_i;
        if (flags & DFQ_GIVEN_RANGE && flags & DFQ_SCALE_F32) {
            mn = (float)given_min;
            mx = (float)given_max;
        }
        if (flags & DFQ_SCALE_F32) {
            float s = (mx - mn) / (float)qmax_i;
            if (s < (float)1e-8) s = (float)1e-8;
            p.s = s;
            p.negmn = -mn;
            p.mn = mn;
        } else {
            double dmx = (flags & DFQ_GIVEN_RANGE) ? given_max : (double)mx;
            double dmn = (flags & DFQ_GIVEN_RANGE) ? given_min : (double)mn;
            double d = (dmx - dmn) / (double)qmax_i;
            if (1e-8 > d) d = 1e-8;
            p.s = (float)d;
            p.negmn = (float)(-dmn);
            p.mn = (float)dmn;
        }
    }
    return p;
}

// One element: add, IEEE divide, clamp, round-half-even, multiply, add -- each
// rounded once (no FMA: -ffp-contract=off).  Returns the dequantized value.
__device__ __forceinline__ float qdq(float x, const QParams& p, float& q) {
    float t = x + p.negmn;
    t = t / p.s;
    t = fminf(fmaxf(t, p.qmin), p.qmax);
    q = rintf(t);
    float y = q * p.s;
    return y + p.mn;
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace dfq

// Host-side error plumbing shared by the translation units.
namespace dfq {
void set_last_hip_error(hipError_t e);
}
#define DFQ_HIP_CHECK(expr)                                   \
    do {                                                      \
        hipError_t _e = (expr);                               \
        if (_e != hipSuccess) {                               \
            dfq::set_last_hip_error(_e);                      \
            return DFQ_ERR_HIP;                               \
        }                                                     \
    } while (0)
#define DFQ_LAUNCH_CHECK()                                    \
    do {                                                      \
        hipError_t _e = hipGetLastError();                    \
        if (_e != hipSuccess) {                               \
            dfq::set_last_hip_error(_e);                      \
            return DFQ_ERR_HIP;                               \
        }                                                     \
    } while (0)
