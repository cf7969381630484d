// Shared device/host helpers for libdfq_hip.so (gfx950 only).
//
// Numerics contract: the library is compiled with
// -ffp-contract=off and the default correctly-rounded fp32 divide/sqrt, so every
// fp32 op below rounds once, exactly like torch's CPU eager ops in the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
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

// Wave min / max by DPP (VALU lane permutes: quad swaps, half-row and row
// mirrors) inside each 16-lane row, then the four rows' results by readlane:
// the same values as the shuffle forms (min / max are exact; only the combine
// order differs) at a fraction of their cost -- each __shfl_xor step is an LDS
// permute round trip, and the rescale tiles reduce every row of their tile.
__device__ __forceinline__ float dpp_f(float v, int ctrl) {
    const int x = __float_as_int(v);
    switch (ctrl) {   // the control must be a compile-time constant
        case 0xB1: return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false));
        case 0x4E: return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false));
        case 0x141: return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x141, 0xF, 0xF, false));
        default: return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x140, 0xF, 0xF, false));
    }
}
__device__ __forceinline__ float rl_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
// (min, max) over aligned groups of G lanes (G a power of two <= 64, wave-uniform):
// DPP quad swaps and half-row / row mirrors inside 16-lane rows (VALU, no LDS
// round trip), then LDS-permute shuffles only for the 32- and 64-lane groups.
// Every lane ends with its group's result.
// 3-input min / max as single v_min3_f32 / v_max3_f32 without the operand
// canonicalisation the compiler adds to fminf / fmaxf of loaded values (one v_max
// x, x per operand).  Quiet NaNs are ignored as by fminf / fmaxf; only a signalling
// NaN operand (which no fp32 weight produced by torch holds) could differ.
__device__ __forceinline__ float min3_nc(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float max3_nc(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ void group_minmax(float& lo, float& hi, int G) {
    if (G >= 2) {
        lo = fminf(lo, dpp_f(lo, 0xB1));
        hi = fmaxf(hi, dpp_f(hi, 0xB1));
    }
    if (G >= 4) {
        lo = fminf(lo, dpp_f(lo, 0x4E));
        hi = fmaxf(hi, dpp_f(hi, 0x4E));
    }
    if (G >= 8) {
        lo = fminf(lo, dpp_f(lo, 0x141));
        hi = fmaxf(hi, dpp_f(hi, 0x141));
    }
    if (G >= 16) {
        lo = fminf(lo, dpp_f(lo, 0x140));
        hi = fmaxf(hi, dpp_f(hi, 0x140));
    }
    for (int off = 16; off < G; off <<= 1) {
        lo = fminf(lo, __shfl_xor(lo, off, kWave));
        hi = fmaxf(hi, __shfl_xor(hi, off, kWave));
    }
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

// Workgroup LDS hand-off: this wave's ds_writes complete, then s_barrier.  No
// vmcnt wait (unlike __syncthreads' fence), so in-flight global stores stay in flight.
__device__ __forceinline__ void block_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
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

// The same result with the IEEE divide taken only near a rounding boundary.
// a = (x + negmn) * rcp(s) is within 2^-22 |t| of t = fl((x + negmn) / s)
// (v_rcp_f32: 1 ulp; the multiply: 1/2 ulp; t itself: 1/2 ulp).  The code only
// depends on which side of a half-integer clamp(t) lies.  c = clamp(a, qmin,
// qmax) is that value's stand-in: inside the range, when c is more than
// |c| 2^-20 (4x the error bound) away from the nearest half-integer,
// rint(c) == rint(clamp(t)); outside it, c is the end point (an integer, 1/2
// from any half-integer) and t is within the error bound of a beyond it, so
// clamp(t) rounds to the same end point; NaN / inf clamp as in qdq.  Otherwise
// -- ties and near-ties, ~1e-5 of the elements at INT8 -- the IEEE divide
// decides.  The dequantize (q * s + mn) is unchanged.  rs = __builtin_amdgcn_rcpf(s).
// The caller branches on a WAVE-uniform "any lane needs it" (ballot), so the
// divide is neither executed nor if-converted into every element's path: ~8
// VALU fewer per element (the sweep is issue-bound at ~500 G elements/s), and the
// one clamp serves both the test and the rounding.
// Step 1: the screened, clamped quotient; need = the IEEE divide must decide (rare).
__device__ __forceinline__ float qdq_screen(float x, const QParams& p, float rs, bool& need) {
    const float a = (x + p.negmn) * rs;
    const float t = fminf(fmaxf(a, p.qmin), p.qmax);
    const float d = __builtin_amdgcn_fractf(t) - 0.5f;   // v_fract: t - floor(t), exact for |t| < 2^24
    need = !(fabsf(d) > fabsf(t) * 0x1p-20f);
    return t;
}
// Step 2 (only where need): the reference's quotient, clamped.
__device__ __forceinline__ float qdq_exact_t(float x, const QParams& p) {
    return fminf(fmaxf((x + p.negmn) / p.s, p.qmin), p.qmax);
}
// Step 3: round half-even, dequantize (as qdq; t is already clamped).
__device__ __forceinline__ float qdq_finish(float t, const QParams& p, float& q) {
    q = rintf(t);
    const float y = q * p.s;
    return y + p.mn;
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------
// ATen's CPU fp32 summation order (at::native cascade_sum, SumKernel.cpp), which
// the reference's torch.sum / torch.mean follow.  Characterised against torch
// 2.10 in the dev container: vector width 8, ILP 4, a 4-level
// cascade with level step 2^max(4, CeilLog2(n)/4), and, for reductions over a
// strided dim of >= 32768 elements, an intra-op split over columns in chunks of
// ceil(F/threads) rounded down to multiples of 32.
// ---------------------------------------------------------------------------
__host__ __device__ inline int aten_ceil_log2(int64_t x) {
    if (x <= 2) return 1;
    int r = 0;
    for (uint64_t v = (uint64_t)(x - 1); v; v >>= 1) ++r;
    return r;
}

// multi_row_sum for one stream: sequential adds, flushed up a 4-level cascade.
// Level step 16 (every size below 2^20): a compile-time step, so each level-0
// block's 16 loads are issued together ahead of its 16 in-order adds (a runtime
// step left one load in flight per add).
template <typename Get>
__host__ __device__ inline float aten_cascade_16(Get get, int64_t size) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int64_t i = 0;
    while (i + 16 <= size) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = get(i + j);
#pragma unroll
        for (int j = 0; j < 16; ++j) a0 += v[j];
        i += 16;
        a1 += a0; a0 = 0.f;
        if (i & (15 << 4)) continue;
        a2 += a1; a1 = 0.f;
        if (i & (15 << 8)) continue;
        a3 += a2; a2 = 0.f;
    }
    for (; i < size; ++i) a0 += get(i);
    a0 += a1;
    a0 += a2;
    a0 += a3;
    return a0;
}

template <typename Get>
__host__ __device__ inline float aten_cascade(Get get, int64_t size) {
    const int lp = aten_ceil_log2(size) / 4 > 4 ? aten_ceil_log2(size) / 4 : 4;
    if (lp == 4) return aten_cascade_16(get, size);
    const int64_t step = (int64_t)1 << lp, mask = step - 1;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int64_t i = 0;
    while (i + step <= size) {
        for (int64_t j = 0; j < step; ++j, ++i) a0 += get(i);
        a1 += a0; a0 = 0.f;
        if (i & (mask << lp)) continue;
        a2 += a1; a1 = 0.f;
        if (i & (mask << (2 * lp))) continue;
        a3 += a2; a2 = 0.f;
    }
    for (; i < size; ++i) a0 += get(i);
    a0 += a1;
    a0 += a2;
    a0 += a3;
    return a0;
}

// row_sum: 4 interleaved cascades (ILP 4), tail into the first, then combined.
template <typename Get>
__host__ __device__ inline float aten_row_sum(Get get, int64_t size) {
    const int64_t sz = size / 4;
    float p0 = aten_cascade([&](int64_t i) { return get(4 * i + 0); }, sz);
    const float p1 = aten_cascade([&](int64_t i) { return get(4 * i + 1); }, sz);
    const float p2 = aten_cascade([&](int64_t i) { return get(4 * i + 2); }, sz);
    const float p3 = aten_cascade([&](int64_t i) { return get(4 * i + 3); }, sz);
    for (int64_t i = 4 * sz; i < size; ++i) p0 += get(i);
    p0 += p1;
    p0 += p2;
    p0 += p3;
    return p0;
}

// Sum over a contiguous dim of n elements (vectorized_inner_sum / scalar_inner_sum).
#ifndef DFQ_INNER_SUM_FAST   // compile-time A/B (scripts/cle_lib_ab.py): 0 = the generic walk only
#define DFQ_INNER_SUM_FAST 1
#endif
template <typename Get>
__host__ __device__ inline float aten_inner_sum(Get get, int64_t n) {
    if (n < 8) return aten_row_sum(get, n);
    const int64_t vs = n / 8;
    float fa = 0.f;
    for (int64_t k = 8 * vs; k < n; ++k) fa += get(k);
    if (DFQ_INNER_SUM_FAST && vs == 1) {
        // n in [8, 16): one element per (vector lane, ILP) stream.  aten_row_sum of
        // one element is ((((0 + 0) + x) + 0) + 0) + 0 with empty cascades, and
        // 0 + x is never -0, so adding the zeros changes no bit: 0 + x.  The generic
        // walk below made the CLE stop rule's per-layer means (8 thread slots) a
        // 4.8 us serial chain (DFQ_CLE_TL).
#pragma unroll
        for (int l = 0; l < 8; ++l) fa += 0.f + get(l);
        return fa;
    }
    for (int l = 0; l < 8; ++l) fa += aten_row_sum([&](int64_t i) { return get(8 * i + l); }, vs);
    return fa;
}

// --- wave-parallel forms of the same orders (bit-identical results) -------
// aten_cascade by one wave: level-0 blocks of 16 (one lane each), level-1 groups
// of 16 blocks, then the level-2/3 combine and the tails on lane 0.  b0s / b1s:
// this wave's LDS scratch (>= size/16 and size/256 floats).  Sizes whose cascade
// step is not 16 (>= 2^20) or that exceed the scratch run on lane 0.
template <typename Get>
__device__ inline float wave_cascade(Get get, int64_t size, int lane, float* b0s, float* b1s, int64_t b0cap) {
    float res = 0.f;
    if (aten_ceil_log2(size) / 4 > 4 || (size >> 4) > b0cap) {
        if (lane == 0) res = aten_cascade(get, size);
        return __shfl(res, 0, 64);
    }
    const int64_t nb0 = size >> 4, tail = size & 15, nb1 = nb0 >> 4, rem_b0 = nb0 & 15;
    const int64_t nb2 = nb1 >> 4, rem_b1 = nb1 & 15;
    for (int64_t m = lane; m < nb0; m += 64) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) a += get(m * 16 + j);
        b0s[m] = a;
    }
    wave_lds_sync();
    for (int64_t q = lane; q < nb1; q += 64) {
        float a = 0.f;
#pragma unroll
        for (int m = 0; m < 16; ++m) a += b0s[q * 16 + m];
        b1s[q] = a;
    }
    wave_lds_sync();
    if (lane == 0) {
        float a3 = 0.f;
        for (int64_t r = 0; r < nb2; ++r) {
            float b2 = 0.f;
            for (int q = 0; q < 16; ++q) b2 += b1s[r * 16 + q];
            a3 += b2;
        }
        float a2p = 0.f;
        for (int64_t q = 0; q < rem_b1; ++q) a2p += b1s[nb2 * 16 + q];
        float a1p = 0.f;
        for (int64_t m = 0; m < rem_b0; ++m) a1p += b0s[nb1 * 16 + m];
        float a0t = 0.f;
        for (int64_t j = 0; j < tail; ++j) a0t += get(nb0 * 16 + j);
        res = a0t;   // a0 += a1; a0 += a2; a0 += a3
        res += a1p;
        res += a2p;
        res += a3;
    }
    wave_lds_sync();   // scratch reused by the caller's next cascade
    return __shfl(res, 0, 64);
}

// aten_row_sum by one wave (4 ILP streams, each a wave_cascade).
template <typename Get>
__device__ inline float wave_row_sum(Get get, int64_t size, int lane, float* b0s, float* b1s, int64_t b0cap) {
    const int64_t sz = size / 4;
    float p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = wave_cascade([&](int64_t i) { return get(4 * i + k); }, sz, lane, b0s, b1s, b0cap);
    float p0 = p[0];
    for (int64_t i = 4 * sz; i < size; ++i) p0 += get(i);
    p0 += p[1];
    p0 += p[2];
    p0 += p[3];
    return p0;
}

// aten_inner_sum by one wave when every stream is short: lanes 0..31 each run one
// of the 32 (vector lane, ILP) cascades sequentially; every lane then runs the
// combine (the same value on every lane).
template <typename Get>
__device__ inline float wave_inner_sum(Get get, int64_t n, int lane) {
    float r = 0.f;
    if (n < 8) {
        if (lane == 0) r = aten_row_sum(get, n);
        return __shfl(r, 0, 64);
    }
    const int64_t vs = n / 8, sz = vs / 4;
    float p = 0.f;
    if (lane < 32) {
        const int l = lane & 7, k = lane >> 3;
        p = aten_cascade([&](int64_t i) { return get(8 * (4 * i + k) + l); }, sz);
        if (k == 0)
            for (int64_t v = 4 * sz; v < vs; ++v) p += get(8 * v + l);   // row_sum tail into p0
    }
    // the combine on every lane from the 32 partials read lane by lane (readlane:
    // uniform values, no 32-register array, no LDS permute per partial)
    auto rl = [&](int s) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), s)); };
    float fa = 0.f;
    for (int64_t e = 8 * vs; e < n; ++e) fa += get(e);
    for (int l = 0; l < 8; ++l) {
        float p0 = rl(l);
        p0 += rl(l + 8);
        p0 += rl(l + 16);
        p0 += rl(l + 24);
        fa += p0;
    }
    return fa;
}

// Agent-coherent fp32 store / load (sc1: no stale copy in another XCD's L2), for
// the words one block hands to another inside a launch (CLE: level-1 sums, chunk
// tails, chunk sums; the BC chain: every vector a later phase reads) without an
// L2 write-back.
// Address-space qualified pointers: a pointer loaded from a descriptor is generic
// (flat loads / stores: both wait counters, no SGPR-base addressing, a 64-bit
// VGPR address per access); cast to the space it lives in where that is known.
#define DFQ_GLOBAL __attribute__((address_space(1)))
#define DFQ_LDS __attribute__((address_space(3)))
typedef float f32x4 __attribute__((ext_vector_type(4)));   // float4 without the class (loads through DFQ_GLOBAL)

__device__ __forceinline__ void st_coh(float* p, float v) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_coh(const float* p) {
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ float ld_coh(const DFQ_GLOBAL float* p) {
    return __uint_as_float(__hip_atomic_load((const DFQ_GLOBAL uint32_t*)p, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
}

// Which reduction aten_outer_col_sum uses for column c: true = the 32-column
// multi_row_sum cascade, false = row_sum (ILP 4).
__host__ __device__ inline bool aten_outer_col_is_cascade(int64_t R, int64_t F, int64_t c, int threads) {
    int64_t c0 = 0, c1 = F;
    if (R * F >= 32768 && threads > 1) {
        const int64_t nt = F < threads ? F : threads;
        const int64_t chunk = ceil_div(F, nt);
        c0 = c1 = -1;
        for (int64_t t = 0; t < nt; ++t) {
            int64_t b = t * chunk, e = b + chunk < F ? b + chunk : F;
            if (b >= F) break;
            b = b >= F ? b : b - b % 32;
            e = e >= F ? e : e - e % 32;
            if (b <= c && c < e) { c0 = b; c1 = e; break; }
        }
        if (c0 < 0) { c0 = 0; c1 = F; }
    }
    const int64_t w = c1 - c0;
    const int64_t g = w >= 8 ? 32 : 4;
    return (c - c0) < g * (w / g);
}

// Column c of a row-major [R, F] summed over R (vectorized_outer_sum /
// scalar_outer_sum inside TensorIterator::parallel_reduce with `threads`).
__host__ __device__ inline float aten_outer_col_sum(const float* a, int64_t R, int64_t F, int64_t c, int threads) {
    int64_t c0 = 0, c1 = F;
    if (R * F >= 32768 && threads > 1) {
        const int64_t nt = F < threads ? F : threads;
        const int64_t chunk = ceil_div(F, nt);
        c0 = c1 = -1;
        for (int64_t t = 0; t < nt; ++t) {
            int64_t b = t * chunk, e = b + chunk < F ? b + chunk : F;
            if (b >= F) break;
            b = b >= F ? b : b - b % 32;
            e = e >= F ? e : e - e % 32;
            if (b <= c && c < e) { c0 = b; c1 = e; break; }
        }
        if (c0 < 0) { c0 = 0; c1 = F; }   // unreachable for 0 <= c < F
    }
    // Column groups of the chunk: vectorized (>= 8 columns) takes 4x8-column
    // multi_row_sum groups, then 8-column row_sum groups, then scalar row_sums;
    // scalar_outer_sum (< 8 columns) takes 4-column multi_row_sum groups first.
    const int64_t w = c1 - c0;
    const int64_t g = w >= 8 ? 32 : 4;
    const bool cascade = (c - c0) < g * (w / g);
    auto get = [&](int64_t r) { return a[r * F + c]; };
    return cascade ? aten_cascade(get, R) : aten_row_sum(get, R);
}

}  // namespace dfq

// Host-side error plumbing shared by the translation units.
namespace dfq {
void set_last_hip_error(hipError_t e);
void set_last_hip_error_text(const char* msg);
// Stream-ordered host -> device upload of a host-built table (task lists, fold
// jobs): `bytes` are copied into a pinned staging slot at once, the DMA is
// enqueued on `s`, and the slot is reused only after an event recorded behind
// that DMA has completed.  The caller's buffer may die at return; nothing
// synchronises the stream.
hipError_t stage_h2d(void* dst, const void* src, size_t bytes, hipStream_t s);
// Environment switches for A/B runs and diagnostics: read only by the diagnostics
// library (libdfq_diag.so, built with -DDFQ_DIAGNOSTICS); the product library
// runs its measured defaults whatever the environment says.
inline const char* ab_env(const char* name) {
#ifdef DFQ_DIAGNOSTICS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}
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
