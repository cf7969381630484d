// Grouped quantize-dequantize sweep over many fp32 weight tensors (gfx950).
//
// Replaces, for every target layer at once:
//   * quantize()/UniformQuantize.forward          utils/quantize.py:16-89
//   * quantize_targ_layer's per-layer loop         utils/layer_transform.py:288-305
//   * clip_weight's clamp                          clip_weight.py:29
//   * the bias-correction error reduction          bias_correction.py:128-131,231
//
// Work decomposition: every tensor is cut on the host into WAVE TASKS of at most
// kChunk (2048) contiguous fp32 elements.  A task is either
//   - "whole rows": up to kMaxRows complete rows; the wave reduces each row's
//     min/max itself (CHANNEL modes, row_len <= kChunk), or
//   - a "block-row piece": rows longer than kChunk (up to 4 pieces, e.g. the
//     4608-element rows of ResNet-50's 512x512x3x3 convs) and small per-tensor
//     ranges are split over the 4 waves of ONE workgroup: the 4 pieces sit at
//     list positions 4k..4k+3, so the 4 waves of a block meet them in the same
//     grid-stride iteration, combine their partial (min, max) through LDS with
//     one s_barrier, and each quantizes its own piece -- a single HBM pass, or
//   - a "piece": its (min, max) come from a workspace slot filled by the
//     reduce launch (large TENSOR-mode ranges; rows longer than 4 pieces).
// One wave owns one task at a time (no workgroup barriers): it streams the chunk
// HBM -> VGPRs with 16-B loads, stages it in a wave-private LDS region for the
// per-row reductions and the KHW error sums, and writes dq (16 B/lane), codes
// (4 B/lane) and E.  Waves walk the task table grid-stride (persistent grid).
#include "dfq_common.h"
#ifdef DFQ_DIAGNOSTICS
#include "dfq_diag.h"
#endif

#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <new>
#include <numeric>
#include <type_traits>
#include <vector>

namespace dfq {

constexpr int kWavesPerBlock = 4;
constexpr int kBlockThreads = kWave * kWavesPerBlock;

// Kernel variants (chunk elements per wave task, rows per whole-row task, LDS-DMA
// prefetch of the next task).  The task table is built for the plan's variant.
struct Variant {
    int chunk;
    int max_rows;
    bool prefetch;
};
// max_rows: rows of one whole-row task; the host caps rows per task at
// max(64 (one short row per lane), chunk / 32) (build()), so the per-row
// parameter arrays (scale, min) take 2 * max_rows floats per wave.
constexpr Variant kVariants[] = {
    {2048, 64, false},    // 0: 8.5 KB LDS / wave, 16 waves / CU
    {1024, 64, true},     // 1: 2 x 4 KB, next task's DMA in flight during compute
    {2048, 64, true},     // 2: 2 x 8 KB
    {1024, 64, false},    // 3: 4.5 KB / wave
    {4096, 128, false},   // 4: 17 KB / wave, 8 waves / CU
    {2048, 64, false},    // 5: variant 0 with non-temporal loads and stores
    {2048, 64, false},    // 6: variant 5, KH*KW sums specialised for 3x3 only (fewer VGPRs)
    {2048, 64, false},    // 7: variant 5, generic KH*KW sums only
    {2560, 80, false},    // 8: variant 6 with 2560-element tasks (12 waves / CU)
    {1024, 64, false},    // 9: variant 6 with 1024-element tasks
    {1536, 64, false},    // 10: variant 6 with 1536-element tasks
    {1024, 64, true},     // 11: 1024-element tasks, next task's DMA in flight, NT
    {1024, 64, false},    // 12: variant 9 with the generic E sums (fewer VGPRs)
    {2048, 64, false},    // 13: variant 6 + per-task timestamps (diagnostics: dfq_debug_timeline)
    {2048, 64, false},    // 14: variant 6 with the IEEE divide on every element (round-2 arithmetic)
    {2048, 64, false},    // 15: variant 6 with the generic quantize loop (flags tested per float4; round 3)
    {2048, 64, false},    // 16: variant 6 with whole-row tasks in two row batches (compute_task_split)
};
constexpr int kNumVariants = 17;
// HostTask / DevTask .nrows <= kGroupTag: a row-group piece of R = kGroupTag - nrows + 1 rows
constexpr int kGroupTag = -64;
constexpr int kGroupMaxRows = 16;
#ifndef DFQ_DEFAULT_VARIANT   // compile-time override for side-by-side A/B builds (scripts/ab_variant_libs.py)
#define DFQ_DEFAULT_VARIANT 6
#endif
constexpr int kDefaultVariant = DFQ_DEFAULT_VARIANT;   // 6 = 5 with 87 instead of 105 VGPRs (profiles/r01/ab_*_v568.json)

struct alignas(16) DevTensor {
    const float* src;
    float* dst;
    void* codes;
    float* scale;
    float* zero;
    float* esum;
    int64_t rows;
    int64_t row_len;
    int32_t khw;
    int32_t bits;
    int32_t mode;
    int32_t flags;
    float clip_lo;
    float clip_hi;
    double given_min;
    double given_max;
    float inv_len;     // 1/row_len, for the element -> row map inside a task
    int32_t vec4;      // 16-B loads / stores legal
    int32_t code_bytes;
    uint32_t len_magic;  // ceil(2^32 / row_len): element -> row as one v_mul_hi_u32 (row_len >= 2)
    const uint32_t* range_enc;   // DFQ_DEVICE_RANGE
};

// A wave task as the host builds it (HostTask) and as the kernels read it
// (DevTask): the device record carries the address of its first element and the
// tensor's 16-B-vector flag, so a wave issues the task's LDS-DMA as soon as the
// record has landed, while the tensor's 128-B descriptor is still on its way
// (one dependent scalar round trip off every task's critical path).
struct HostTask {
    int64_t elem_start;  // first element (tensor-relative)
    int32_t tensor;
    int32_t n;           // elements in the task
    int32_t row0;        // first row of a whole-row task / the row of a long-row piece
    int32_t nrows;       // > 0: whole rows; 0: slot piece; -1/-2/-4: block-row piece; <= kGroupTag: row group
    int32_t slot;        // workspace (min,max) slot for pieces, -1 = given range
    int32_t first;       // this piece writes scale/zero for its slot
};
struct alignas(16) DevTask {
    const float* src;    // T.src + elem_start
    int32_t tensor;
    int32_t n;
    int32_t row0;
    int32_t nrows;
    int32_t slot;
    int32_t flags;       // bit 0: first (as HostTask); bit 1: T.vec4
};
static_assert(sizeof(DevTask) == 32, "one 32-B scalar load per task record");
__device__ __forceinline__ int64_t task_elem_start(const DevTask& k, const DevTensor& T) { return k.src - T.src; }

// Per-wave LDS image: [NB buffers of CHUNK floats][MAXROWS scales][MAXROWS mins]
// [MAXROWS reciprocal scales],
// carved out of ONE __shared__ array (a second __shared__ object next to an
// LDS-DMA target can make hipcc drain vmcnt before every ds_read).
template <int CHUNK, int MAXROWS, int NB>
struct LdsLayout {
    static constexpr int kPerWave = NB * CHUNK + 3 * MAXROWS;
    static constexpr int kTotal = kWavesPerBlock * kPerWave;
};

__device__ __forceinline__ bool is_sym(int mode) { return mode == DFQ_TENSOR_SYM || mode == DFQ_CHANNEL_SYM; }

template <bool NT, typename V>
__device__ __forceinline__ void st(V* p, const V& v);

__device__ __forceinline__ void store_code(void* codes, int cb, int64_t idx, float q) {
    if (cb == 1) {
        st<false>(static_cast<int8_t*>(codes) + idx, (int8_t)(int)q);  // same bits as uint8 for 0..255
    } else {
        st<false>(static_cast<int16_t*>(codes) + idx, (int16_t)(int)q);
    }
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

// HBM -> LDS without a VGPR landing (global_load_lds_dwordx4 / _dword): lane l's
// bytes land at lds_base + l*size, so one wave-instruction fills a contiguous
// 1 KiB (16 B/lane) or 256 B (4 B/lane) block of the task's LDS image.
template <bool NT = false>
__device__ __forceinline__ void glds16(const float* g, float* lds_base) {
    __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_base, 16, 0, NT ? 2 : 0);
}
template <bool NT = false>
__device__ __forceinline__ void glds4(const float* g, float* lds_base) {
    __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_base, 4, 0, NT ? 2 : 0);
}
// The same DMA issued through inline asm, which the compiler's wait-count pass does
// not see as a pending LDS write: with the builtin, every LDS read after a
// partial vmcnt wait got its own vmcnt(0) (the compiler cannot tell which DMA a
// read depends on), which undoes the two-batch overlap (compute_task_split).
// Every LDS read of a task's chunk is then ordered by the explicit waits alone.
template <bool NT = false>
__device__ __forceinline__ void glds16_asm(const float* g, float* lds_base) {
    const uint32_t m0 = (uint32_t)(uintptr_t)(lds_void_t*)lds_base;
    if constexpr (NT) asm volatile("global_load_lds_dwordx4 %0, off nt" ::"v"(g), "{m0}"(m0) : "memory");
    else asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}
template <bool NT = false>
__device__ __forceinline__ void glds4_asm(const float* g, float* lds_base) {
    const uint32_t m0 = (uint32_t)(uintptr_t)(lds_void_t*)lds_base;
    if constexpr (NT) asm volatile("global_load_lds_dword %0, off nt" ::"v"(g), "{m0}"(m0) : "memory");
    else asm volatile("global_load_lds_dword %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}
// Output stores; NT: non-temporal (streamed out, never re-read by this launch).
// Stores through address_space(1) pointers: the descriptor fields are generic
// pointers, and a flat_store also counts on lgkmcnt, so every LDS wait would
// drain the wave's outstanding stores.  global_store_* does not.
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <bool NT, typename V>
__device__ __forceinline__ void st(V* p, const V& v) {
    if constexpr (sizeof(V) == 16) {
        const f32x4 w = {v.x, v.y, v.z, v.w};
        DFQ_GLOBAL f32x4* g = (DFQ_GLOBAL f32x4*)p;
        if constexpr (NT) __builtin_nontemporal_store(w, g);
        else *g = w;
    } else {
        DFQ_GLOBAL V* g = (DFQ_GLOBAL V*)p;
        if constexpr (NT) __builtin_nontemporal_store(v, g);
        else *g = v;
    }
}
__device__ __forceinline__ float ld(const float* p) { return *(const DFQ_GLOBAL float*)p; }
__device__ __forceinline__ float4 ld(const float4* p) {
    const f32x4 v = *(const DFQ_GLOBAL f32x4*)p;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------
// Reduce launch: per-slot (min,max) of pieces via ordered-uint atomics.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlockThreads)
sweep_reduce_kernel(const DevTensor* __restrict__ tensors, const DevTask* __restrict__ tasks,
                    int64_t ntasks, uint32_t* __restrict__ slot_min, uint32_t* __restrict__ slot_max) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave0 = (int64_t)blockIdx.x * kWavesPerBlock + wave_uniform(threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t t = wave0; t < ntasks; t += nwaves) {
        const DevTask task = tasks[t];
        const float* src = task.src;
        float vmin = INFINITY, vmax = -INFINITY;
        if (task.flags & 2) {
            const int nj = task.n >> 2;
#pragma unroll 8
            for (int j = lane; j < nj; j += kWave) {
                const float4 v = ld(reinterpret_cast<const float4*>(src) + j);
                vmin = fminf(vmin, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
                vmax = fmaxf(vmax, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
            }
        } else {
#pragma unroll 8
            for (int e = lane; e < task.n; e += kWave) {
                const float x = ld(src + e);
                vmin = fminf(vmin, x);
                vmax = fmaxf(vmax, x);
            }
        }
        vmin = wave_min(vmin);
        vmax = wave_max(vmax);
        if (lane == 0) {
            atomicMin(&slot_min[task.slot], enc_ord(vmin));
            atomicMax(&slot_max[task.slot], enc_ord(vmax));
        }
    }
}

// ---------------------------------------------------------------------------
// Main launch: one wave task.
// ---------------------------------------------------------------------------
// Issue the task's HBM -> LDS DMA (all loads in flight; no wait).
template <bool NT = false, bool ASM = false>
__device__ __forceinline__ void issue_task_load(const DevTask& task, float* data, int lane) {
    const float* src = task.src;
    const int n = task.n;
    if (task.flags & 2) {
        const int nj = n >> 2;
        for (int m = 0; m * kWave < nj; ++m) {
            const int j = lane + m * kWave;
            if (j < nj) {
                if constexpr (ASM) glds16_asm<NT>(src + 4 * j, data + 4 * kWave * m);
                else glds16<NT>(src + 4 * j, data + 4 * kWave * m);
            }
        }
    } else {
        for (int m = 0; m * kWave < n; ++m) {
            const int e = lane + m * kWave;
            if (e < n) {
                if constexpr (ASM) glds4_asm<NT>(src + e, data + kWave * m);
                else glds4<NT>(src + e, data + kWave * m);
            }
        }
    }
}


// The VEC quantize loop with the task's output set fixed at compile time (clip,
// code format, error-sum form): straight-line per-float4 bodies without the
// generic loop's per-iteration flag branches.  Bit-identical with the generic loop
// (same IEEE operation sequence per element); what differs is how each step is
// issued on a wave64 SIMD, where every VALU op costs 4 cycles and this loop is the
// single-model sweep's VALU budget:
//  * fp32 pairs as packed ops (v_pk_add_f32 / v_pk_mul_f32: two lanes' worth per op);
//  * the element -> row map as one v_mul_hi_u32 by ceil(2^32 / row_len) (exact for
//    e < 2^16, row_len < 2^13), the row's 1/s read from LDS next to s and mn (no
//    per-float4 v_rcp);
//  * rint(t) as (t + 1.5*2^23) - 1.5*2^23 (t is clamped to [qmin, qmax], |t| < 2^22:
//    round-to-nearest-even at the integer ulp, the same value as rintf); the sum's
//    low mantissa bits are q's two's complement, so the codes are byte / half
//    selects (v_perm_b32) of it;
//  * the reciprocal screen as |t - rint(t)| >= 0.5 - qabs 2^-20 (qabs = the larger of
//    |qmin|, |qmax| >= |t|): a superset of the elements within |t| 2^-20 of a
//    rounding boundary, which are the only ones whose reciprocal quotient can round
//    differently from the IEEE divide; those take the divide.
//  * clamps as v_med3 (no operand canonicalisation: fminf / fmaxf on values the
//    compiler cannot prove canonical cost a v_max x, x each).
// CB: 0 no codes, 1 int8 / uint8, 2 int16, 3 packed int4.  EM: 0 no error sums,
// 1 E stored (KH*KW = 1), 2 eps back to LDS (KH*KW > 1).
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <bool CLIP, int CB, int EM, bool NT>
__device__ __forceinline__ void quant_vec4(const DevTensor& T, int n, int64_t base, float* data, const float* ls,
                                           const float* lmn, const float* lrs, const QParams& pc, bool whole,
                                           int eoff, int lane, float qmin, float qmax, bool sym) {
    constexpr float kMagic = 12582912.0f;   // 1.5 * 2^23
    const int nj = n >> 2;
    float* dq = T.dst + base;
    const float clo = T.clip_lo, chi = T.clip_hi;
    // whole-row tasks: the element's row; pieces: their one parameter set, in slot 0
    const uint32_t magic = whole ? T.len_magic : 0u;
    const float thr = 0.5f - fmaxf(-qmin, qmax) * 0x1p-20f;
    const f32x2 mg = {kMagic, kMagic};
    struct Q4 {   // one float4's state between the screen and the stores
        float4 x;
        float s, mn;
        float t[4];
        f32x2 ta, tb, qa, qb, da, db;
    };
    auto prep = [&](int j, uint32_t e, Q4& q) {
        q.x = reinterpret_cast<const float4*>(data)[j];
        const uint32_t r = __umulhi(e, magic);   // one row per float4 (4 | len, 4 | goff)
        q.s = ls[r];
        q.mn = lmn[r];
        const float rs = lrs[r];
        const f32x2 nm = {-q.mn, -q.mn};   // x + (-mn) (symmetric: x + -0.0, which is x)
        const f32x2 rs2 = {rs, rs};
        const f32x2 a = (f32x2{q.x.x, q.x.y} + nm) * rs2, b = (f32x2{q.x.z, q.x.w} + nm) * rs2;
        q.t[0] = __builtin_amdgcn_fmed3f(a.x, qmin, qmax);
        q.t[1] = __builtin_amdgcn_fmed3f(a.y, qmin, qmax);
        q.t[2] = __builtin_amdgcn_fmed3f(b.x, qmin, qmax);
        q.t[3] = __builtin_amdgcn_fmed3f(b.y, qmin, qmax);
        q.ta = f32x2{q.t[0], q.t[1]} + mg;
        q.tb = f32x2{q.t[2], q.t[3]} + mg;
        q.qa = q.ta - mg;
        q.qb = q.tb - mg;
        // opaque to the optimiser: merged with the rare path's values as they are,
        // not recomputed from t after the branch
        asm("" : "+v"(q.ta), "+v"(q.tb), "+v"(q.qa), "+v"(q.qb));
        q.da = f32x2{q.t[0], q.t[1]} - q.qa;
        q.db = f32x2{q.t[2], q.t[3]} - q.qb;
    };
    auto dmax = [&](const Q4& q) { return fmaxf(fmaxf(fabsf(q.da.x), fabsf(q.da.y)), fmaxf(fabsf(q.db.x), fabsf(q.db.y))); };
    auto fix = [&](Q4& q) {   // the IEEE divide for the screened elements
        const float negmn = -q.mn;
        if (fabsf(q.da.x) >= thr) q.t[0] = __builtin_amdgcn_fmed3f((q.x.x + negmn) / q.s, qmin, qmax);
        if (fabsf(q.da.y) >= thr) q.t[1] = __builtin_amdgcn_fmed3f((q.x.y + negmn) / q.s, qmin, qmax);
        if (fabsf(q.db.x) >= thr) q.t[2] = __builtin_amdgcn_fmed3f((q.x.z + negmn) / q.s, qmin, qmax);
        if (fabsf(q.db.y) >= thr) q.t[3] = __builtin_amdgcn_fmed3f((q.x.w + negmn) / q.s, qmin, qmax);
        q.ta = f32x2{q.t[0], q.t[1]} + mg;
        q.tb = f32x2{q.t[2], q.t[3]} + mg;
        q.qa = q.ta - mg;
        q.qb = q.tb - mg;
    };
    auto out = [&](int j, const Q4& q) {
        const f32x2 s2 = {q.s, q.s}, mn2 = {q.mn, q.mn};
        const f32x2 ya = q.qa * s2 + mn2, yb = q.qb * s2 + mn2;   // q * s, then + mn: two roundings (no contraction)
        float y[4] = {ya.x, ya.y, yb.x, yb.y};
        if constexpr (CLIP) {
#pragma unroll
            for (int k = 0; k < 4; ++k) y[k] = __builtin_amdgcn_fmed3f(y[k], clo, chi);
        }
        st<NT>(reinterpret_cast<float4*>(dq) + j, make_float4(y[0], y[1], y[2], y[3]));
        const uint32_t u0 = __float_as_uint(q.ta.x), u1 = __float_as_uint(q.ta.y);
        const uint32_t u2 = __float_as_uint(q.tb.x), u3 = __float_as_uint(q.tb.y);
        if constexpr (CB == 1) {   // bytes 0 of u0..u3
            const uint32_t c = __builtin_amdgcn_perm(u1, u0, 0x0c0c0400u) | __builtin_amdgcn_perm(u3, u2, 0x04000c0cu);
            st<NT>(reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(T.codes) + base) + j, c);
        } else if constexpr (CB == 3) {   // DFQ_PACK_INT4: 4 codes -> 2 bytes (base % 4 == 0)
            const uint32_t c = (u0 & 0xFu) | ((u1 & 0xFu) << 4) | ((u2 & 0xFu) << 8) | ((u3 & 0xFu) << 12);
            st<NT>(reinterpret_cast<uint16_t*>(static_cast<uint8_t*>(T.codes) + base / 2) + j, (uint16_t)c);
        } else if constexpr (CB == 2) {   // halves 0 of u0..u3
            const uint64_t c = (uint64_t)__builtin_amdgcn_perm(u1, u0, 0x05040100u) |
                               ((uint64_t)__builtin_amdgcn_perm(u3, u2, 0x05040100u) << 32);
            st<NT>(reinterpret_cast<uint64_t*>(static_cast<uint16_t*>(T.codes) + base) + j, c);
        }
        if constexpr (EM != 0) {
            const f32x2 ea = f32x2{y[0], y[1]} - f32x2{q.x.x, q.x.y}, eb = f32x2{y[2], y[3]} - f32x2{q.x.z, q.x.w};
            const float4 ev = make_float4(ea.x, ea.y, eb.x, eb.y);
            if constexpr (EM == 1) st<NT>(reinterpret_cast<float4*>(T.esum + base) + j, ev);
            else reinterpret_cast<float4*>(data)[j] = ev;
        }
    };
    // two independent float4s per lane and step (one dependent chain per float4 is
    // too little work between LDS round trips at 2-3 waves per SIMD); the second
    // one past the task's end recomputes the first and stores nothing
    uint32_t e = (uint32_t)(4 * lane + eoff);
    for (int j = lane; j < nj; j += 2 * kWave, e += 8 * kWave) {
        const int j1 = j + kWave;
        const bool has1 = j1 < nj;
        Q4 qa, qb;
        prep(j, e, qa);
        prep(has1 ? j1 : j, has1 ? e + 4 * kWave : e, qb);
        if (__builtin_amdgcn_ballot_w64(fmaxf(dmax(qa), dmax(qb)) >= thr)) {   // wave-uniform, rare
            fix(qa);
            fix(qb);
        }
        out(j, qa);
        if (has1) out(j1, qb);
    }
}

template <bool CLIP, int CB, bool NT>
__device__ __forceinline__ void quant_vec4_e(int em, const DevTensor& T, int n, int64_t base, float* data,
                                             const float* ls, const float* lmn, const float* lrs, const QParams& pc,
                                             bool whole, int eoff, int lane, float qmin, float qmax, bool sym) {
    if (em == 0) quant_vec4<CLIP, CB, 0, NT>(T, n, base, data, ls, lmn, lrs, pc, whole, eoff, lane, qmin, qmax, sym);
    else if (em == 1) quant_vec4<CLIP, CB, 1, NT>(T, n, base, data, ls, lmn, lrs, pc, whole, eoff, lane, qmin, qmax, sym);
    else quant_vec4<CLIP, CB, 2, NT>(T, n, base, data, ls, lmn, lrs, pc, whole, eoff, lane, qmin, qmax, sym);
}

template <bool CLIP, bool NT>
__device__ __forceinline__ void quant_vec4_c(int cb, int em, const DevTensor& T, int n, int64_t base, float* data,
                                             const float* ls, const float* lmn, const float* lrs, const QParams& pc,
                                             bool whole, int eoff, int lane, float qmin, float qmax, bool sym) {
    switch (cb) {
        case 0: quant_vec4_e<CLIP, 0, NT>(em, T, n, base, data, ls, lmn, lrs, pc, whole, eoff, lane, qmin, qmax, sym); break;
        case 1: quant_vec4_e<CLIP, 1, NT>(em, T, n, base, data, ls, lmn, lrs, pc, whole, eoff, lane, qmin, qmax, sym); break;
        case 2: quant_vec4_e<CLIP, 2, NT>(em, T, n, base, data, ls, lmn, lrs, pc, whole, eoff, lane, qmin, qmax, sym); break;
        default: quant_vec4_e<CLIP, 3, NT>(em, T, n, base, data, ls, lmn, lrs, pc, whole, eoff, lane, qmin, qmax, sym);
    }
}

// Steps 2-4 on a chunk that has landed in ``data``.
// ESPEC: compile-time KH*KW error sums -- 2: 3x3/5x5/7x7/2x2, 1: 3x3, 0: none
// goff >= 0: a row-group piece whose per-row parameters are already in ls / lmn
// (local row 0 = the row holding the piece's first element, goff = that element's
// offset inside it).
// SCREEN: the screened reciprocal quantize (qdq_screen, the IEEE divide only near a
// rounding boundary); false: the IEEE divide for every element (round-2 arithmetic,
// diagnostics variant 14).  Bit-identical results.
template <int MAXROWS, bool VEC, bool NT = false, int ESPEC = 2, bool SCREEN = true, bool FAST = true>
__device__ __forceinline__ void compute_task(const DevTensor& T, const DevTask& task, float* data, float* ls,
                                             float* lmn, const uint32_t* __restrict__ slot_min,
                                             const uint32_t* __restrict__ slot_max, int lane, float bmn = 0.f,
                                             float bmx = 0.f, int goff = -1, uint64_t* tlm = nullptr,
                                             uint32_t abl = 0) {
    const int n = task.n;
    const bool sym = is_sym(T.mode);
    const int len = (int)T.row_len;

    // 2. per-row parameters (whole-row tasks) or the slot's parameters (pieces)
    QParams pc{};
    const bool group = goff >= 0;
    const bool whole = task.nrows > 0 || group;
    const int eoff = group ? goff : 0;
    if (group) {
        // parameters set by the caller
    } else if (whole) {
        // G lanes per row (G * next_pow2(nrows) = 64): every row of the task is
        // reduced at once; shuffles stay inside a G-lane group and every group
        // leader builds its row's parameters concurrently.
        const int nrows = task.nrows;
        int p2 = 1;
        while (p2 < nrows && p2 < kWave) p2 <<= 1;
        const int G = kWave / p2;
        const int sub = lane / G, sl = lane % G;
        for (int r0 = 0; r0 < nrows; r0 += p2) {
            const int r = r0 + sub;
            float vmin = INFINITY, vmax = -INFINITY;
            if (abl & 1) {   // diagnostics ablation: no row reduce
                vmin = -1.f;
                vmax = 1.f;
            } else if (r < nrows) {
                const float* row = data + r * len;
                if (VEC) {
                    // 4 LDS loads in flight per lane, then their min / max (a lane walks
                    // up to 16 float4s of its row; one round trip per 4 instead of per 1)
                    const int q4 = len >> 2;
                    const float4* row4 = reinterpret_cast<const float4*>(row);
                    for (int i = sl; i < q4; i += 4 * G) {
                        // past the row's end a lane re-reads the row's last float4 (min / max
                        // are idempotent): no per-load exec masks
                        float4 v[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) v[u] = row4[min(i + u * G, q4 - 1)];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            vmin = min3_nc(min3_nc(vmin, v[u].x, v[u].y), v[u].z, v[u].w);
                            vmax = max3_nc(max3_nc(vmax, v[u].x, v[u].y), v[u].z, v[u].w);
                        }
                    }
                } else {
                    for (int i = sl; i < len; i += G) {
                        const float v = row[i];
                        vmin = fminf(vmin, v);
                        vmax = fmaxf(vmax, v);
                    }
                }
            }
            group_minmax(vmin, vmax, G);   // DPP inside 16-lane rows (no LDS round trips)
            if (tlm && r0 == 0) tlm[2] = wall_clock64();   // diagnostics: the first rows' ranges reduced
            if (sl == 0 && r < nrows) {
                const QParams p = make_qparams(vmin, vmax, T.bits, sym, T.flags, T.given_min, T.given_max);
                ls[r] = p.s;
                lmn[r] = p.mn;
                lmn[MAXROWS + r] = __builtin_amdgcn_rcpf(p.s);   // the quantize loop's 1/s
                const int64_t row_g = task.row0 + r;
                if (T.scale) st<false>(T.scale + row_g, p.s);
                if (T.zero) st<false>(T.zero + row_g, p.mn);
            }
            if (tlm && r0 == 0) tlm[3] = wall_clock64();   // diagnostics: their parameters built
        }
        wave_lds_sync();
    } else {
        float mn = bmn, mx = bmx;   // block-row piece: the workgroup's combined range
        if (task.slot >= 0) {
            mn = dec_ord(slot_min[task.slot]);
            mx = dec_ord(slot_max[task.slot]);
        } else if (T.flags & DFQ_DEVICE_RANGE) {
            mn = dec_ord(~T.range_enc[0]);
            mx = dec_ord(T.range_enc[1]);
        }
        pc = make_qparams(mn, mx, T.bits, sym, T.flags, T.given_min, T.given_max);
        if ((task.flags & 1) && lane == 0) {
            const int64_t row_g = (T.mode == DFQ_CHANNEL_ASYM || T.mode == DFQ_CHANNEL_SYM) ? task.row0 : 0;
            if (T.scale) st<false>(T.scale + row_g, pc.s);
            if (T.zero) st<false>(T.zero + row_g, pc.mn);
        }
        if (VEC && lane == 0) {   // the fixed-form quantize loop reads parameters from slot 0
            ls[0] = pc.s;
            lmn[0] = pc.mn;
            lmn[MAXROWS] = __builtin_amdgcn_rcpf(pc.s);
        }
        if (VEC) wave_lds_sync();
    }

    if (tlm) tlm[0] = wall_clock64();   // diagnostics timeline (variant 13): parameters done
    // 3. quantize / dequantize / clip from LDS; write dq + codes; eps for bias correction.
    //    eps overwrites the x it came from (same lane, same slot), so no hazard.
    const bool clip = (T.flags & DFQ_CLIP) != 0;
    const bool want_e = T.esum != nullptr;
    const int khw = T.khw;
    const float qmin = sym ? -(float)(1 << (T.bits - 1)) : 0.f;
    const float qmax = sym ? (float)((1 << (T.bits - 1)) - 1) : (float)((1 << T.bits) - 1);
    const int64_t base = task_elem_start(task, T);

    auto params_for = [&](int e) -> QParams {
        if (!whole) return pc;
        // row = floor(e / len): (e + 0.5)/len is >= 0.5/len from an integer and
        // e < 2048, so this fp32 estimate is exact.
        int r = (int)(((float)(e + eoff) + 0.5f) * T.inv_len);
        r = min(r, MAXROWS - 1);
        QParams p;
        p.s = ls[r];
        p.mn = lmn[r];
        p.negmn = -p.mn;
        p.qmin = qmin;
        p.qmax = qmax;
        return p;
    };
    auto one = [&](float xv, const QParams& p, float& qv) -> float {
        if constexpr (!SCREEN) {
            float yv = qdq(xv, p, qv);
            if (clip) yv = fminf(fmaxf(yv, T.clip_lo), T.clip_hi);
            return yv;
        }
        bool need;
        float t = qdq_screen(xv, p, __builtin_amdgcn_rcpf(p.s), need);
        if (__builtin_amdgcn_ballot_w64(need)) {   // wave-uniform, rare
            if (need) t = qdq_exact_t(xv, p);
        }
        float yv = qdq_finish(t, p, qv);
        if (clip) yv = fminf(fmaxf(yv, T.clip_lo), T.clip_hi);
        return yv;
    };
    // four elements sharing one row's parameters: one reciprocal, one ballot
    auto four = [&](const float4& xv, const QParams& p, float& q0, float& q1, float& q2, float& q3) -> float4 {
        if constexpr (!SCREEN) return make_float4(one(xv.x, p, q0), one(xv.y, p, q1), one(xv.z, p, q2), one(xv.w, p, q3));
        const float rs = __builtin_amdgcn_rcpf(p.s);
        bool n0, n1, n2, n3;
        float t0 = qdq_screen(xv.x, p, rs, n0), t1 = qdq_screen(xv.y, p, rs, n1);
        float t2 = qdq_screen(xv.z, p, rs, n2), t3 = qdq_screen(xv.w, p, rs, n3);
        if (__builtin_amdgcn_ballot_w64(n0 | n1 | n2 | n3)) {   // wave-uniform, rare
            if (n0) t0 = qdq_exact_t(xv.x, p);
            if (n1) t1 = qdq_exact_t(xv.y, p);
            if (n2) t2 = qdq_exact_t(xv.z, p);
            if (n3) t3 = qdq_exact_t(xv.w, p);
        }
        float4 y = make_float4(qdq_finish(t0, p, q0), qdq_finish(t1, p, q1), qdq_finish(t2, p, q2),
                               qdq_finish(t3, p, q3));
        if (clip) {
            y.x = fminf(fmaxf(y.x, T.clip_lo), T.clip_hi);
            y.y = fminf(fmaxf(y.y, T.clip_lo), T.clip_hi);
            y.z = fminf(fmaxf(y.z, T.clip_lo), T.clip_hi);
            y.w = fminf(fmaxf(y.w, T.clip_lo), T.clip_hi);
        }
        return y;
    };

    // the generic VEC loop: every output flag tested per float4
    auto vec_generic = [&]() {
        const int nj = n >> 2;
#pragma unroll 2
        for (int j = lane; j < nj; j += kWave) {
            const float4 xv = reinterpret_cast<const float4*>(data)[j];
            const QParams p = params_for(4 * j);   // 4 | len, 4 | goff: one row per float4
            float q0, q1, q2, q3;
            const float4 yq = four(xv, p, q0, q1, q2, q3);
            const float y0 = yq.x, y1 = yq.y, y2 = yq.z, y3 = yq.w;
            if (T.dst) st<NT>(reinterpret_cast<float4*>(T.dst + base) + j, make_float4(y0, y1, y2, y3));
            if (T.codes) {
                if (T.code_bytes == 1) {
                    const uint32_t c = ((uint32_t)(uint8_t)(int)q0) | ((uint32_t)(uint8_t)(int)q1 << 8) |
                                       ((uint32_t)(uint8_t)(int)q2 << 16) | ((uint32_t)(uint8_t)(int)q3 << 24);
                    st<NT>(reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(T.codes) + base) + j, c);
                } else if (T.code_bytes == 0) {   // DFQ_PACK_INT4: 4 codes -> 2 bytes (base % 4 == 0)
                    const uint32_t c = ((uint32_t)(int)q0 & 0xFu) | (((uint32_t)(int)q1 & 0xFu) << 4) |
                                       (((uint32_t)(int)q2 & 0xFu) << 8) | (((uint32_t)(int)q3 & 0xFu) << 12);
                    st<NT>(reinterpret_cast<uint16_t*>(static_cast<uint8_t*>(T.codes) + base / 2) + j, (uint16_t)c);
                } else {
                    const uint64_t c = ((uint64_t)(uint16_t)(int)q0) | ((uint64_t)(uint16_t)(int)q1 << 16) |
                                       ((uint64_t)(uint16_t)(int)q2 << 32) | ((uint64_t)(uint16_t)(int)q3 << 48);
                    st<NT>(reinterpret_cast<uint64_t*>(static_cast<uint16_t*>(T.codes) + base) + j, c);
                }
            }
            if (want_e) {
                const float4 ev = make_float4(y0 - xv.x, y1 - xv.y, y2 - xv.z, y3 - xv.w);
                if (khw == 1) st<NT>(reinterpret_cast<float4*>(T.esum + base) + j, ev);
                else reinterpret_cast<float4*>(data)[j] = ev;
            }
        }
    };
    if (abl & 6) {   // diagnostics ablation: 2 = stores without the arithmetic, 4 = no quantize loop
        if ((abl & 64) && VEC) {   // 64 (with 4): the arithmetic without the stores
            const int nj = n >> 2;
            float acc = 0.f;
            for (int j = lane; j < nj; j += kWave) {
                const float4 xv = reinterpret_cast<const float4*>(data)[j];
                float q0, q1, q2, q3;
                const float4 y = four(xv, params_for(4 * j), q0, q1, q2, q3);
                acc += (y.x + y.y) + (y.z + y.w) + (q0 + q1) + (q2 + q3);
            }
            if (acc == 1234.5678f) st<false>(T.dst + base, acc);   // keeps the work
        } else if (!(abl & 4) && VEC) {
            const int nj = n >> 2;
            for (int j = lane; j < nj; j += kWave) {
                const float4 xv = reinterpret_cast<const float4*>(data)[j];
                st<NT>(reinterpret_cast<float4*>(T.dst + base) + j, xv);
                if (T.codes) st<NT>(reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(T.codes) + base) + j, __float_as_uint(xv.x));
            }
        } else if (!(abl & 4)) {
            for (int e = lane; e < n; e += kWave) {
                st<false>(T.dst + base + e, data[e]);
                if (T.codes) st<false>(static_cast<uint8_t*>(T.codes) + base + e, (uint8_t)__float_as_uint(data[e]));
            }
        }
    } else if constexpr (VEC) {
        bool done = false;
        if constexpr (SCREEN && FAST && MAXROWS == 64) {
            const float* lrs = lmn + MAXROWS;
            if (T.dst && (!clip || T.clip_lo <= T.clip_hi)) {   // one compile-time body per (clip, codes, E form)
                const int cb = !T.codes ? 0 : (T.code_bytes == 1 ? 1 : (T.code_bytes == 0 ? 3 : 2));
                const int em = !want_e ? 0 : (khw == 1 ? 1 : 2);
                if (clip) quant_vec4_c<true, NT>(cb, em, T, n, base, data, ls, lmn, lrs, pc, whole, eoff, lane, qmin, qmax, sym);
                else quant_vec4_c<false, NT>(cb, em, T, n, base, data, ls, lmn, lrs, pc, whole, eoff, lane, qmin, qmax, sym);
                done = true;
            }
        }
        if (!done) vec_generic();
    } else if (T.codes && T.code_bytes == 0) {
        // packed nibbles on the scalar path: the task starts at an even element
        // (build()), so even lanes own a byte and take the odd neighbour's code by
        // a shuffle; every lane runs every step so the shuffle sees defined values
        for (int e0 = 0; e0 < n; e0 += kWave) {
            const int e = e0 + lane;
            const bool ok = e < n;
            uint32_t qi = 0;
            if (ok) {
                const float xv = data[e];
                float qv;
                const float yv = one(xv, params_for(e), qv);
                if (T.dst) st<false>(T.dst + base + e, yv);
                qi = (uint32_t)(int)qv & 0xFu;
                if (want_e) {
                    if (khw == 1) st<false>(T.esum + base + e, yv - xv);
                    else data[e] = yv - xv;
                }
            }
            const uint32_t hi = (uint32_t)__shfl_down((int)qi, 1, kWave);
            if (ok && (e & 1) == 0)
                st<false>(static_cast<uint8_t*>(T.codes) + (base + e) / 2, (uint8_t)(qi | (hi << 4)));
        }
    } else {
#pragma unroll 4
        for (int e = lane; e < n; e += kWave) {
            const float xv = data[e];
            float qv;
            const float yv = one(xv, params_for(e), qv);
            if (T.dst) st<false>(T.dst + base + e, yv);
            if (T.codes) store_code(T.codes, T.code_bytes, base + e, qv);
            if (want_e) {
                if (khw == 1) st<false>(T.esum + base + e, yv - xv);
                else data[e] = yv - xv;
            }
        }
    }

    if (tlm) tlm[1] = wall_clock64();   // quantize loop issued
    // 4. KHW error sums: E[p] = sum_k eps[p*khw + k] in ATen's order
    if (want_e && khw > 1) {
        wave_lds_sync();
        const int np = n / khw;
        const int64_t pbase = base / khw;
        // torch.sum(eps.view(O, I, -1), -1) order; the common kernel sizes get a
        // compile-time length so the ATen cascade unrolls into straight adds.
        auto esums = [&](auto kconst) {
            constexpr int K = decltype(kconst)::value;
            for (int pi = lane; pi < np; pi += kWave) {
                const float* e = data + pi * K;
                st<false>(T.esum + pbase + pi, aten_inner_sum([&](int64_t k) { return e[k]; }, (int64_t)K));
            }
        };
        auto generic = [&]() {
            for (int pi = lane; pi < np; pi += kWave) {
                const float* e = data + pi * khw;
                st<false>(T.esum + pbase + pi, aten_inner_sum([&](int64_t k) { return e[k]; }, khw));
            }
        };
        if constexpr (ESPEC == 2) {
            switch (khw) {
                case 9: esums(std::integral_constant<int, 9>{}); break;     // 3x3
                case 49: esums(std::integral_constant<int, 49>{}); break;   // 7x7
                case 25: esums(std::integral_constant<int, 25>{}); break;   // 5x5
                case 4: esums(std::integral_constant<int, 4>{}); break;     // 2x2
                default: generic();
            }
        } else if constexpr (ESPEC == 1) {
            if (khw == 9) esums(std::integral_constant<int, 9>{});
            else generic();
        } else {
            generic();
        }
    }
    wave_lds_sync();  // LDS is reused by this wave's next task
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the count is an immediate):
// every value 0..8, larger ones round down to 8 (waiting longer is always safe).
__device__ __forceinline__ void vm_wait_le(int n) {
    switch (n < 0 ? 0 : (n > 8 ? 8 : n)) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    }
}

// A whole-row task in two row batches (the single-model latency lever of DESIGN.md
// 3.1): the wave waits only for the load instructions that cover rows [0, h),
// reduces their ranges, builds their parameters and quantizes and STORES them
// while the loads of rows [h, nrows) are still landing; then it waits for those
// (vmcnt counts loads, LDS-DMA and stores together in issue order,
// MI355X_MICROARCH.md: at most lb younger operations outstanding means every load
// of the task has landed, for any lb <= the stores issued since) and does the
// rest.  The same per-row arithmetic and stores as compute_task's fixed-form loop
// (bit-identical); the KH*KW error sums run over the whole task at the end.
// Returns false (nothing done, loads still in flight) when the task does not split:
// the caller takes the one-wait path.
template <int MAXROWS, bool NT, int ESPEC>
__device__ __forceinline__ bool compute_task_split(const DevTensor& T, const DevTask& task, float* data, float* ls,
                                                   float* lmn, int lane) {
    const int n = task.n, nrows = task.nrows, len = (int)T.row_len;
    const bool clip = (T.flags & DFQ_CLIP) != 0;
    if (MAXROWS != 64 || nrows < 2 || !T.vec4 || !T.dst || (clip && !(T.clip_lo <= T.clip_hi))) return false;
    const int nj = n >> 2;
    const int M = (nj + kWave - 1) / kWave;   // load instructions issued (issue_task_load: 1 KiB each)
    const int h = min(nrows - 1, ((M >> 1) * 4 * kWave) / len);   // rows inside the first half of the loads
    if (M < 2 || h < 1) return false;
    const int m1 = (h * len + 4 * kWave - 1) / (4 * kWave);   // load instructions covering rows [0, h)
    const bool sym = is_sym(T.mode);
    const int khw = T.khw;
    const bool want_e = T.esum != nullptr;
    const float qmin = sym ? -(float)(1 << (T.bits - 1)) : 0.f;
    const float qmax = sym ? (float)((1 << (T.bits - 1)) - 1) : (float)((1 << T.bits) - 1);
    const int64_t base = task_elem_start(task, T);
    const int cb = !T.codes ? 0 : (T.code_bytes == 1 ? 1 : (T.code_bytes == 0 ? 3 : 2));
    const int em = !want_e ? 0 : (khw == 1 ? 1 : 2);
    const float* lrs = lmn + MAXROWS;
    const QParams pc{};
    auto rows = [&](int ra, int rb) {
        // ranges and parameters of rows [ra, rb) (compute_task's whole-row reduce)
        const int nr = rb - ra;
        int p2 = 1;
        while (p2 < nr && p2 < kWave) p2 <<= 1;
        const int G = kWave / p2;
        const int sub = lane / G, sl = lane % G;
        for (int r0 = ra; r0 < rb; r0 += p2) {
            const int r = r0 + sub;
            float vmin = INFINITY, vmax = -INFINITY;
            if (r < rb) {
                const int q4 = len >> 2;
                const float4* row4 = reinterpret_cast<const float4*>(data + r * len);
                for (int i = sl; i < q4; i += 4 * G) {
                    float4 v[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) v[u] = row4[min(i + u * G, q4 - 1)];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        vmin = min3_nc(min3_nc(vmin, v[u].x, v[u].y), v[u].z, v[u].w);
                        vmax = max3_nc(max3_nc(vmax, v[u].x, v[u].y), v[u].z, v[u].w);
                    }
                }
            }
            group_minmax(vmin, vmax, G);
            if (sl == 0 && r < rb) {
                const QParams p = make_qparams(vmin, vmax, T.bits, sym, T.flags, T.given_min, T.given_max);
                ls[r] = p.s;
                lmn[r] = p.mn;
                lmn[MAXROWS + r] = __builtin_amdgcn_rcpf(p.s);
                const int64_t row_g = task.row0 + r;
                if (T.scale) st<false>(T.scale + row_g, p.s);
                if (T.zero) st<false>(T.zero + row_g, p.mn);
            }
        }
        wave_lds_sync();
        // quantize rows [ra, rb): the fixed-form loop on that element span
        const int e0 = ra * len, ne = (rb - ra) * len;
        if (clip) quant_vec4_c<true, NT>(cb, em, T, ne, base + e0, data + e0, ls, lmn, lrs, pc, true, e0, lane, qmin,
                                         qmax, sym);
        else quant_vec4_c<false, NT>(cb, em, T, ne, base + e0, data + e0, ls, lmn, lrs, pc, true, e0, lane, qmin, qmax,
                                     sym);
    };
    vm_wait_le(M - m1);   // rows [0, h) have landed
    wave_lds_sync();
    rows(0, h);
    // the loop above issued >= one store per iteration of ceil(h len / 4 / 128)
    vm_wait_le(((h * len >> 2) + 2 * kWave - 1) / (2 * kWave));   // every load of the task has landed
    wave_lds_sync();
    rows(h, nrows);
    if (want_e && khw > 1) {   // 4. KHW error sums over the whole task (compute_task's step 4)
        wave_lds_sync();
        const int np = n / khw;
        const int64_t pbase = base / khw;
        auto esums = [&](auto kconst) {
            constexpr int K = decltype(kconst)::value;
            for (int pi = lane; pi < np; pi += kWave) {
                const float* e = data + pi * K;
                st<false>(T.esum + pbase + pi, aten_inner_sum([&](int64_t k) { return e[k]; }, (int64_t)K));
            }
        };
        auto generic = [&]() {
            for (int pi = lane; pi < np; pi += kWave) {
                const float* e = data + pi * khw;
                st<false>(T.esum + pbase + pi, aten_inner_sum([&](int64_t k) { return e[k]; }, khw));
            }
        };
        if constexpr (ESPEC == 2) {
            switch (khw) {
                case 9: esums(std::integral_constant<int, 9>{}); break;
                case 49: esums(std::integral_constant<int, 49>{}); break;
                case 25: esums(std::integral_constant<int, 25>{}); break;
                case 4: esums(std::integral_constant<int, 4>{}); break;
                default: generic();
            }
        } else if constexpr (ESPEC == 1) {
            if (khw == 9) esums(std::integral_constant<int, 9>{});
            else generic();
        } else {
            generic();
        }
    }
    wave_lds_sync();   // LDS is reused by this wave's next task
    return true;
}

// Diagnostics timeline (variant 13): per main-list task {start, data landed, done}
// in s_memrealtime ticks (100 MHz) plus the executing wave's hardware ids.
__device__ uint64_t* g_timeline = nullptr;
__device__ int64_t g_timeline_cap = 0;
// Diagnostics ablations (variant 13 only; dfq_debug_ablate): 1 no row reduce, 2 stores
// without the quantize arithmetic, 4 no quantize loop, 8 no input loads, 16 return at
// once (the launch alone), 32 task / tensor records and loads only (no compute),
// 64|4 the quantize arithmetic without its stores.
__device__ uint32_t g_ablate = 0;

template <int CHUNK, int MAXROWS, bool PREFETCH, bool NT = false, int ESPEC = 2, bool TL = false, bool SCREEN = true,
          bool FAST = true, bool SPLIT = false>
__global__ void __launch_bounds__(kBlockThreads)
sweep_main_kernel(const DevTensor* __restrict__ tensors, const DevTask* __restrict__ tasks, int64_t ntasks,
                  const uint32_t* __restrict__ slot_min, const uint32_t* __restrict__ slot_max) {
    constexpr int NB = PREFETCH ? 2 : 1;
    using Lay = LdsLayout<CHUNK, MAXROWS, NB>;
    __shared__ __attribute__((aligned(16))) float lds[Lay::kTotal];
    const int lane = threadIdx.x & (kWave - 1);
    const int w = wave_uniform(threadIdx.x >> 6);
    float* wl = lds + w * Lay::kPerWave;
    float* ls = wl + NB * CHUNK;
    float* lmn = ls + MAXROWS;
    const int64_t wave0 = (int64_t)blockIdx.x * kWavesPerBlock + w;
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    if constexpr (TL) {
        if (g_ablate & 16) return;   // diagnostics ablation: the launch alone
    }
    if constexpr (!PREFETCH) {
        DevTask task;
        if (wave0 < ntasks) task = tasks[wave0];
        for (int64_t t = wave0; t < ntasks; t += nwaves) {
            uint64_t tl0 = 0, tl1 = 0;
            uint32_t abl = 0;
            if constexpr (TL) {
                tl0 = wall_clock64();
                abl = g_ablate;
            }
            if (!(abl & 8)) issue_task_load<NT, SPLIT>(task, wl, lane);   // needs only the task record
            const DevTensor T = tensors[task.tensor];
            DevTask next = task;   // next record's scalar load overlaps this task
            if (t + nwaves < ntasks) next = tasks[t + nwaves];
            if constexpr (SPLIT && SCREEN && FAST && !TL) {
                // whole-row tasks in two row batches, the first stored while the
                // second's loads land (compute_task_split)
                if (task.nrows > 0 && compute_task_split<MAXROWS, NT, ESPEC>(T, task, wl, ls, lmn, lane)) {
                    task = next;
                    continue;
                }
            }
            vm_wait_all();
            if constexpr (TL) tl1 = wall_clock64();
            wave_lds_sync();
            if constexpr (TL) {
                if (abl & 32) {   // diagnostics ablation: task and tensor records (and loads) only
                    if (lane == 0 && T.row_len == -7) g_timeline[0] = 0;   // keeps T's load
                    task = next;
                    continue;
                }
            }
            float bmn = 0.f, bmx = 0.f;
            int goff = -1;
            if (task.nrows <= kGroupTag) {
                // row-group piece: the 4 waves of this block hold 4 pieces of R complete
                // rows.  Per-row partial (min, max) of this piece's row segments into
                // this wave's ls (max) / lmn (min) slots, one barrier, each wave combines
                // the rows its piece touches, a second barrier, then its row parameters.
                const int R = kGroupTag - task.nrows + 1;
                const int len = (int)T.row_len;
                const int g0 = (int)(task_elem_start(task, T) - (int64_t)task.row0 * len);   // piece offset in the group
                const int rf = g0 / len;
                const int rl = task.n > 0 ? (g0 + task.n - 1) / len : rf - 1;
                for (int r = 0; r < R; ++r) {
                    float vmin = INFINITY, vmax = -INFINITY;
                    if (r >= rf && r <= rl) {
                        const int a = max(r * len, g0) - g0, b = min((r + 1) * len, g0 + task.n) - g0;
                        if (T.vec4) {
                            for (int j = (a >> 2) + lane; j < (b >> 2); j += kWave) {
                                const float4 v = reinterpret_cast<const float4*>(wl)[j];
                                vmin = fminf(vmin, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
                                vmax = fmaxf(vmax, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
                            }
                        } else {
                            for (int e = a + lane; e < b; e += kWave) {
                                vmin = fminf(vmin, wl[e]);
                                vmax = fmaxf(vmax, wl[e]);
                            }
                        }
                        vmin = wave_min(vmin);
                        vmax = wave_max(vmax);
                    }
                    if (lane == 0) {
                        lmn[r] = vmin;
                        ls[r] = vmax;
                    }
                }
                block_lds_sync();
                constexpr int P = Lay::kPerWave;
                const int rr = rf + lane;   // one lane per row this piece touches
                float gmn = INFINITY, gmx = -INFINITY;
                if (rr <= rl) {
                    const float* b0 = lds + NB * CHUNK;   // wave 0's ls; lmn = ls + MAXROWS
#pragma unroll
                    for (int q = 0; q < kWavesPerBlock; ++q) {
                        gmx = fmaxf(gmx, b0[q * P + rr]);
                        gmn = fminf(gmn, b0[q * P + MAXROWS + rr]);
                    }
                }
                block_lds_sync();   // every wave has read the partials
                if (rr <= rl) {
                    const QParams p = make_qparams(gmn, gmx, T.bits, is_sym(T.mode), T.flags, T.given_min,
                                                   T.given_max);
                    ls[lane] = p.s;
                    lmn[lane] = p.mn;
                    lmn[MAXROWS + lane] = __builtin_amdgcn_rcpf(p.s);
                    if (rr * len >= g0) {   // the row starts in this piece: its parameters are stored once
                        const int64_t row_g = task.row0 + rr;
                        if (T.scale) st<false>(T.scale + row_g, p.s);
                        if (T.zero) st<false>(T.zero + row_g, p.mn);
                    }
                }
                wave_lds_sync();
                goff = g0 - rf * len;
            } else if (task.nrows < 0) {   // block-row piece: all 4 waves of this block are here
                float vmin = INFINITY, vmax = -INFINITY;
                if (T.vec4) {
                    for (int j = lane; j < (task.n >> 2); j += kWave) {
                        const float4 v = reinterpret_cast<const float4*>(wl)[j];
                        vmin = fminf(vmin, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
                        vmax = fmaxf(vmax, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
                    }
                } else {
                    for (int e = lane; e < task.n; e += kWave) {
                        vmin = fminf(vmin, wl[e]);
                        vmax = fmaxf(vmax, wl[e]);
                    }
                }
                vmin = wave_min(vmin);
                vmax = wave_max(vmax);
                // partial (min, max) in this wave's own row-parameter slots (unused by
                // block-row pieces), read by the block's other waves after the barrier
                if (lane == 0) {
                    ls[0] = vmin;
                    ls[1] = vmax;
                }
                block_lds_sync();
                constexpr int P = Lay::kPerWave;
                if (task.nrows == -kWavesPerBlock) {
                    const float* b0 = lds + NB * CHUNK;
                    bmn = fminf(fminf(b0[0], b0[P]), fminf(b0[2 * P], b0[3 * P]));
                    bmx = fmaxf(fmaxf(b0[1], b0[P + 1]), fmaxf(b0[2 * P + 1], b0[3 * P + 1]));
                } else {   // pairs of waves (0,1), (2,3)
                    const float* b0 = lds + (w & ~1) * P + NB * CHUNK;
                    bmn = fminf(b0[0], b0[P]);
                    bmx = fmaxf(b0[1], b0[P + 1]);
                }
                block_lds_sync();   // the slots are rewritten by the next task
            }
            uint64_t marks[4] = {0, 0, 0, 0};
            uint64_t* tlm = TL ? marks : nullptr;
            if (T.vec4)
                compute_task<MAXROWS, true, NT, ESPEC, SCREEN, FAST>(T, task, wl, ls, lmn, slot_min, slot_max, lane,
                                                                     bmn, bmx, goff, tlm, abl);
            else
                compute_task<MAXROWS, false, NT, ESPEC, SCREEN, FAST>(T, task, wl, ls, lmn, slot_min, slot_max, lane,
                                                                      bmn, bmx, goff, tlm, abl);
            if constexpr (TL) {
                if (lane == 0 && t < g_timeline_cap) {
                    uint32_t hw;
                    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                    uint32_t xcc;
                    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                    const uint64_t tl2 = wall_clock64();
                    uint64_t* r = g_timeline + 8 * t;   // {start, landed, params, quantized, done, tensor | xcc | hw ids, ...}
                    r[0] = tl0;
                    r[1] = tl1;
                    r[2] = marks[0];
                    r[3] = marks[1];
                    r[4] = tl2;
                    r[5] = ((uint64_t)task.tensor << 40) | ((uint64_t)(xcc & 0xFF) << 32) | hw;
                    r[6] = marks[2];
                    r[7] = marks[3];
                }
            }
            task = next;
        }
    } else {
        // Double-buffered: the next task's DMA is issued before this task computes.
        int cur = 0;
        int64_t t = wave0;
        if (t < ntasks) {
            const DevTask task = tasks[t];
            issue_task_load<NT>(task, wl, lane);
        }
        for (; t < ntasks; t += nwaves) {
            const DevTask task = tasks[t];
            const DevTensor T = tensors[task.tensor];
            vm_wait_all();          // this task's chunk (and the previous task's stores)
            wave_lds_sync();
            const int64_t tn = t + nwaves;
            if (tn < ntasks) {
                const DevTask nt = tasks[tn];
                issue_task_load<NT>(nt, wl + (cur ^ 1) * CHUNK, lane);
            }
            float* data = wl + cur * CHUNK;
            if (T.vec4) compute_task<MAXROWS, true, NT, ESPEC, SCREEN>(T, task, data, ls, lmn, slot_min, slot_max, lane);
            else compute_task<MAXROWS, false, NT, ESPEC, SCREEN>(T, task, data, ls, lmn, slot_min, slot_max, lane);
            cur ^= 1;
        }
    }
}

// ---------------------------------------------------------------------------
// Host: validation, task building, plans.
// ---------------------------------------------------------------------------
static bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

static int validate(const dfq_tensor_desc& d) {
    if (d.rows < 0 || d.row_len < 0) return DFQ_ERR_INVALID;
    if (!d.src && d.rows * d.row_len > 0) return DFQ_ERR_INVALID;
    if (d.bits < 2 || d.bits > 16) return DFQ_ERR_INVALID;
    if (d.mode < DFQ_TENSOR_ASYM || d.mode > DFQ_CHANNEL_SYM) return DFQ_ERR_INVALID;
    if (d.khw < 1) return DFQ_ERR_INVALID;
    if (d.esum && (d.row_len % d.khw) != 0) return DFQ_ERR_SHAPE;
    if (d.rows > INT32_MAX) return DFQ_ERR_UNSUPPORTED;
    const bool channel = d.mode >= DFQ_CHANNEL_ASYM;
    if (channel && (d.flags & DFQ_GIVEN_RANGE)) return DFQ_ERR_INVALID;
    if (d.flags & DFQ_DEVICE_RANGE) {
        if (channel || (d.flags & DFQ_GIVEN_RANGE) || !d.range_enc) return DFQ_ERR_INVALID;
    }
    return DFQ_OK;
}

struct Built {
    std::vector<DevTensor> tensors;
    std::vector<HostTask> reduce;
    std::vector<HostTask> blockrow;   // groups of kWavesPerBlock, placed first in the main list
    std::vector<HostTask> main;       // block rows, then tasks needing no reduce, then slot pieces
    std::vector<HostTask> slotted;    // slot pieces, in reduce order (appended to main at the end)
    int64_t slots = 0;
    int64_t elems = 0;
    int64_t algo_bytes = 0;
};

static DevTensor to_dev(const dfq_tensor_desc& d) {
    DevTensor t{};
    t.src = d.src; t.dst = d.dst; t.codes = d.codes; t.scale = d.scale; t.zero = d.zero; t.esum = d.esum;
    t.rows = d.rows; t.row_len = d.row_len; t.khw = d.khw; t.bits = d.bits; t.mode = d.mode;
    t.flags = d.flags; t.clip_lo = d.clip_lo; t.clip_hi = d.clip_hi;
    t.given_min = d.given_min; t.given_max = d.given_max;
    t.range_enc = (d.flags & DFQ_DEVICE_RANGE) ? d.range_enc : nullptr;
    t.inv_len = d.row_len > 0 ? 1.0f / (float)d.row_len : 0.f;
    t.len_magic = (d.row_len >= 2 && d.row_len < (int64_t(1) << 31))
                      ? (uint32_t)(((uint64_t(1) << 32) + (uint64_t)d.row_len - 1) / (uint64_t)d.row_len)
                      : 0u;
    t.code_bytes = (d.flags & DFQ_PACK_INT4) ? 0 : (d.bits <= 8 ? 1 : 2);   // 0: packed nibbles
    const int64_t n = d.rows * d.row_len;
    const bool channel = d.mode >= DFQ_CHANNEL_ASYM;
    bool v = (n % 4 == 0) && aligned(d.src, 16) && (!d.dst || aligned(d.dst, 16)) &&
             (!d.codes || aligned(d.codes, t.code_bytes ? 4 * t.code_bytes : 2)) &&
             (!d.esum || d.khw > 1 || aligned(d.esum, 16));
    if (channel) v = v && (d.row_len % 4 == 0);
    t.vec4 = v ? 1 : 0;
    return t;
}

// Piece length: a multiple of khw (E sums never straddle a piece), of 4 (vec4)
// and of 2 (packed nibbles: a byte never straddles two tasks).
static int piece_len(int khw, bool vec4, int chunk, bool packed = false) {
    const int unit = vec4 ? std::lcm(4, khw) : (packed ? std::lcm(2, khw) : khw);
    int p = (chunk / unit) * unit;
    return p > 0 ? p : -1;
}

// A/B and diagnostics switches (DFQ_SWEEP_VARIANT / _REDUCE_SPAN /
// _SHUFFLE / _BLOCKS_PER_CU) are read only by the diagnostics library
// (libdfq_diag.so, -DDFQ_DIAGNOSTICS); the product library runs the measured
// defaults whatever the environment says.

// DFQ_SWEEP_GROUP_ROWS=1 (diagnostics): per-channel rows of kChunk/2 .. 4 kChunk
// elements as row groups instead of whole-row tasks / block-row pieces.  Bit-exact
// and neutral (-1.4 .. +1.4 % on the five replicated configs interleaved on one box,
// profiles/r02/ab_group_rows.json: task fill is not what limits the 3x3 families),
// so the product keeps the simpler tasks.
static bool group_rows_enabled() {
    const char* e = ab_env("DFQ_SWEEP_GROUP_ROWS");
    return e && e[0] == '1';
}

// DFQ_SWEEP_BLOCKROW=0 (diagnostics library): long rows through the reduce launch
// instead (an alternative schedule, parity-tested against the default).
static bool blockrow_enabled() {
    const char* e = ab_env("DFQ_SWEEP_BLOCKROW");
    return !(e && e[0] == '0');
}

// Two-pass ranges pipelined in slabs (the quantize pass of slab k re-reading its
// inputs while they are still in the 256 MB Infinity Cache, on two streams) were
// measured slower at every slab size (profiles/r02/ab_slab.json: 16-256 MB slabs
// 1.34-3.9 ms per step against 1.11 for the two passes back to back) and deleted
// in round 4.

// Reduce-launch tasks: consecutive pieces of one range merged up to `span`
// elements per wave task (fewer same-address atomics, longer read streams).
// DFQ_SWEEP_REDUCE_SPAN overrides (A/B).
static int64_t reduce_span() {
    const char* e = ab_env("DFQ_SWEEP_REDUCE_SPAN");
    return (e && *e) ? std::max<int64_t>(1, atoll(e)) : 16384;
}
static void push_reduce(std::vector<HostTask>& R, const HostTask& k, int64_t span) {
    if (!R.empty()) {
        HostTask& p = R.back();
        if (p.slot == k.slot && p.tensor == k.tensor && p.elem_start + p.n == k.elem_start &&
            (int64_t)p.n + k.n <= span) {
            p.n += k.n;
            return;
        }
    }
    R.push_back(k);
}

// DFQ_SWEEP_SHUFFLE=<seed> (A/B): visit the main list's 4-task units (one
// workgroup's grid-stride step; block-row groups stay whole) in a seeded random
// order instead of list order.
static void shuffle_quads(Built& B) {
    const char* e = ab_env("DFQ_SWEEP_SHUFFLE");
    if (!e || !*e) return;
    const int64_t units = (int64_t)B.main.size() / kWavesPerBlock;
    if (units < 2) return;
    uint64_t x = (uint64_t)atoll(e) * 0x9E3779B97F4A7C15ull + 1;
    auto next = [&x]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (int64_t u = units - 1; u > 0; --u) {
        const int64_t v = (int64_t)(next() % (uint64_t)(u + 1));
        if (v != u)
            std::swap_ranges(B.main.begin() + u * kWavesPerBlock, B.main.begin() + (u + 1) * kWavesPerBlock,
                             B.main.begin() + v * kWavesPerBlock);
    }
}

static int build(const dfq_tensor_desc* descs, int32_t n, Built& B, const Variant& V) {
    const int64_t rspan = reduce_span();
    const bool use_blockrow = blockrow_enabled();
    const int kChunk = V.chunk, kMaxRows = V.max_rows;
    for (int32_t ti = 0; ti < n; ++ti) {
        const dfq_tensor_desc& d = descs[ti];
        int rc = validate(d);
        if (rc) return rc;
        DevTensor T = to_dev(d);
        const bool packed = (d.flags & DFQ_PACK_INT4) != 0;
        if (packed && d.bits > 4) return DFQ_ERR_INVALID;
        // packed codes need every task to start at an even element: per channel,
        // odd rows must come in pairs within one whole-row task (row_len <= chunk/2)
        if (packed && d.mode >= DFQ_CHANNEL_ASYM && (d.row_len & 1) && 2 * d.row_len > kChunk &&
            d.rows > 1)
            return DFQ_ERR_UNSUPPORTED;
        const int64_t total = d.rows * d.row_len;
        B.elems += total;
        // algorithmic bytes: read x, write dq / codes / E / per-row params once
        int64_t bytes = 4 * total;
        if (d.dst) bytes += 4 * total;
        if (d.codes) bytes += T.code_bytes ? (int64_t)T.code_bytes * total : total / 2;
        if (d.esum) bytes += 4 * (total / d.khw);
        const bool channel = d.mode >= DFQ_CHANNEL_ASYM;
        const int64_t nparams = channel ? d.rows : 1;
        if (d.scale) bytes += 4 * nparams;
        if (d.zero) bytes += 4 * nparams;
        B.algo_bytes += bytes;
        B.tensors.push_back(T);
        if (total == 0) continue;
        const int plen = piece_len(d.khw, T.vec4, kChunk, packed);
        if (plen <= 0) return DFQ_ERR_UNSUPPORTED;   // khw > kChunk
        // a given or device-resident range: single-pass tasks, no slot
        const bool given = (d.flags & (DFQ_GIVEN_RANGE | DFQ_DEVICE_RANGE)) != 0;
        const int64_t blen = channel ? d.row_len : total;   // the range's extent
        // Row groups (per-channel rows of kChunk/2 .. 4 kChunk elements): R whole rows
        // split into 4 balanced pieces, one per wave of a block, the rows' ranges
        // combined through LDS -- tasks hold ~R len / 4 elements instead of one row
        // (1,152-element 3x3 rows: 56 % of a task) or half a row.
        int64_t grp_rows = 0, grp_unit = 0;
        if (channel && use_blockrow && !V.prefetch && !given && d.row_len > kChunk / 2 &&
            d.row_len <= (int64_t)kWavesPerBlock * kChunk && group_rows_enabled()) {
            grp_unit = T.vec4 ? std::lcm<int64_t>(4, d.khw) : (packed ? std::lcm<int64_t>(2, d.khw) : d.khw);
            for (int64_t R = std::min<int64_t>(kGroupMaxRows, (int64_t)kWavesPerBlock * kChunk / d.row_len); R >= 1;
                 --R) {
                const int64_t piece = ceil_div(ceil_div(R * d.row_len, grp_unit), (int64_t)kWavesPerBlock) * grp_unit;
                if (piece <= kChunk) {
                    grp_rows = R;
                    break;
                }
            }
            // whole-row tasks already fill >= 85 % of a task: keep them
            if (grp_rows > 0 && d.row_len <= kChunk && (kChunk / d.row_len) * d.row_len * 100 >= 85 * kChunk)
                grp_rows = 0;
        }
        if (grp_rows > 0) {
            for (int64_t r0 = 0; r0 < d.rows; r0 += grp_rows) {
                const int64_t R = std::min<int64_t>(grp_rows, d.rows - r0);
                const int64_t tot = R * d.row_len;
                const int64_t piece = ceil_div(ceil_div(tot, grp_unit), (int64_t)kWavesPerBlock) * grp_unit;
                for (int i = 0; i < kWavesPerBlock; ++i) {
                    const int64_t off = std::min<int64_t>((int64_t)i * piece, tot);
                    HostTask k{};
                    k.tensor = ti; k.slot = -1; k.first = 0;
                    k.nrows = kGroupTag - (int32_t)(R - 1);
                    k.row0 = (int32_t)r0;
                    k.elem_start = r0 * d.row_len + off;
                    k.n = (int32_t)std::min<int64_t>(piece, tot - off);
                    B.blockrow.push_back(k);
                }
            }
            continue;
        }
        const bool block_row = use_blockrow && !V.prefetch && !given && blen <= (int64_t)kWavesPerBlock * plen &&
                               (!channel || d.row_len > kChunk);
        if (block_row) {
            // A group of 4 list entries = 4 waves of one block: one row in 4 pieces,
            // or (rows <= 2 pieces) two rows in 2 pieces each.  Balanced pieces:
            // the group waits for its slowest wave.
            const int64_t nr = channel ? d.rows : 1;
            const int gs = blen <= 2 * (int64_t)plen ? 2 : kWavesPerBlock;
            const int64_t unit = T.vec4 ? std::lcm<int64_t>(4, d.khw) : (packed ? std::lcm<int64_t>(2, d.khw) : d.khw);
            const int64_t bpl = ceil_div(ceil_div(blen, unit), (int64_t)gs) * unit;
            const int64_t rows_per_group = kWavesPerBlock / gs;
            for (int64_t r0 = 0; r0 < nr; r0 += rows_per_group) {
                for (int i = 0; i < kWavesPerBlock; ++i) {
                    const int64_t r = r0 + i / gs;
                    const int64_t off = (int64_t)(i % gs) * bpl;
                    HostTask k{};
                    k.tensor = ti; k.nrows = -gs; k.slot = -1;
                    if (r < nr) {
                        k.elem_start = r * blen + std::min<int64_t>(off, blen);
                        k.n = (int32_t)std::max<int64_t>(0, std::min<int64_t>(bpl, blen - off));
                        k.row0 = (int32_t)r; k.first = (i % gs == 0);
                    } else {   // padding half-group: no data, writes nothing
                        k.elem_start = r0 * blen; k.n = 0; k.row0 = (int32_t)r0; k.first = 0;
                    }
                    B.blockrow.push_back(k);
                }
            }
        } else if (channel && d.row_len <= kChunk) {
            // short rows (depthwise 3x3: 9 elements) are reduced one lane per row and run
            // the scalar path: at most one row per lane keeps such a task's latency
            // near a vector task's (single-model sweeps are latency-bound)
            const int64_t row_cap = d.row_len < 32 ? kWave : kMaxRows;
            int64_t rpt = std::max<int64_t>(1, std::min<int64_t>(row_cap, kChunk / d.row_len));
            if (packed && (d.row_len & 1) && rpt > 1) rpt &= ~int64_t(1);   // even task starts
            for (int64_t r = 0; r < d.rows; r += rpt) {
                const int64_t nr = std::min<int64_t>(rpt, d.rows - r);
                HostTask k{};
                k.elem_start = r * d.row_len; k.tensor = ti; k.n = (int32_t)(nr * d.row_len);
                k.row0 = (int32_t)r; k.nrows = (int32_t)nr; k.slot = -1; k.first = 0;
                B.main.push_back(k);
            }
        } else if (channel) {   // long rows: one slot per row
            for (int64_t r = 0; r < d.rows; ++r) {
                const int64_t slot = B.slots++;
                for (int64_t off = 0; off < d.row_len; off += plen) {
                    HostTask k{};
                    k.elem_start = r * d.row_len + off; k.tensor = ti;
                    k.n = (int32_t)std::min<int64_t>(plen, d.row_len - off);
                    k.row0 = (int32_t)r; k.nrows = 0; k.slot = (int32_t)slot; k.first = (off == 0);
                    push_reduce(B.reduce, k, rspan);
                    B.slotted.push_back(k);
                }
            }
        } else {                // tensor modes: one slot per tensor (none for a given range)
            const int64_t slot = given ? -1 : B.slots++;
            for (int64_t off = 0; off < total; off += plen) {
                HostTask k{};
                k.elem_start = off; k.tensor = ti; k.n = (int32_t)std::min<int64_t>(plen, total - off);
                k.row0 = 0; k.nrows = 0; k.slot = (int32_t)slot; k.first = (off == 0);
                if (!given) {
                    push_reduce(B.reduce, k, rspan);
                    B.slotted.push_back(k);
                } else {
                    B.main.push_back(k);
                }
            }
        }
    }
    B.main.insert(B.main.begin(), B.blockrow.begin(), B.blockrow.end());
    B.main.insert(B.main.end(), B.slotted.begin(), B.slotted.end());   // slot pieces after the single-pass tasks
    shuffle_quads(B);
    return DFQ_OK;
}

// The device form of a task list (DevTask: the first element's address, the
// tensor's vector flag) into `out`.
static void put_tasks(const std::vector<HostTask>& h, const std::vector<DevTensor>& T, char* out) {
    DevTask* d = reinterpret_cast<DevTask*>(out);
    for (size_t i = 0; i < h.size(); ++i) {
        const HostTask& k = h[i];
        const DevTensor& t = T[k.tensor];
        d[i] = DevTask{t.src + k.elem_start, k.tensor, k.n, k.row0, k.nrows, k.slot,
                       (k.first ? 1 : 0) | (t.vec4 ? 2 : 0)};
    }
}

static int variant_from_env() {
    const char* e = ab_env("DFQ_SWEEP_VARIANT");
    if (!e || !*e) return kDefaultVariant;
    const int v = atoi(e);
    return (v >= 0 && v < kNumVariants) ? v : kDefaultVariant;
}


// Small lists (see build_planned) run variant 10's 1,536-element tasks; one round
// of resident sweep blocks on the 256-CU part is 4 per CU.
constexpr int kSmallVariant = 10;
constexpr int64_t kResidentBlocks = 4 * 256;

static int lds_bytes(const Variant& V) {
    return 4 * kWavesPerBlock * ((V.prefetch ? 2 : 1) * V.chunk + 3 * V.max_rows);
}

using MainKernel = void (*)(const DevTensor*, const DevTask*, int64_t, const uint32_t*, const uint32_t*);

static MainKernel main_kernel(int variant) {
#define DFQ_V(i) kVariants[i].chunk, kVariants[i].max_rows, kVariants[i].prefetch
#ifndef DFQ_DIAGNOSTICS
    // the product library carries the default variant and the small-list one
    if (variant == kSmallVariant) return sweep_main_kernel<DFQ_V(kSmallVariant), true, 1>;
    return sweep_main_kernel<DFQ_V(kDefaultVariant), true, 1, false, true, true, kDefaultVariant == 16>;
#else
    switch (variant) {
        case 1: return sweep_main_kernel<DFQ_V(1)>;
        case 2: return sweep_main_kernel<DFQ_V(2)>;
        case 3: return sweep_main_kernel<DFQ_V(3)>;
        case 4: return sweep_main_kernel<DFQ_V(4)>;
        case 5: return sweep_main_kernel<DFQ_V(5), true>;
        case 6: return sweep_main_kernel<DFQ_V(6), true, 1>;
        case 7: return sweep_main_kernel<DFQ_V(7), true, 0>;
        case 8: return sweep_main_kernel<DFQ_V(8), true, 1>;
        case 9: return sweep_main_kernel<DFQ_V(9), true, 1>;
        case 10: return sweep_main_kernel<DFQ_V(10), true, 1>;
        case 11: return sweep_main_kernel<DFQ_V(11), true, 1>;
        case 12: return sweep_main_kernel<DFQ_V(12), true, 0>;
        case 13: return sweep_main_kernel<DFQ_V(13), true, 1, true>;
        case 14: return sweep_main_kernel<DFQ_V(14), true, 1, false, false>;
        case 15: return sweep_main_kernel<DFQ_V(15), true, 1, false, true, false>;
        case 16: return sweep_main_kernel<DFQ_V(16), true, 1, false, true, true, true>;
        default: return sweep_main_kernel<DFQ_V(0)>;
    }
#endif
#undef DFQ_V
}

// Grid: up to 64 blocks per CU (16384 blocks), far more than are resident (4-5
// per CU for the sweep kernels).  Each wave's grid-stride list is then only a
// few tasks long and the dispatcher hands CUs new blocks as old ones retire --
// dynamic load balance over tasks of uneven cost.  Measured against resident-
// only grids (profiles/r01/ab_grid.txt): MobileNetV2 +25 %, ResNet-50 / DeepLab
// +4-6 %; 32-128 per CU are within a few %, fully unrolled grids (one block per
// 4 tasks) lose 10 %.  DFQ_SWEEP_BLOCKS_PER_CU overrides (A/B).
constexpr int kBlocksPerCu = 64;
static int blocks_per_cu() {
    static const int v = [] {
        const char* e = ab_env("DFQ_SWEEP_BLOCKS_PER_CU");
        return e && *e ? std::max(1, std::min(1024, atoi(e))) : kBlocksPerCu;
    }();
    return v;
}
static int grid_for(int64_t ntasks) {
    const int64_t want = ceil_div(ntasks, kWavesPerBlock);
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, 256 * (int64_t)blocks_per_cu()));
}
static int grid_for_variant(int64_t ntasks, int) { return grid_for(ntasks); }

static void launch_main(int variant, int grid, hipStream_t s, const DevTensor* t, const DevTask* k, int64_t n,
                        const uint32_t* smin, const uint32_t* smax) {
    hipLaunchKernelGGL(main_kernel(variant), dim3(grid), dim3(kBlockThreads), 0, s, t, k, n, smin, smax);
}

}  // namespace dfq

using namespace dfq;

struct dfq_sweep_plan {
    int variant = kDefaultVariant;
    DevTensor* d_tensors = nullptr;
    DevTask* d_reduce = nullptr;
    DevTask* d_main = nullptr;
    uint32_t* d_slots = nullptr;   // [slots] mins then [slots] maxs
    void* d_owned = nullptr;       // the tables' allocation when no workspace was given
    int64_t n_reduce = 0, n_main = 0, n_slots = 0, n_tensors = 0, n_elems = 0, algo_bytes = 0;
};

namespace dfq {
// Device layout of a plan's tables: [tensors | reduce tasks | main tasks | slots],
// each 256-B aligned (one allocation or one caller workspace).
struct PlanLayout {
    int64_t o_tensors = 0, o_reduce = 0, o_main = 0, o_slots = 0, total = 0;
};
static int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }
static PlanLayout plan_layout(const Built& B, int64_t n) {
    PlanLayout L;
    L.o_tensors = 0;
    L.o_reduce = L.o_tensors + align256((int64_t)sizeof(DevTensor) * n);
    L.o_main = L.o_reduce + align256((int64_t)sizeof(DevTask) * (int64_t)B.reduce.size());
    L.o_slots = L.o_main + align256((int64_t)sizeof(DevTask) * (int64_t)B.main.size());
    L.total = L.o_slots + align256((int64_t)sizeof(uint32_t) * 2 * B.slots);
    return L;
}
}  // namespace dfq

// The plan's kernel variant and task table.  A diagnostics DFQ_SWEEP_VARIANT wins.
// Otherwise the default variant's 2,048-element tasks, unless the list is small
// enough that 1,536-element tasks (variant 10) still fit in ONE round of resident
// blocks (4 per CU at 97 VGPRs): a one-round grid of range-dependent tasks is
// latency-bound, and 4/3 as many waves hide more of it (MobileNetV2 single model:
// 560 -> 747 blocks).  Lists past one round keep 2,048 (DeepLab's single model at
// 1,536 needs 1,123 blocks and measured 12.0 against 9.2 us; profiles/r06/chunk_rule_ab_r06o.jsonl).
static int build_planned(const dfq_tensor_desc* descs, int32_t n, Built& B, int& variant) {
    const char* e = ab_env("DFQ_SWEEP_VARIANT");
    variant = variant_from_env();
    if (int rc = build(descs, n, B, kVariants[variant])) return rc;
    if ((e && *e) || variant != kDefaultVariant || kDefaultVariant != 6) return DFQ_OK;
    const int64_t limit = kResidentBlocks;
    const int64_t blocks = ceil_div((int64_t)B.main.size(), (int64_t)kWavesPerBlock);
    if (B.main.empty() || 4 * blocks > 3 * limit) return DFQ_OK;   // 4/3 the tasks would not fit one round
    Built S;
    if (build(descs, n, S, kVariants[kSmallVariant]) != DFQ_OK) return DFQ_OK;
    if (ceil_div((int64_t)S.main.size(), (int64_t)kWavesPerBlock) > limit) return DFQ_OK;
    B = std::move(S);
    variant = kSmallVariant;
    return DFQ_OK;
}

extern "C" int64_t dfq_sweep_plan_ws_bytes(const dfq_tensor_desc* descs, int32_t n) {
    if ((n > 0 && !descs) || n < 0) return -1;
    Built B;
    int variant = 0;
    if (build_planned(descs, n, B, variant)) return -1;
    return plan_layout(B, n).total;
}

// ws == NULL: the plan owns one hipMalloc'ed table block (blocking copy).  Else the
// tables go to the caller's stream-ordered workspace: one copy on `stream`, then a
// sync of that stream (the host staging dies with the call).
static int sweep_plan_create_impl(const dfq_tensor_desc* descs, int32_t n, void* ws, int64_t ws_bytes,
                                  hipStream_t stream, dfq_sweep_plan** out) {
    if (!out || (n > 0 && !descs) || n < 0) return DFQ_ERR_INVALID;
    *out = nullptr;
    int variant = 0;
    Built B;
    int rc = build_planned(descs, n, B, variant);
    if (rc) return rc;
    const PlanLayout Lo = plan_layout(B, n);
    if (ws && (ws_bytes < Lo.total || reinterpret_cast<uintptr_t>(ws) % 256 != 0)) return DFQ_ERR_WORKSPACE;
    dfq_sweep_plan* p = new (std::nothrow) dfq_sweep_plan();
    if (!p) return DFQ_ERR_NOMEM;
    p->variant = variant;
    p->n_reduce = (int64_t)B.reduce.size();
    p->n_main = (int64_t)B.main.size();
    p->n_slots = B.slots;
    p->n_tensors = n;
    p->n_elems = B.elems;
    p->algo_bytes = B.algo_bytes;
    hipError_t e = hipSuccess;
    char* base = static_cast<char*>(ws);
    if (!base) {
        e = hipMalloc(&p->d_owned, Lo.total);
        base = static_cast<char*>(p->d_owned);
    }
    p->d_tensors = reinterpret_cast<DevTensor*>(base + Lo.o_tensors);
    p->d_reduce = reinterpret_cast<DevTask*>(base + Lo.o_reduce);
    p->d_main = reinterpret_cast<DevTask*>(base + Lo.o_main);
    p->d_slots = reinterpret_cast<uint32_t*>(base + Lo.o_slots);
    if (e == hipSuccess) {
        std::vector<char> blob(Lo.o_slots, 0);   // the host-built tables
        if (n > 0) std::memcpy(blob.data() + Lo.o_tensors, B.tensors.data(), sizeof(DevTensor) * n);
        put_tasks(B.reduce, B.tensors, blob.data() + Lo.o_reduce);
        put_tasks(B.main, B.tensors, blob.data() + Lo.o_main);
        if (ws) {   // stream-ordered: pinned staging, no host synchronisation
            e = stage_h2d(base, blob.data(), Lo.o_slots, stream);
        } else {
            e = hipMemcpy(base, blob.data(), Lo.o_slots, hipMemcpyHostToDevice);
        }
    }
    if (e != hipSuccess) {
        set_last_hip_error(e);
        (void)hipFree(p->d_owned);
        delete p;
        return DFQ_ERR_HIP;
    }
    *out = p;
    return DFQ_OK;
}

extern "C" int dfq_sweep_plan_create(const dfq_tensor_desc* descs, int32_t n, dfq_sweep_plan** out) {
    return sweep_plan_create_impl(descs, n, nullptr, 0, nullptr, out);
}

extern "C" int dfq_sweep_plan_create_ws(const dfq_tensor_desc* descs, int32_t n, void* ws, int64_t ws_bytes,
                                        void* stream, dfq_sweep_plan** out) {
    if (!ws) return DFQ_ERR_WORKSPACE;
    return sweep_plan_create_impl(descs, n, ws, ws_bytes, static_cast<hipStream_t>(stream), out);
}

extern "C" int dfq_sweep_plan_execute(dfq_sweep_plan* p, void* stream) {
    if (!p) return DFQ_ERR_INVALID;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (p->n_reduce > 0) {
        DFQ_HIP_CHECK(hipMemsetAsync(p->d_slots, 0xFF, sizeof(uint32_t) * p->n_slots, s));
        DFQ_HIP_CHECK(hipMemsetAsync(p->d_slots + p->n_slots, 0x00, sizeof(uint32_t) * p->n_slots, s));
    }
    // one reduce launch over every slot piece, then one main launch
    if (p->n_reduce > 0) {
        hipLaunchKernelGGL(sweep_reduce_kernel, dim3(grid_for(p->n_reduce)), dim3(kBlockThreads), 0, s, p->d_tensors,
                           p->d_reduce, p->n_reduce, p->d_slots, p->d_slots + p->n_slots);
        DFQ_LAUNCH_CHECK();
    }
    if (p->n_main > 0) {
        launch_main(p->variant, grid_for_variant(p->n_main, p->variant), s, p->d_tensors, p->d_main, p->n_main,
                    p->d_slots, p->d_slots + p->n_slots);
        DFQ_LAUNCH_CHECK();
    }
    return DFQ_OK;
}

extern "C" int dfq_sweep_plan_stats(const dfq_sweep_plan* p, dfq_sweep_stats* st) {
    if (!p || !st) return DFQ_ERR_INVALID;
    st->n_tensors = p->n_tensors;
    st->n_elems = p->n_elems;
    st->n_tasks_reduce = p->n_reduce;
    st->n_tasks_main = p->n_main;
    st->algo_bytes = p->algo_bytes;
    st->launches = (p->n_reduce > 0 ? 1 : 0) + (p->n_main > 0 ? 1 : 0);
    st->grid_blocks = p->n_main > 0 ? grid_for_variant(p->n_main, p->variant) : 0;
    st->variant = p->variant;
    return DFQ_OK;
}

extern "C" int dfq_sweep_plan_destroy(dfq_sweep_plan* p) {
    if (!p) return DFQ_OK;
    (void)hipFree(p->d_owned);   // NULL for workspace-backed plans
    delete p;
    return DFQ_OK;
}

// ---------------------------------------------------------------------------
// Single-tensor path: the workspace carries [slots | tensor | tasks]; the host-built
// tables go up through the pinned staging ring (stage_h2d), so a call is
// asynchronous on the caller's stream like every other entry point.
// ---------------------------------------------------------------------------
namespace dfq {
static size_t single_ws_layout(const Built& B, size_t* off_tensor, size_t* off_reduce, size_t* off_main) {
    size_t o = 0;
    o += sizeof(uint32_t) * 2 * (size_t)B.slots;
    o = (o + 63) & ~size_t(63);
    *off_tensor = o; o += sizeof(DevTensor) * B.tensors.size();
    o = (o + 63) & ~size_t(63);
    *off_reduce = o; o += sizeof(DevTask) * B.reduce.size();
    o = (o + 63) & ~size_t(63);
    *off_main = o; o += sizeof(DevTask) * B.main.size();
    return o;
}
}  // namespace dfq

extern "C" int dfq_quantize_ws_bytes(const dfq_tensor_desc* d, size_t* bytes) {
    if (!d || !bytes) return DFQ_ERR_INVALID;
    Built B;
    int rc = build(d, 1, B, kVariants[kDefaultVariant]);
    if (rc) return rc;
    size_t a, b, c;
    *bytes = single_ws_layout(B, &a, &b, &c);
    return DFQ_OK;
}

extern "C" int dfq_quantize_tensor(const dfq_tensor_desc* d, void* ws, size_t ws_bytes, void* stream) {
    if (!d) return DFQ_ERR_INVALID;
    Built B;
    int rc = build(d, 1, B, kVariants[kDefaultVariant]);
    if (rc) return rc;
    size_t ot, orr, om;
    const size_t need = single_ws_layout(B, &ot, &orr, &om);
    if (!ws || ws_bytes < need) return DFQ_ERR_WORKSPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    char* base = static_cast<char*>(ws);
    uint32_t* slots = reinterpret_cast<uint32_t*>(base);
    DevTensor* dt = reinterpret_cast<DevTensor*>(base + ot);
    DevTask* dr = reinterpret_cast<DevTask*>(base + orr);
    DevTask* dm = reinterpret_cast<DevTask*>(base + om);
    // one table blob [tensor | reduce tasks | main tasks] through the pinned staging
    // ring: stream-ordered, no host synchronisation
    {
        const size_t tb = om + sizeof(DevTask) * B.main.size() - ot;
        std::vector<char> blob(tb, 0);
        std::memcpy(blob.data(), B.tensors.data(), sizeof(DevTensor));
        put_tasks(B.reduce, B.tensors, blob.data() + (orr - ot));
        put_tasks(B.main, B.tensors, blob.data() + (om - ot));
        DFQ_HIP_CHECK(stage_h2d(dt, blob.data(), tb, s));
    }
    if (!B.reduce.empty()) {
        DFQ_HIP_CHECK(hipMemsetAsync(slots, 0xFF, sizeof(uint32_t) * B.slots, s));
        DFQ_HIP_CHECK(hipMemsetAsync(slots + B.slots, 0x00, sizeof(uint32_t) * B.slots, s));
        hipLaunchKernelGGL(sweep_reduce_kernel, dim3(grid_for((int64_t)B.reduce.size())), dim3(kBlockThreads), 0, s,
                           dt, dr, (int64_t)B.reduce.size(), slots, slots + B.slots);
        DFQ_LAUNCH_CHECK();
    }
    if (!B.main.empty()) {
        launch_main(kDefaultVariant, grid_for_variant((int64_t)B.main.size(), kDefaultVariant), s, dt, dm,
                    (int64_t)B.main.size(), slots,
                    slots + B.slots);
        DFQ_LAUNCH_CHECK();
    }
    return DFQ_OK;
}

#ifdef DFQ_DIAGNOSTICS
// Diagnostics: point variant 13's timeline at `buf` (4 uint64 per main-list task,
// `cap` tasks); NULL/0 disables.  Not part of the reference interface.
extern "C" int dfq_debug_timeline(void* buf, int64_t cap) {
    uint64_t* p = static_cast<uint64_t*>(buf);
    DFQ_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_timeline), &p, sizeof(p)));
    DFQ_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_timeline_cap), &cap, sizeof(cap)));
    return DFQ_OK;
}

// Diagnostics: variant 13's ablation bits (g_ablate); results are wrong while set.
extern "C" int dfq_debug_ablate(uint32_t flags) {
    DFQ_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_ablate), &flags, sizeof(flags)));
    return DFQ_OK;
}
#endif  // DFQ_DIAGNOSTICS

// Code-object loading at library initialisation (dfq_preload): the first launch of
// a kernel otherwise pays for loading its translation unit's code object.
namespace dfq {
hipError_t preload_sweep() {
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(main_kernel(kDefaultVariant)));
    if (e == hipSuccess) e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(sweep_reduce_kernel));
    return e;
}
}  // namespace dfq
