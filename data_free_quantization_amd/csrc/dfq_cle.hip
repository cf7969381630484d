// Cross-layer equalization on the GPU (gfx950): the whole cross_layer_equalization
// loop of Cross_layer_equal.py:63-116 device-resident (dfq_cle_plan_*).
// Relations are grouped into independent chains (connected components of the
// tensors they touch) and the k-th relation of every chain runs in one launch;
// the per-iteration metric sum_l mean|W_l - W_l_prev| (fp32 torch.mean in ATen's
// reduction order, then numpy's pairwise float64 sum) and the stop rule are
// evaluated on the device.  The host enqueues iterations and polls the stop
// rule's word in pinned memory.  One relation at a time: dfq_cle_relation.hip.
// fp32 arithmetic is ordered exactly as the reference's torch CPU ops.
#include "dfq_cle_common.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <list>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <new>
#include <numeric>
#include <vector>

using namespace dfq;

// ============================================================================
// Device-resident CLE loop (dfq_cle_plan_*)
// ============================================================================
namespace dfq {

struct CleRel {
    float* w1;
    float* w2;
    float* b1;
    float* bnw;
    float* bnb;
    float* sacc;
    int64_t c1, len1, o2, i2, khw2, o2g;
    int64_t moff;       // this relation's [W1 | W2] range words inside one parity's mins (and maxs)
    int32_t sacc_init;
    int32_t vec1;       // W1 rows 16-B aligned (float4 path)
    int32_t vec2;       // W2 contiguous channel segments 16-B aligned (i2 == 1)
    int32_t fuse_next;  // >= 0: this relation's W2 is that relation's W1 -- the rescale
                        // of W2 also produces its row ranges (fused schedule)
    int32_t dw_prev;    // >= 0: this relation's W1 is that relation's depthwise W2: its W1 row
                        // ranges are derived (cle_rel_scale) and both run in one launch
    int32_t w1_self;    // 1: its W1 rescale also writes the next iteration's W1 row ranges
    int32_t w2_self;    // 1: its depthwise W2 rescale (kApplyDwBoth) writes the next W2 ranges
};

// Range-launch kinds: W1 rows, W2 contiguous channels (i2 == 1), W2 row tiles
// (i2 > 1, ordered-uint atomics), reset of the OTHER parity's W2 words.
// Rescale-launch kinds: W1 elements, W2 elements, per-channel vectors.
enum : int32_t { kRangeW1 = 0, kRangeW2Contig = 1, kRangeW2Tile = 2, kRangeReset = 3, kRangeResetW1 = 4 };
enum : int32_t { kApplyW1 = 0, kApplyW2Contig = 1, kApplyW2Tile = 2, kApplyChannels = 3, kApplyDwBoth = 4 };

struct CleTask {
    int32_t rel;
    int32_t kind;
    int64_t a, b;     // rows / channels / elements [a, b)
    int64_t c0, c1;   // W2 tiles: columns [c0, c1) (one thread each)
};

struct CleLayer {
    float* w;
    float* snap;
    int64_t n;
    int64_t nt;   // torch.mean's chunks (1: serial sum)
};

// One fp32 torch.mean chunk (a thread's share of at::parallel_for in
// two_pass_reduction): elements [c0, c0 + len) of layer `layer`, slot t.
struct CleChunk {
    int32_t layer;
    int32_t t;
    int64_t c0;
    int64_t len;
};

struct CleState {
    double diff;         // Cross_layer_equal.py `diff`
    double thr;          // Treshhold
    int32_t iter_count;  // consecutive iterations with |diff - diff_tmp| <= 1e-9
    int32_t iters;       // iterations run
    int32_t done;
    int32_t count;       // Count
    int32_t max_iters;
    int32_t error;       // 2: a tile block saw an unexpected iteration parity (never expected)
};

constexpr int kCleW1RowsPerTask = 4;       // one wave per row
constexpr int kCleW2ChansPerTask = 4;      // one wave per contiguous column

// Short rows (< 64 elements: depthwise filters, the first layers' rows) take a
// group of G lanes each (G = the next power of two >= the length), 64 / G rows
// per wave, instead of a whole wave per row -- 4-7x fewer tasks for MobileNetV2's
// depthwise filters and narrow rows, whose cost is the dependent round trips.
__host__ __device__ inline int row_group_lanes(int64_t len) {
    if (len >= 64) return 64;
    int g = 1;
    while (g < len) g <<= 1;
    return g;
}
// rows (or channel segments) per task: 4 waves x the rows a wave holds
__host__ __device__ inline int64_t rows_per_task(int64_t len) { return 4 * (64 / row_group_lanes(len)); }

__device__ __forceinline__ float group_min(float v, int g) {
    for (int off = g >> 1; off >= 1; off >>= 1) v = fminf(v, __shfl_xor(v, off, 64));
    return v;
}
__device__ __forceinline__ float group_max(float v, int g) {
    for (int off = g >> 1; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return v;
}
// f(row, active, sub-lane, G) for rows [a, b) of length len < 64: every lane of
// the block calls f the same number of times (shuffles stay convergent)
template <class F>
__device__ __forceinline__ void for_short_rows(int64_t a, int64_t b, int64_t len, F&& f) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int G = row_group_lanes(len), rpw = 64 / G;
    const int sub = lane / G, sl = lane % G;
    for (int64_t base = a + (int64_t)wv * rpw; base < b; base += (int64_t)(kThreads / 64) * rpw) {
        const int64_t c = base + sub;
        f(c, c < b, sl, G);
    }
}
constexpr int64_t kCleChansPerTask = 1024;
// Rescale tasks hold rows_per_task rows (one per wave).  W1 tasks of short rows
// (under kCleW1SmallElems elements per task: MobileNetV2's expand convs) take twice
// that: step 0 of MobileNetV2 had 1,648 W1 tasks of ~2 us in 2,433 blocks, more than
// are resident, so its last blocks started 8.7 us into the launch
// (profiles/r06/cle_tl_r06h.log); A/B profiles/r06/cle_ab_rows_r06i.jsonl.
// Diagnostics switches: DFQ_CLE_W1_ROWS (a fixed factor) / DFQ_CLE_DW_ROWS.
constexpr int64_t kCleW1SmallElems = 2048, kCleDwRowsMult = 1;

// min / max of n floats at p, one wave, 4 loads in flight per lane
__device__ __forceinline__ void wave_range(const float* __restrict__ p_, int64_t n, bool vec, int lane, float& vmin,
                                           float& vmax) {
    const DFQ_GLOBAL float* __restrict__ p = (const DFQ_GLOBAL float*)p_;   // global: not flat
    vmin = INFINITY;
    vmax = -INFINITY;
    if (vec) {
        const DFQ_GLOBAL f32x4* p4 = (const DFQ_GLOBAL f32x4*)p;
        const int64_t n4 = n >> 2;
        for (int64_t i = lane; i < n4; i += 4 * 64) {
            f32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n4) v[u] = p4[i + 64 * u];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n4) {
                    vmin = fminf(vmin, fminf(fminf(v[u].x, v[u].y), fminf(v[u].z, v[u].w)));
                    vmax = fmaxf(vmax, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)));
                }
        }
    } else {
        for (int64_t i = lane; i < n; i += 4 * 64) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n) v[u] = p[i + 64 * u];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n) {
                    vmin = fminf(vmin, v[u]);
                    vmax = fmaxf(vmax, v[u]);
                }
        }
    }
    cle_wave_minmax(vmin, vmax);
}

// p[0..n) *= f(), one wave; 4 loads in flight per lane before the stores.  The
// factor (range-table reads) is evaluated after the first loads are issued, so
// the data and the range words are one memory round trip, not two.
template <class F>
__device__ __forceinline__ void wave_scale(float* __restrict__ p_, int64_t n, bool vec, int lane, F&& factor) {
    DFQ_GLOBAL float* __restrict__ p = (DFQ_GLOBAL float*)p_;   // global: not flat
    float f = 0.f;
    bool have = false;
    if (vec) {
        DFQ_GLOBAL f32x4* p4 = (DFQ_GLOBAL f32x4*)p;
        const int64_t n4 = n >> 2;
        for (int64_t i = lane; i < n4; i += 4 * 64) {
            f32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n4) v[u] = p4[i + 64 * u];
            if (!have) {
                f = factor();
                have = true;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n4) {
                    v[u].x = v[u].x * f;
                    v[u].y = v[u].y * f;
                    v[u].z = v[u].z * f;
                    v[u].w = v[u].w * f;
                    p4[i + 64 * u] = v[u];
                }
        }
    } else {
        for (int64_t i = lane; i < n; i += 4 * 64) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n) v[u] = p[i + 64 * u];
            if (!have) {
                f = factor();
                have = true;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n) p[i + 64 * u] = v[u] * f;
        }
    }
}

// wave_scale that also returns the (min, max) of the products (every lane).
template <class F>
__device__ __forceinline__ void wave_scale_mm(float* __restrict__ p_, int64_t n, bool vec, int lane, float& vmin,
                                              float& vmax, F&& factor) {
    DFQ_GLOBAL float* __restrict__ p = (DFQ_GLOBAL float*)p_;   // global: not flat
    vmin = INFINITY;
    vmax = -INFINITY;
    float f = 0.f;
    bool have = false;
    if (vec) {
        DFQ_GLOBAL f32x4* p4 = (DFQ_GLOBAL f32x4*)p;
        const int64_t n4 = n >> 2;
        for (int64_t i = lane; i < n4; i += 4 * 64) {
            f32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n4) v[u] = p4[i + 64 * u];
            if (!have) {
                f = factor();
                have = true;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n4) {
                    v[u].x = v[u].x * f;
                    v[u].y = v[u].y * f;
                    v[u].z = v[u].z * f;
                    v[u].w = v[u].w * f;
                    p4[i + 64 * u] = v[u];
                    vmin = fminf(vmin, fminf(fminf(v[u].x, v[u].y), fminf(v[u].z, v[u].w)));
                    vmax = fmaxf(vmax, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)));
                }
        }
    } else {
        for (int64_t i = lane; i < n; i += 4 * 64) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n) v[u] = p[i + 64 * u];
            if (!have) {
                f = factor();
                have = true;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + 64 * u < n) {
                    const float y = v[u] * f;
                    p[i + 64 * u] = y;
                    vmin = fminf(vmin, y);
                    vmax = fmaxf(vmax, y);
                }
        }
    }
    cle_wave_minmax(vmin, vmax);
}

// p[0..n) *= f() and the (min, max) of the products, one wave (scalar loads:
// used for short depthwise rows); the factor is read after the first load
template <class F>
__device__ __forceinline__ void wave_scale_range(float* __restrict__ p_, int64_t n, int lane, float& vmin, float& vmax,
                                                 F&& factor) {
    DFQ_GLOBAL float* __restrict__ p = (DFQ_GLOBAL float*)p_;   // global: not flat
    vmin = INFINITY;
    vmax = -INFINITY;
    float f = 0.f;
    bool have = false;
    for (int64_t i = lane; i < n; i += 64) {
        const float x = p[i];
        if (!have) {
            f = factor();
            have = true;
        }
        const float y = x * f;
        p[i] = y;
        vmin = fminf(vmin, y);
        vmax = fmaxf(vmax, y);
    }
    cle_wave_minmax(vmin, vmax);
}

// W2 row tiles with KH*KW = khw in (1, kTileMaxKhw] and one group: thread t owns
// the tile's flattened positions p = t + 256 m (m < khw) -- consecutive threads
// on consecutive floats, khw independent loads per row in flight -- instead of
// one thread per column walking its khw floats serially.
constexpr int kTileMaxKhw = 9;   // 3x3 (and 2x2); larger kernels keep the per-column walk
// Rows per position-parallel rescale tile (<= kColTileRows): their loads are in
// flight together (16-row tiles took ~70 us a task on ResNet-50's 3x3 layers,
// 4-row tiles ~11 us: profiles/r03/cle_tl_*.log)
#ifndef DFQ_CLE_POS_ROWS   // compile-time A/B (scripts/cle_lib_ab.py builds side by side)
#define DFQ_CLE_POS_ROWS 4
#endif
constexpr int kPosTileMaxRows = DFQ_CLE_POS_ROWS;

__device__ __forceinline__ bool tile_by_position(const CleRel& R, const CleTask& tk) {
    return R.khw2 > 1 && R.khw2 <= kTileMaxKhw && (tk.a / R.o2g) == ((tk.b - 1) / R.o2g);
}

// Column ranges of the tile: per-position (min, max) over its rows, then over each
// column's khw positions through LDS (tl: 2 * kThreads * kTileMaxKhw floats).
__device__ void tile_range_by_position(const CleRel& R, const CleTask& tk, uint32_t* __restrict__ mn,
                                       uint32_t* __restrict__ mx, float* __restrict__ tl) {
    const int t = threadIdx.x;
    const int khw = (int)R.khw2;
    const int64_t rowlen = R.i2 * R.khw2;
    const int ncol = (int)(tk.c1 - tk.c0);
    const int npos = ncol * khw;
    const DFQ_GLOBAL float* base = (const DFQ_GLOBAL float*)(R.w2 + tk.c0 * R.khw2);
    float vmn[kTileMaxKhw], vmx[kTileMaxKhw];
#pragma unroll
    for (int m = 0; m < kTileMaxKhw; ++m) {
        vmn[m] = INFINITY;
        vmx[m] = -INFINITY;
    }
    for (int64_t o = tk.a; o < tk.b; ++o) {
        const DFQ_GLOBAL float* rp = base + o * rowlen;
        float v[kTileMaxKhw];
#pragma unroll
        for (int m = 0; m < kTileMaxKhw; ++m)
            if (m < khw && t + kThreads * m < npos) v[m] = rp[t + kThreads * m];
#pragma unroll
        for (int m = 0; m < kTileMaxKhw; ++m)
            if (m < khw && t + kThreads * m < npos) {
                vmn[m] = fminf(vmn[m], v[m]);
                vmx[m] = fmaxf(vmx[m], v[m]);
            }
    }
#pragma unroll
    for (int m = 0; m < kTileMaxKhw; ++m)
        if (m < khw && t + kThreads * m < npos) {
            tl[t + kThreads * m] = vmn[m];
            tl[kThreads * kTileMaxKhw + t + kThreads * m] = vmx[m];
        }
    __syncthreads();
    if (t < ncol) {
        float a = INFINITY, b = -INFINITY;
        for (int k = 0; k < khw; ++k) {
            a = fminf(a, tl[t * khw + k]);
            b = fmaxf(b, tl[kThreads * kTileMaxKhw + t * khw + k]);
        }
        const int64_t c = R.c1 + (tk.a / R.o2g) * R.i2 + tk.c0 + t;
        atomicMin(&mn[c], enc_ord(a));
        atomicMax(&mx[c], enc_ord(b));
    }
    __syncthreads();   // tl is reused by the next task
}

// Range tasks [t0, t1) for parity `par`, taken by blocks blk, blk + nblk, ...
// (tl: 2 * kThreads * kTileMaxKhw floats of LDS).
__device__ __forceinline__ void cle_range_body(const CleRel* __restrict__ rels, const CleTask* __restrict__ tasks,
                                               int64_t t0, int64_t t1, uint32_t* __restrict__ rng, int64_t M, int par,
                                               int64_t blk, int64_t nblk, float* tl) {
    uint32_t* mins = rng + (int64_t)par * 2 * M;
    uint32_t* maxs = mins + M;
    uint32_t* omins = rng + (int64_t)(par ^ 1) * 2 * M;
    uint32_t* omaxs = omins + M;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    for (int64_t t = t0 + blk; t < t1; t += nblk) {
        const CleTask tk = tasks[t];
        const CleRel& R = rels[tk.rel];
        uint32_t* mn = mins + R.moff;
        uint32_t* mx = maxs + R.moff;
        if (tk.kind == kRangeW1 && R.len1 < 64) {   // short rows: a lane group per row
            for_short_rows(tk.a, tk.b, R.len1, [&](int64_t c, bool act, int sl, int G) {
                float vmin = INFINITY, vmax = -INFINITY;
                if (act)
                    for (int64_t i = sl; i < R.len1; i += G) {
                        const float x = ((DFQ_GLOBAL float*)R.w1)[c * R.len1 + i];
                        vmin = fminf(vmin, x);
                        vmax = fmaxf(vmax, x);
                    }
                vmin = group_min(vmin, G);
                vmax = group_max(vmax, G);
                if (act && sl == 0) {
                    mn[c] = enc_ord(vmin);
                    mx[c] = enc_ord(vmax);
                }
            });
        } else if (tk.kind == kRangeW2Contig && R.o2g * R.khw2 < 64) {
            const int64_t seg = R.o2g * R.khw2;
            for_short_rows(tk.a, tk.b, seg, [&](int64_t c, bool act, int sl, int G) {
                float vmin = INFINITY, vmax = -INFINITY;
                if (act)
                    for (int64_t i = sl; i < seg; i += G) {
                        const float x = ((DFQ_GLOBAL float*)R.w2)[c * seg + i];
                        vmin = fminf(vmin, x);
                        vmax = fmaxf(vmax, x);
                    }
                vmin = group_min(vmin, G);
                vmax = group_max(vmax, G);
                if (act && sl == 0) {
                    mn[R.c1 + c] = enc_ord(vmin);
                    mx[R.c1 + c] = enc_ord(vmax);
                }
            });
        } else if (tk.kind == kRangeW1) {   // one wave per W1 row
            for (int64_t c = tk.a + wv; c < tk.b; c += kThreads / 64) {
                float vmin, vmax;
                wave_range(R.w1 + c * R.len1, R.len1, R.vec1, lane, vmin, vmax);
                if (lane == 0) {
                    mn[c] = enc_ord(vmin);
                    mx[c] = enc_ord(vmax);
                }
            }
        } else if (tk.kind == kRangeW2Contig) {   // one wave per contiguous W2 channel
            const int64_t seg = R.o2g * R.khw2;
            for (int64_t c = tk.a + wv; c < tk.b; c += kThreads / 64) {
                float vmin, vmax;
                wave_range(R.w2 + c * seg, seg, R.vec2, lane, vmin, vmax);
                if (lane == 0) {
                    mn[R.c1 + c] = enc_ord(vmin);
                    mx[R.c1 + c] = enc_ord(vmax);
                }
            }
        } else if (tk.kind == kRangeW2Tile) {   // rows [a, b) of W2, one thread per column
            if (tile_by_position(R, tk)) {
                tile_range_by_position(R, tk, mn, mx, tl);
                continue;
            }
            const int64_t rowlen = R.i2 * R.khw2;
            const bool one_group = (tk.a / R.o2g) == ((tk.b - 1) / R.o2g);
            for (int64_t i = tk.c0 + threadIdx.x; i < tk.c1; i += kThreads) {
                float vmin = INFINITY, vmax = -INFINITY;
                if (one_group && R.khw2 == 1) {   // 1x1 / Linear: the tile's column, 16 loads in flight
                    float v[kColTileRows];
#pragma unroll
                    for (int j = 0; j < kColTileRows; ++j)
                        if (tk.a + j < tk.b) v[j] = ((DFQ_GLOBAL float*)R.w2)[(tk.a + j) * rowlen + i];
#pragma unroll
                    for (int j = 0; j < kColTileRows; ++j)
                        if (tk.a + j < tk.b) {
                            vmin = fminf(vmin, v[j]);
                            vmax = fmaxf(vmax, v[j]);
                        }
                    const int64_t c = R.c1 + (tk.a / R.o2g) * R.i2 + i;
                    atomicMin(&mn[c], enc_ord(vmin));
                    atomicMax(&mx[c], enc_ord(vmax));
                    continue;
                }
                int64_t g_prev = -1;
                for (int64_t o = tk.a; o < tk.b; ++o) {
                    const int64_t g = o / R.o2g;
                    if (g != g_prev && g_prev >= 0) {   // tile straddles groups: flush
                        atomicMin(&mn[R.c1 + g_prev * R.i2 + i], enc_ord(vmin));
                        atomicMax(&mx[R.c1 + g_prev * R.i2 + i], enc_ord(vmax));
                        vmin = INFINITY;
                        vmax = -INFINITY;
                    }
                    g_prev = g;
                    const DFQ_GLOBAL float* p = (const DFQ_GLOBAL float*)(R.w2 + o * rowlen + i * R.khw2);
                    for (int64_t k = 0; k < R.khw2; ++k) {
                        vmin = fminf(vmin, p[k]);
                        vmax = fmaxf(vmax, p[k]);
                    }
                }
                if (g_prev >= 0) {
                    atomicMin(&mn[R.c1 + g_prev * R.i2 + i], enc_ord(vmin));
                    atomicMax(&mx[R.c1 + g_prev * R.i2 + i], enc_ord(vmax));
                }
            }
        } else {   // kRangeReset(W1): the other parity's W2 (W1) words, for the next iteration's atomics
            const int64_t off = R.moff + (tk.kind == kRangeReset ? R.c1 : 0);
            for (int64_t c = tk.a + threadIdx.x; c < tk.b; c += kThreads) {
                omins[off + c] = 0xFFFFFFFFu;
                omaxs[off + c] = 0u;
            }
        }
    }
}

// `next` = 1: the ranges of the NEXT iteration (launched after this iteration's
// last rescale, fused into the metric-tile launch; see cle_loop_step_kernel)
__global__ void __launch_bounds__(kThreads)
cle_loop_range_kernel(const CleRel* __restrict__ rels, const CleTask* __restrict__ tasks, int64_t t0, int64_t t1,
                      uint32_t* __restrict__ rng, int64_t M, const CleState* __restrict__ st, int next) {
    __shared__ float tl[2 * kThreads * kTileMaxKhw];
    if (st->done) return;
    cle_range_body(rels, tasks, t0, t1, rng, M, (st->iters + next) & 1, blockIdx.x, gridDim.x, tl);
}

// The scale of relation R for channel c (mins / maxs: the parity's range words).
// A relation whose W1 is the depthwise W2 of relation Q (R.dw_prev) has no W1
// range words: its W1 row c is Q's filter c after Q's rescale, fl(x * inv_Q[c]),
// and with inv_Q > 0 that product is monotonic in x, so the row's min / max are
// fl(min_c * inv_Q) / fl(max_c * inv_Q) -- Q's W2 range words (the filter at the
// start of the iteration) scaled.  Every task of R can therefore compute its scale
// in the same launch that rescales Q (kApplyDwBoth writes the filter once).
__device__ __forceinline__ CleScale cle_rel_scale(const CleRel* __restrict__ rels, const CleRel& R,
                                                  const uint32_t* __restrict__ mins, const uint32_t* __restrict__ maxs,
                                                  int64_t c, int is_signed, float eps, double smin, double smax) {
    if (R.dw_prev < 0) return cle_scale(mins + R.moff, maxs + R.moff, R.c1, c, is_signed, eps, smin, smax);
    const CleRel& Q = rels[R.dw_prev];
    const CleScale q = cle_scale(mins + Q.moff, maxs + Q.moff, Q.c1, c, is_signed, eps, smin, smax);
    const float mn1 = dec_ord(mins[Q.moff + Q.c1 + c]) * q.inv;
    const float mx1 = dec_ord(maxs[Q.moff + Q.c1 + c]) * q.inv;
    return cle_scale_from(mn1, mx1, dec_ord(mins[R.moff + R.c1 + c]), dec_ord(maxs[R.moff + R.c1 + c]), is_signed, eps,
                          smin, smax);
}

// LDS of one rescale task (the position-parallel and fused tiles)
struct CleApplyLds {
    float red[2][kThreads / 64][kColTileRows];
    float inv_s[kThreads];
    float inv_pos[kThreads * kTileMaxKhw];
    float rows[kColTileRows * kThreads];   // a 1x1 W2 tile's rescaled values, for its per-row ranges
};

// Rescale tasks [t0, t1) of iteration parity `par`, taken by blocks blk, blk + nblk, ...
#ifdef DFQ_DIAGNOSTICS
// DFQ_CLE_TL (diagnostics): per rescale task of one steady-state iteration,
// {start, end} in s_memrealtime ticks (100 MHz) and the block's XCC / CU ids.
__device__ uint64_t* g_cle_tl = nullptr;
// ... and per block of the iteration's last launch (tiles / ranges / stop rule):
// {start, end, role (1 tile, 2 range), 0}; slot kCleTl2Fin: the stop rule's {start,
// end, chunk sums staged, layer means done}
__device__ uint64_t* g_cle_tl2 = nullptr;
// DFQ_CLE_TL_STEP=k: record the blocks of step k's launches instead (the launch whose
// rescale tasks start at table index g_cle_tl2_a0; -1: every launch, the last wins)
__device__ int64_t g_cle_tl2_a0 = -1;
constexpr int kCleTl2Fin = 8192;
#endif

// POS: the step has position-parallel (KH*KW > 1) W2 tiles; without them the
// body needs far fewer VGPRs (more waves per SIMD for the latency-bound tasks)
template <bool POS = true>
__device__ __forceinline__ void cle_apply_body(const CleRel* __restrict__ rels, const CleTask* __restrict__ tasks,
                                               int64_t t0, int64_t t1, uint32_t* __restrict__ rng, int64_t M,
                                               int par, bool first_iter, int is_signed, float eps, double smin,
                                               double smax, int64_t blk, int64_t nblk, CleApplyLds& A,
                                               float* __restrict__ vsave = nullptr, int32_t* __restrict__ vtag = nullptr,
                                               int32_t iter = 0) {
    auto& red = A.red;
    float* rows = A.rows;
    float* inv_s = A.inv_s;
    float* inv_pos = A.inv_pos;
    uint32_t* mins = rng + (int64_t)par * 2 * M;
    uint32_t* maxs = mins + M;
    uint32_t* nmins = rng + (int64_t)(par ^ 1) * 2 * M;   // the next iteration's words (self ranges)
    uint32_t* nmaxs = nmins + M;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    for (int64_t t = t0 + blk; t < t1; t += nblk) {
#ifdef DFQ_DIAGNOSTICS
        const bool tl_on = g_cle_tl != nullptr;   // block-uniform
        const uint64_t tl_start = tl_on ? __builtin_amdgcn_s_memrealtime() : 0;
        uint64_t tl_sub = 0;   // position tiles: phase ends (10 ns ticks after start, 16 bits each)
#define DFQ_CLE_TL_MARK(k) \
        if (tl_on) tl_sub |= (1ull << 63) | (((__builtin_amdgcn_s_memrealtime() - tl_start) & 0xffffull) << (16 * (k)));
#else
#define DFQ_CLE_TL_MARK(k)
#endif
        const CleTask tk = tasks[t];
        const CleRel& R = rels[tk.rel];
        const uint32_t* mn = mins + R.moff;
        const uint32_t* mx = maxs + R.moff;
        if (tk.kind == kApplyW1 && R.len1 < 64) {   // short rows: a lane group per row
            for_short_rows(tk.a, tk.b, R.len1, [&](int64_t c, bool act, int sl, int G) {
                float y0 = INFINITY, y1 = -INFINITY;
                if (act && sl < R.len1) {   // G >= len1: one element per lane
                    DFQ_GLOBAL float* p = (DFQ_GLOBAL float*)(R.w1 + c * R.len1 + sl);
                    const float x = *p;   // in flight while the scale's range words load
                    const float y = x * cle_rel_scale(rels, R, mins, maxs, c, is_signed, eps, smin, smax).s;
                    *p = y;
                    y0 = y1 = y;
                }
                if (R.w1_self) {   // the row is final for this iteration: its next range
                    y0 = group_min(y0, G);
                    y1 = group_max(y1, G);
                    if (act && sl == 0) {
                        nmins[R.moff + c] = enc_ord(y0);
                        nmaxs[R.moff + c] = enc_ord(y1);
                    }
                }
            });
        } else if (tk.kind == kApplyDwBoth && R.o2g * R.khw2 < 64) {
            const CleRel& N = rels[tk.c0];
            const int64_t seg = R.o2g * R.khw2;
            for_short_rows(tk.a, tk.b, seg, [&](int64_t c, bool act, int sl, int G) {
                float z0 = INFINITY, z1 = -INFINITY;
                if (act && sl < seg) {   // G >= seg: one element per lane
                    DFQ_GLOBAL float* p = (DFQ_GLOBAL float*)(R.w2 + c * seg + sl);
                    const float x = *p;
                    const float inv = cle_rel_scale(rels, R, mins, maxs, c, is_signed, eps, smin, smax).inv;
                    const float sn = cle_rel_scale(rels, N, mins, maxs, c, is_signed, eps, smin, smax).s;
                    const float y = x * inv;
                    const float z = y * sn;
                    *p = z;
                    z0 = z1 = z;
                }
                if (R.w2_self) {   // the filter is final for this iteration: its next range
                    z0 = group_min(z0, G);
                    z1 = group_max(z1, G);
                    if (act && sl == 0) {
                        nmins[R.moff + R.c1 + c] = enc_ord(z0);
                        nmaxs[R.moff + R.c1 + c] = enc_ord(z1);
                    }
                }
            });
        } else if (tk.kind == kApplyW2Contig && R.o2g * R.khw2 < 64) {
            const int64_t seg = R.o2g * R.khw2;
            const bool fuse = R.fuse_next >= 0;
            for_short_rows(tk.a, tk.b, seg, [&](int64_t c, bool act, int sl, int G) {
                float vmin = INFINITY, vmax = -INFINITY;
                if (act && sl < seg) {   // G >= seg: one element per lane
                    DFQ_GLOBAL float* p = (DFQ_GLOBAL float*)(R.w2 + c * seg + sl);
                    const float x = *p;
                    const float y = x * cle_rel_scale(rels, R, mins, maxs, c, is_signed, eps, smin, smax).inv;
                    *p = y;
                    vmin = vmax = y;
                }
                if (fuse) {   // o2g == 1: the segment is row c of the next relation's W1
                    vmin = group_min(vmin, G);
                    vmax = group_max(vmax, G);
                    if (act && sl == 0) {
                        const int64_t off = rels[R.fuse_next].moff;
                        mins[off + c] = enc_ord(vmin);
                        maxs[off + c] = enc_ord(vmax);
                    }
                }
            });
        } else if (tk.kind == kApplyW1) {   // W1[c, :] *= s[c], one wave per row
            for (int64_t c = tk.a + wv; c < tk.b; c += kThreads / 64) {
                auto sc = [&] { return cle_rel_scale(rels, R, mins, maxs, c, is_signed, eps, smin, smax).s; };
                if (R.w1_self) {   // the row is final for this iteration: its next range
                    float y0, y1;
                    wave_scale_mm(R.w1 + c * R.len1, R.len1, R.vec1, lane, y0, y1, sc);
                    if (lane == 0) {
                        nmins[R.moff + c] = enc_ord(y0);
                        nmaxs[R.moff + c] = enc_ord(y1);
                    }
                } else {
                    wave_scale(R.w1 + c * R.len1, R.len1, R.vec1, lane, sc);
                }
            }
        } else if (tk.kind == kApplyDwBoth) {
            // relation R's depthwise W2 filter c, which is relation tk.c0's W1 row c:
            // *= 1/s_R[c], then *= s_next[c] (two roundings, as the reference's two
            // in-place multiplies), written once
            const CleRel& N = rels[tk.c0];
            const int64_t seg = R.o2g * R.khw2;
            for (int64_t c = tk.a + wv; c < tk.b; c += kThreads / 64) {
                const float inv = cle_rel_scale(rels, R, mins, maxs, c, is_signed, eps, smin, smax).inv;
                const float sn = cle_rel_scale(rels, N, mins, maxs, c, is_signed, eps, smin, smax).s;
                DFQ_GLOBAL float* p = (DFQ_GLOBAL float*)(R.w2 + c * seg);
                float z0 = INFINITY, z1 = -INFINITY;
                for (int64_t i = lane; i < seg; i += 64) {
                    const float y = p[i] * inv;
                    const float z = y * sn;
                    p[i] = z;
                    z0 = fminf(z0, z);
                    z1 = fmaxf(z1, z);
                }
                if (R.w2_self) {
                    cle_wave_minmax(z0, z1);
                    if (lane == 0) {
                        nmins[R.moff + R.c1 + c] = enc_ord(z0);
                        nmaxs[R.moff + R.c1 + c] = enc_ord(z1);
                    }
                }
            }
        } else if (tk.kind == kApplyW2Contig) {   // W2 channel segment *= 1/s[c]
            const int64_t seg = R.o2g * R.khw2;
            for (int64_t c = tk.a + wv; c < tk.b; c += kThreads / 64) {
                auto inv = [&] { return cle_rel_scale(rels, R, mins, maxs, c, is_signed, eps, smin, smax).inv; };
                if (R.fuse_next >= 0) {   // o2g == 1: the segment is row c of W2 = row c of the next W1
                    float vmin, vmax;
                    wave_scale_range(R.w2 + c * seg, seg, lane, vmin, vmax, inv);
                    if (lane == 0) {
                        const int64_t off = rels[R.fuse_next].moff;
                        mins[off + c] = enc_ord(vmin);
                        maxs[off + c] = enc_ord(vmax);
                    }
                } else {
                    wave_scale(R.w2 + c * seg, seg, R.vec2, lane, inv);
                }
            }
        } else if (POS && tk.kind == kApplyW2Tile && tile_by_position(R, tk) && tk.b - tk.a <= kPosTileMaxRows) {
            // position-parallel tile (KH*KW > 1): the columns' 1/s into LDS, then each
            // row's positions scaled; fused: the rows' (min, max) for the next W1
            const int t = threadIdx.x;
            const int khw = (int)R.khw2;
            const int64_t rowlen = R.i2 * R.khw2;
            const int ncol = (int)(tk.c1 - tk.c0);
            const int npos = ncol * khw;
            DFQ_GLOBAL float* base = (DFQ_GLOBAL float*)(R.w2 + tk.c0 * R.khw2);
            const bool fuse = R.fuse_next >= 0;
            if (t < ncol)
                inv_s[t] = cle_rel_scale(rels, R, mins, maxs, (tk.a / R.o2g) * R.i2 + tk.c0 + t, is_signed, eps, smin, smax).inv;
            __syncthreads();
            DFQ_CLE_TL_MARK(0)
            for (int q = t; q < npos; q += kThreads) inv_pos[q] = inv_s[q / khw];   // 1/s per position
            __syncthreads();
            DFQ_CLE_TL_MARK(1)
            // Every row's loads in flight together, then the rows' scaled stores:
            // one memory round trip per tile instead of one per row (~5 us a row
            // under the step's load, ResNet-50's 3x3 tiles; DFQ_CLE_TL)
            // (row bases uniform, the lane's offset a 32-bit index: SGPR-base loads
            // sharing one VGPR offset, not 36 64-bit VGPR addresses)
            float v[kPosTileMaxRows][kTileMaxKhw];
#pragma unroll
            for (int r = 0; r < kPosTileMaxRows; ++r) {
                const DFQ_GLOBAL float* rb = base + (tk.a + r) * rowlen;
#pragma unroll
                for (int m = 0; m < kTileMaxKhw; ++m)
                    if (tk.a + r < tk.b && m < khw && t + kThreads * m < npos) v[r][m] = rb[t + kThreads * m];
            }
#pragma unroll
            for (int r = 0; r < kPosTileMaxRows; ++r) {
                if (tk.a + r >= tk.b) break;   // uniform
                DFQ_GLOBAL float* rp = base + (tk.a + r) * rowlen;
                float lo = INFINITY, hi = -INFINITY;
#pragma unroll
                for (int m = 0; m < kTileMaxKhw; ++m)
                    if (m < khw && t + kThreads * m < npos) {
                        const float y = v[r][m] * inv_pos[t + kThreads * m];
                        rp[t + kThreads * m] = y;
                        lo = fminf(lo, y);
                        hi = fmaxf(hi, y);
                    }
                if (fuse) {
                    cle_wave_minmax(lo, hi);
                    if (lane == 0) {
                        red[0][wv][r] = lo;
                        red[1][wv][r] = hi;
                    }
                }
            }
            __syncthreads();
            DFQ_CLE_TL_MARK(2)
            if (fuse && t < tk.b - tk.a) {
                float a = red[0][0][t], b = red[1][0][t];
                for (int w = 1; w < kThreads / 64; ++w) {
                    a = fminf(a, red[0][w][t]);
                    b = fmaxf(b, red[1][w][t]);
                }
                const int64_t off = rels[R.fuse_next].moff + tk.a + t;
                atomicMin(&mins[off], enc_ord(a));
                atomicMax(&maxs[off], enc_ord(b));
            }
            __syncthreads();   // inv_s / red are reused by the next task
        } else if (tk.kind == kApplyW2Tile && R.fuse_next >= 0) {
            // rows [a, b) x columns [c0, c0 + 256) of W2, one thread per column, and the
            // tile's per-row (min, max) of the results -> the next relation's W1 rows
            // (each row's wave reduction in uniform control flow: no per-row arrays)
            const int64_t rowlen = R.i2 * R.khw2;
            const int64_t i = tk.c0 + threadIdx.x;
            const bool act = i < tk.c1;
            const bool one_group = (tk.a / R.o2g) == ((tk.b - 1) / R.o2g);
            const int nr = (int)(tk.b - tk.a);
            if (one_group && R.khw2 == 1) {   // 1x1 / Linear: the column's loads first
                // The tile's values go to LDS as rows[j][column]; after one barrier,
                // lane t reduces 16 columns of row t / 16 and the 16 lanes of a DPP
                // row combine them (4 steps): per task 16 short reductions on 256
                // lanes instead of 16 dependent 64-lane wave reductions (3.3 of
                // these tasks' 7.4 us, DFQ_CLE_TL).  fminf / fmaxf skip the NaN that
                // marks a column past the tile.
                float v[kColTileRows];
#pragma unroll
                for (int j = 0; j < kColTileRows; ++j)
                    if (act && j < nr) v[j] = ((DFQ_GLOBAL float*)R.w2)[(tk.a + j) * rowlen + i];
                const float inv =
                    act ? cle_rel_scale(rels, R, mins, maxs, (tk.a / R.o2g) * R.i2 + i, is_signed, eps, smin, smax).inv : 0.f;
#pragma unroll
                for (int j = 0; j < kColTileRows; ++j) {
                    if (j < nr) {   // uniform
                        float y = __builtin_nanf("");
                        if (act) {
                            y = v[j] * inv;
                            ((DFQ_GLOBAL float*)R.w2)[(tk.a + j) * rowlen + i] = y;
                        }
                        rows[j * kThreads + threadIdx.x] = y;
                    }
                    if (j == 0) {   // the column's loads and its scale have landed
                        DFQ_CLE_TL_MARK(0)
                    }
                }
                DFQ_CLE_TL_MARK(1)   // every row stored
                block_lds_sync();
                const int r = threadIdx.x >> 4, sg = threadIdx.x & 15;
                float lo = INFINITY, hi = -INFINITY;
                if (r < nr) {
                    const float4* q = reinterpret_cast<const float4*>(rows + r * kThreads + sg * 16);
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const float4 x = q[u];
                        lo = fminf(lo, fminf(fminf(x.x, x.y), fminf(x.z, x.w)));
                        hi = fmaxf(hi, fmaxf(fmaxf(x.x, x.y), fmaxf(x.z, x.w)));
                    }
                }
                lo = fminf(lo, dpp_f(lo, 0xB1));
                hi = fmaxf(hi, dpp_f(hi, 0xB1));
                lo = fminf(lo, dpp_f(lo, 0x4E));
                hi = fmaxf(hi, dpp_f(hi, 0x4E));
                lo = fminf(lo, dpp_f(lo, 0x141));
                hi = fmaxf(hi, dpp_f(hi, 0x141));
                lo = fminf(lo, dpp_f(lo, 0x140));
                hi = fmaxf(hi, dpp_f(hi, 0x140));
                DFQ_CLE_TL_MARK(2)
                if (sg == 0 && r < nr) {
                    const int64_t off = rels[R.fuse_next].moff + tk.a + r;
                    atomicMin(&mins[off], enc_ord(lo));
                    atomicMax(&maxs[off], enc_ord(hi));
                }
            } else {
                int64_t g_prev = -1;
                float inv = 0.f;
                for (int j = 0; j < nr; ++j) {
                    const int64_t o = tk.a + j;
                    float lo = INFINITY, hi = -INFINITY;
                    if (act) {
                        const int64_t g = o / R.o2g;
                        if (g != g_prev) {
                            inv = cle_rel_scale(rels, R, mins, maxs, g * R.i2 + i, is_signed, eps, smin, smax).inv;
                            g_prev = g;
                        }
                        DFQ_GLOBAL float* p = (DFQ_GLOBAL float*)(R.w2 + o * rowlen + i * R.khw2);
                        for (int64_t k = 0; k < R.khw2; ++k) {
                            const float y = p[k] * inv;
                            p[k] = y;
                            lo = fminf(lo, y);
                            hi = fmaxf(hi, y);
                        }
                    }
                    float a = lo, b = hi;
                    cle_wave_minmax(a, b);
                    if (lane == 0) {
                        red[0][wv][j] = a;
                        red[1][wv][j] = b;
                    }
                }
                __syncthreads();
                if (threadIdx.x < tk.b - tk.a) {
                    const int j = threadIdx.x;
                    float a = red[0][0][j], b = red[1][0][j];
                    for (int w = 1; w < kThreads / 64; ++w) {
                        a = fminf(a, red[0][w][j]);
                        b = fmaxf(b, red[1][w][j]);
                    }
                    const int64_t off = rels[R.fuse_next].moff + tk.a + j;
                    atomicMin(&mins[off], enc_ord(a));
                    atomicMax(&maxs[off], enc_ord(b));
                }
            }
            __syncthreads();   // red / rows are reused by the next task
        } else if (tk.kind == kApplyW2Tile) {   // rows [a, b) of W2, one thread per column
            const int64_t rowlen = R.i2 * R.khw2;
            const bool one_group = (tk.a / R.o2g) == ((tk.b - 1) / R.o2g);
            for (int64_t i = tk.c0 + threadIdx.x; i < tk.c1; i += kThreads) {
                if (one_group && R.khw2 == 1) {   // 1x1 / Linear: the tile's column, loads first
                    float v[kColTileRows];
#pragma unroll
                    for (int j = 0; j < kColTileRows; ++j)
                        if (tk.a + j < tk.b) v[j] = ((DFQ_GLOBAL float*)R.w2)[(tk.a + j) * rowlen + i];
                    const float inv = cle_rel_scale(rels, R, mins, maxs, (tk.a / R.o2g) * R.i2 + i, is_signed, eps, smin,
                                                smax).inv;
                    ((DFQ_GLOBAL float*)R.w2)[tk.a * rowlen + i] = v[0] * inv;
                    DFQ_CLE_TL_MARK(0)   // the column's loads and its scale have landed
#pragma unroll
                    for (int j = 1; j < kColTileRows; ++j)
                        if (tk.a + j < tk.b) ((DFQ_GLOBAL float*)R.w2)[(tk.a + j) * rowlen + i] = v[j] * inv;
                    DFQ_CLE_TL_MARK(1)
                    continue;
                }
                int64_t g_prev = -1;
                float inv = 0.f;
                for (int64_t o = tk.a; o < tk.b; ++o) {
                    const int64_t g = o / R.o2g;
                    if (g != g_prev) {
                        inv = cle_rel_scale(rels, R, mins, maxs, g * R.i2 + i, is_signed, eps, smin, smax).inv;
                        g_prev = g;
                    }
                    DFQ_GLOBAL float* p = (DFQ_GLOBAL float*)(R.w2 + o * rowlen + i * R.khw2);
                    for (int64_t k = 0; k < R.khw2; ++k) p[k] = p[k] * inv;
                }
            }
        } else {
            // lagged schedule: the per-channel vectors before this iteration's
            // multiply, and the iteration that saved them (per task), for the
            // rollback of a speculative iteration (cle_loop_rollback_kernel)
            if (vtag && threadIdx.x == 0) vtag[t] = iter;
            for (int64_t c = tk.a + threadIdx.x; c < tk.b; c += kThreads) {
                const CleScale cs = cle_rel_scale(rels, R, mins, maxs, c, is_signed, eps, smin, smax);
                if (vsave) {
                    float* v = vsave + 2 * R.moff;   // [b1 | bnw | bnb | sacc] x c1
                    if (R.b1) v[c] = R.b1[c];
                    if (R.bnw) v[R.c1 + c] = R.bnw[c];
                    if (R.bnb) v[2 * R.c1 + c] = R.bnb[c];
                    if (R.sacc) v[3 * R.c1 + c] = R.sacc[c];
                }
                if (R.b1) R.b1[c] = R.b1[c] * cs.s;
                if (R.bnw) R.bnw[c] = R.bnw[c] * cs.s;
                if (R.bnb) R.bnb[c] = R.bnb[c] * cs.s;
                if (R.sacc) R.sacc[c] = (R.sacc_init && first_iter) ? cs.s : R.sacc[c] * cs.s;
            }
        }
#ifdef DFQ_DIAGNOSTICS
        if (tl_on) {   // the last executed iteration's times remain
            __syncthreads();   // the block's task is done (timing only)
            if (threadIdx.x == 0) {
                uint32_t hw, xcc;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                uint64_t* r = g_cle_tl + 4 * t;
                r[0] = tl_start;
                r[1] = __builtin_amdgcn_s_memrealtime();
                r[2] = tl_sub ? tl_sub : (((uint64_t)xcc << 32) | hw);
                r[3] = (uint64_t)tk.kind | ((uint64_t)tk.rel << 8) | ((uint64_t)(tk.b - tk.a) << 24);
            }
        }
#endif
    }
}

// The metric's fp32 sums (torch.mean's vectorized_inner_sum over one chunk) as a
// fixed tree.  A chunk of len elements is 32 streams (s = 8k + l: 8 vector lanes x
// ILP 4; stream element i is chunk element 32i + s) of sz = len/32 elements, each
// a 4-level cascade with 16-element level-0 blocks (step 2^4 for every chunk below
// 16M elements).  One level-1 group of all 32 streams is 8192 CONTIGUOUS elements:
//   * cle_tiles_body: one workgroup per 8192-element tile: |W - snap| (snap := W
//     on the way), 512 threads-worth of level-0 block sums, then 32 level-1 sums
//     -> b1buf; the chunk's remainder (partial group, level-0 tail, row_sum tail
//     vectors, scalar tail) is one more "tail tile";
//   * cle_chunk_sum_with: one wave per chunk finishes the cascade in ATen's order
//     (level 2/3, a0 += a1 += a2 += a3, ILP, lanes, scalar tail).
constexpr int kCleTile = 8192;            // 32 streams x 16 x 16
constexpr int kCleTailWords = 64;         // per chunk: 32 stream partials, 24 row-tail, 8 scalar-tail values

struct CleUnit {
    int32_t chunk;
    int32_t tile;     // < nb1: full level-1 tile; == nb1: the chunk's tail tile
};

// Before the first iteration, ONE launch instead of six fills, a state upload and
// the snapshot kernel: both parities' range words armed (mins = 0xFF.., maxs = 0;
// layout [parity][mins M | maxs M]), the chunk sums and arrival counters zeroed,
// the rollback tags set to -1, the loop state from the launch argument, and
// snap := W (one workgroup per metric tile; the chunks of < 8 elements by block 0).
__global__ void __launch_bounds__(kThreads)
cle_loop_init_kernel(const CleLayer* __restrict__ layers, const CleChunk* __restrict__ chunks, int64_t nchunks,
                     const CleUnit* __restrict__ units, int64_t nunits, uint32_t* __restrict__ rng, int64_t M,
                     float* __restrict__ part, int64_t npart, uint32_t* __restrict__ cnt, int64_t ncnt,
                     int32_t* __restrict__ vtag, int64_t nvtag, CleState* __restrict__ st, CleState init) {
    const int64_t gt = (int64_t)blockIdx.x * kThreads + threadIdx.x, gs = (int64_t)gridDim.x * kThreads;
    for (int64_t i = gt; i < 4 * M; i += gs) rng[i] = ((i / M) & 1) ? 0u : 0xFFFFFFFFu;
    for (int64_t i = gt; i < npart; i += gs) part[i] = 0.f;
    for (int64_t i = gt; i < ncnt; i += gs) cnt[i] = 0u;
    for (int64_t i = gt; i < nvtag; i += gs) vtag[i] = -1;
    if (gt == 0) *st = init;
    for (int64_t u = blockIdx.x; u < nunits; u += gridDim.x) {
        const CleUnit un = units[u];
        const CleChunk ch = chunks[un.chunk];
        const CleLayer Ly = layers[ch.layer];
        const int64_t nb1 = (ch.len / 32) / 256;
        const int64_t e0 = (int64_t)un.tile * 8192;
        const int64_t e1 = un.tile < nb1 ? e0 + 8192 : ch.len;
        for (int64_t i = e0 + threadIdx.x; i < e1; i += kThreads) Ly.snap[ch.c0 + i] = Ly.w[ch.c0 + i];
    }
    if (blockIdx.x == 0)
        for (int64_t k = 0; k < nchunks; ++k) {
            const CleChunk ch = chunks[k];
            if (ch.len >= 8) continue;
            const CleLayer Ly = layers[ch.layer];
            for (int64_t i = threadIdx.x; i < ch.len; i += kThreads) Ly.snap[ch.c0 + i] = Ly.w[ch.c0 + i];
        }
}


// Metric tiles taken by blocks blk, blk + nblk, ... (d: kCleTile + kCleTailWords
// floats of LDS, b0: 512).
struct CleNoUnitHook {
    __device__ void operator()(const CleUnit&, const CleChunk&, int64_t) const {}
};

// hook(unit, chunk, nb1) runs after each unit (LDS free again).  (Tried on the
// snapshot stores: issued after the unit's arrival -- out of the arrival's
// vmcnt(0) drain -- no faster, tiles slower, 84 B of spills (cle_ab_r04p);
// non-temporal, the same (cle_ab_r04z).)
template <class Hook = CleNoUnitHook>
__device__ __forceinline__ void cle_tiles_body(const CleLayer* __restrict__ layers, const CleChunk* __restrict__ chunks,
                                               const int64_t* __restrict__ b1off, const CleUnit* __restrict__ units,
                                               int64_t nunits, float* __restrict__ b1buf, float* __restrict__ tailbuf,
                                               int64_t blk, int64_t nblk, float* d, float* b0, Hook hook = Hook()) {
    const int tid = threadIdx.x;
    for (int64_t u = blk; u < nunits; u += nblk) {
        const CleUnit un = units[u];
        const CleChunk ch = chunks[un.chunk];
        const CleLayer Ly = layers[ch.layer];
        const DFQ_GLOBAL float* __restrict__ w = (const DFQ_GLOBAL float*)(Ly.w + ch.c0);
        DFQ_GLOBAL float* __restrict__ sn = (DFQ_GLOBAL float*)(Ly.snap + ch.c0);
        const int64_t len = ch.len, sz = len / 32, vs = len / 8;
        const int64_t nb1 = sz / 256;
        const bool full = un.tile < nb1;
        const int64_t e0 = (int64_t)un.tile * kCleTile;
        const int64_t cnt = full ? kCleTile : len - e0;
        if (full) {
            // level 0 straight from the loads: thread t owns (block m, stream s) for
            // q = t and t + 256; its 16 elements 32 (16 m + j) + s sit at stride 32,
            // so each load instruction covers whole 128-B lines across the lanes,
            // and the 16-term sum runs in ATen's order in registers (32 loads in
            // flight per thread, no LDS staging of |W - W_prev|)
            float xs[2][16], ys[2][16];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int q = tid + h * kThreads;
                const int64_t base = e0 + 32 * (16 * (q >> 5)) + (q & 31);
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    xs[h][j] = w[base + 32 * j];
                    ys[h][j] = sn[base + 32 * j];
                }
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int q = tid + h * kThreads;
                const int64_t base = e0 + 32 * (16 * (q >> 5)) + (q & 31);
                float a = 0.f;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    a += fabsf(xs[h][j] - ys[h][j]);
                    sn[base + 32 * j] = xs[h][j];
                }
                b0[q] = a;   // b0[m * 32 + s]
            }
            __syncthreads();
            if (tid < 32) {   // level 1
                float a = 0.f;
#pragma unroll
                for (int m = 0; m < 16; ++m) a += b0[m * 32 + tid];
                st_coh(b1buf + b1off[un.chunk] + (int64_t)un.tile * 32 + tid, a);
            }
        } else {
            for (int64_t e = tid; e < cnt; e += 8 * kThreads) {   // |W - W_prev|, snap := W; 8 loads in flight
                float x[8], y[8];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (e + u * kThreads < cnt) {
                        x[u] = w[e0 + e + u * kThreads];
                        y[u] = sn[e0 + e + u * kThreads];
                    }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (e + u * kThreads < cnt) {
                        d[e + u * kThreads] = fabsf(x[u] - y[u]);
                        sn[e0 + e + u * kThreads] = x[u];
                    }
            }
            __syncthreads();
            const int64_t ni = sz - nb1 * 256;   // stream elements left: rem_b0 blocks + tail0
            const int64_t rem_b0 = ni / 16, tail0 = ni % 16;
            float* tb = tailbuf + (int64_t)un.chunk * kCleTailWords;
            if (tid < 32) {
                float a1p = 0.f;
                for (int64_t m = 0; m < rem_b0; ++m) {
                    float a = 0.f;
                    for (int j = 0; j < 16; ++j) a += d[32 * (16 * m + j) + tid];
                    a1p += a;
                }
                float a0t = 0.f;
                for (int64_t j = 0; j < tail0; ++j) a0t += d[32 * (16 * rem_b0 + j) + tid];
                float p = a0t;   // a0 += a1 (a2 and a3 follow in the combine)
                p += a1p;
                st_coh(tb + tid, p);
            } else if (tid < 64) {   // raw row_sum-tail vectors (v in [4sz, vs)) and scalar tail
                const int t = tid - 32;
                const int64_t nv = vs - 4 * sz;
                if (t < 24 && t < nv * 8) st_coh(tb + 32 + t, d[8 * (4 * sz) + t - e0]);
                if (t < 8 && t < len - 8 * vs) st_coh(tb + 56 + t, d[8 * vs + t - e0]);
            }
        }
        __syncthreads();   // LDS reused by the next unit
        hook(un, ch, nb1);
    }
}

constexpr int kCleTilesLds = kCleTile + kCleTailWords + 512;
constexpr int kCleRangeLds = 2 * kThreads * kTileMaxKhw;

// One chunk's sum from its tiles' level-1 sums and tail words (one wave; the
// result on every lane): the rest of the cascade, the ILP and lane combines and
// the scalar tail, in ATen's order.  Coherent loads: other blocks wrote b1 / tb.
template <class LdB1, class LdTb>
__device__ __forceinline__ float cle_chunk_sum_with(const CleChunk& ch, LdB1&& b1, LdTb&& tb, int lane) {
    const int64_t len = ch.len;
    const int64_t sz = len / 32, vs = len / 8;
    const int64_t nb1 = sz / 256, nb2 = nb1 / 16, rem_b1 = nb1 % 16;
    float fa = 0.f;
    float p = 0.f;
    if (lane < 32) {
        float a3 = 0.f;
        for (int64_t r = 0; r < nb2; ++r) {
            float b2 = 0.f;
            for (int q = 0; q < 16; ++q) b2 += b1((r * 16 + q) * 32 + lane);
            a3 += b2;
        }
        float a2p = 0.f;
        for (int64_t q = 0; q < rem_b1; ++q) a2p += b1((nb2 * 16 + q) * 32 + lane);
        p = tb(lane);   // a0 + a1
        p += a2p;
        p += a3;
    }
    // the combine on every lane, the 32 stream partials read by readlane (uniform
    // values: no 32-register array, no LDS permute per partial)
    auto ps = [&](int s) { return rl_f(p, s); };
    for (int64_t e = 0; e < len - 8 * vs; ++e) fa += tb(56 + e);   // scalar tail first
    const int64_t nv = vs - 4 * sz;
    for (int l = 0; l < 8; ++l) {
        float p0 = ps(l);
        for (int64_t v = 0; v < nv; ++v) p0 += tb(32 + v * 8 + l);   // row_sum tail into p0
        p0 += ps(l + 8);
        p0 += ps(l + 16);
        p0 += ps(l + 24);
        fa += p0;
    }
    return fa;
}

__device__ __forceinline__ float cle_chunk_sum(const CleChunk& ch, const float* b1, const float* tb, int lane) {
    const DFQ_GLOBAL float* g1 = (const DFQ_GLOBAL float*)b1;
    const DFQ_GLOBAL float* gt = (const DFQ_GLOBAL float*)tb;
    return cle_chunk_sum_with(ch, [g1](int64_t i) { return ld_coh(g1 + i); }, [gt](int64_t i) { return ld_coh(gt + i); },
                              lane);
}

// Tiny chunk (< 8 elements, no tiles): scalar row_sum of |W - snap| on lane 0, snap := W.
__device__ __forceinline__ float cle_tiny_chunk_sum(const CleLayer* __restrict__ layers, const CleChunk& ch) {
    const CleLayer Ly = layers[ch.layer];
    float* w = Ly.w + ch.c0;
    float* sn = Ly.snap + ch.c0;
    return aten_inner_sum([&](int64_t e) {
        const float x = w[e];
        const float dd = fabsf(x - sn[e]);
        sn[e] = x;
        return dd;
    }, ch.len);
}

// numpy pairwise float64 sum (identity 0 + pairwise_sum), as np.sum(diff_list).
// numpy's pairwise leaf: n <= 128 values, 8 accumulators.
template <class P>   // P: a typed (LDS / global) pointer to the values
__device__ __forceinline__ double np_pairwise_leaf(P x, int64_t n) {
    if (n < 8) {
        double res = 0.;
        for (int64_t i = 0; i < n; ++i) res += x[i];
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = x[j];
    int64_t i;
    for (i = 8; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += x[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += x[i];
    return res;
}

// numpy's recursion (blocks of <= 128 with 8 accumulators; split at n/2 rounded
// down to a multiple of 8) as an explicit post-order walk on one thread; a single
// leaf (every model here: <= 128 target layers) skips the frame stack.  The
// stack (kNpFrames frames) lives in the caller's LDS (`stack`: >= kNpStackFloats
// floats, 8-B aligned), so the kernel needs no scratch memory.
struct NpFrame {
    int64_t o, n;
    int64_t state;
};
constexpr int kNpFrames = 48;
constexpr int kNpStackFloats = kNpFrames * (int)(sizeof(NpFrame) + sizeof(double)) / 4;
template <class P>
__device__ double np_pairwise(P a, int64_t n, float* stack) {
    if (n <= 128) return 0. + np_pairwise_leaf(a, n);
    NpFrame* fr = reinterpret_cast<NpFrame*>(stack);
    double* acc = reinterpret_cast<double*>(fr + kNpFrames);
    int fp = 0, ap = 0;
    fr[fp++] = {0, n, 0};
    while (fp > 0) {
        NpFrame& f = fr[fp - 1];
        if (f.n <= 128) {
            acc[ap++] = np_pairwise_leaf(a + f.o, f.n);
            --fp;
        } else if (f.state == 0) {
            int64_t n2 = f.n / 2;
            n2 -= n2 % 8;
            f.state = 1;
            const NpFrame left{f.o, n2, 0}, right{f.o + n2, f.n - n2, 0};
            fr[fp++] = right;   // evaluated second
            fr[fp++] = left;    // evaluated first
        } else {
            const double right = acc[--ap];
            const double left = acc[--ap];
            acc[ap++] = left + right;
            --fp;
        }
    }
    return 0. + acc[0];   // add.reduce starts from the identity
}

// Per-layer fp32 mean from the chunk sums (final_reduce over the 8-slot buffer,
// then / n), np.sum over layers, history and the stop rule.  One block.
// kLeafOnly: nl <= 128 (numpy's pairwise sum is one leaf) -- no frame stack, so
// no scratch in the persistent kernel
// kCoherent: the chunk sums come from other blocks of the same launch (agent-
// coherent loads); else from an earlier launch (plain loads).
template <bool kLeafOnly = false, bool kCoherent = false>
__device__ __forceinline__ void cle_final_body(const CleLayer* __restrict__ layers, int32_t nl,
                                               const float* __restrict__ part, int32_t S, double* __restrict__ means,
                                               double* __restrict__ hist, CleState* __restrict__ st, double* sm,
                                               float* part_lds = nullptr, float* np_stack = nullptr,
                                               uint32_t* hflag = nullptr) {
    // The stop rule's inputs in one parallel pass of loads into LDS (part_lds): the
    // chunk sums, the layers' {(float)n, serial} and the state's 10 words.  Read
    // where they are used instead, they were dependent round trips of a serial
    // stop rule (7.6 us, DFQ_CLE_TL, the last launch's block timeline); loaded
    // into registers up front, they pushed the kernel past its 128 VGPRs.
    // Nothing else writes the state during this launch.
#ifdef DFQ_DIAGNOSTICS
    uint64_t* tlm = (kCoherent && threadIdx.x == 0 && g_cle_tl2) ? g_cle_tl2 + 4 * kCleTl2Fin : nullptr;
#endif
    constexpr int kStateWords = (int)(sizeof(CleState) / 4);
    static_assert(sizeof(CleState) % 4 == 0, "CleState: whole 4-B words");
    const int64_t nps = (int64_t)nl * (S + 2);
    DFQ_LDS float* pls = (DFQ_LDS float*)part_lds;   // typed: LDS / global accesses, not flat
    if (part_lds) {
        for (int64_t i = threadIdx.x; i < nps + kStateWords; i += blockDim.x) {
            const DFQ_GLOBAL float* src = (const DFQ_GLOBAL float*)(i < nps ? part + i
                                                                           : reinterpret_cast<const float*>(st) + (i - nps));
            pls[i] = kCoherent ? ld_coh(src) : *src;
        }
        __syncthreads();
    }
#ifdef DFQ_DIAGNOSTICS
    if (tlm) tlm[2] = __builtin_amdgcn_s_memrealtime();
#endif
    DFQ_LDS double* ms = (DFQ_LDS double*)sm;
    DFQ_GLOBAL double* mg = (DFQ_GLOBAL double*)means;
    const bool m_lds = nl <= 1024;
    double* m = m_lds ? sm : means;
    // (generic pointers here: the typed two-path form spilled 48-60 B in the loop
    // kernel; wave 0 has no stores outstanding at this point, so the flat loads
    // cost no extra wait)
    for (int l = threadIdx.x; l < nl; l += blockDim.x) {
        // serial: sum = 0 + (0 + slot); two_pass_reduction: its S-slot buffer
        // (at::get_num_threads()) summed as a contiguous reduction
        const float* pl = (part_lds ? part_lds : part) + (int64_t)l * S;
        auto ld = [&](int64_t e) { return (part_lds || !kCoherent) ? pl[e] : ld_coh(pl + e); };
        const float* lm = part_lds ? part_lds + (int64_t)nl * S + 2 * l : nullptr;
        const bool serial = lm ? lm[1] != 0.f : layers[l].nt == 1;
        const float sum = serial ? 0.f + (0.f + ld(0)) : 0.f + aten_inner_sum([&](int64_t e) { return ld(e); }, S);
        m[l] = (double)(sum / (lm ? lm[0] : (float)layers[l].n));
    }
    __syncthreads();
#ifdef DFQ_DIAGNOSTICS
    if (tlm) tlm[3] = __builtin_amdgcn_s_memrealtime();
#endif
    if (threadIdx.x == 0) {
        CleState s0;
        if (part_lds) {
            __builtin_memcpy(&s0, part_lds + nps, sizeof(CleState));
        } else {
            s0 = *st;
        }
        double dt = 0.0;
        if constexpr (kLeafOnly) {
            dt = nl > 0 ? 0. + (m_lds ? np_pairwise_leaf(ms, nl) : np_pairwise_leaf(mg, nl)) : 0.0;
        } else {
            dt = nl > 0 ? (m_lds ? np_pairwise(ms, nl, np_stack) : np_pairwise(mg, nl, np_stack)) : 0.0;
        }
        const int it = s0.iters;
        hist[it] = dt;
        int ic = s0.iter_count;
        double diff = s0.diff;
        if (fabs(diff - dt) > 1e-9) {
            ic = 0;
            diff = dt;
        } else {
            ic += 1;
        }
        const bool cont = (diff > s0.thr) && (ic < s0.count);
        const int done = (!cont || it + 1 >= s0.max_iters) ? 1 : 0;
        st->iters = it + 1;
        st->iter_count = ic;
        st->diff = diff;
        st->done = done;
        // the host's copy of the stop rule (pinned host memory; a system-scope
        // vector store), written every iteration: the loop's host side polls it for
        // the stop and paces its enqueue by it (cle_run_locked)
        if (hflag)
            __hip_atomic_store(hflag, ((uint32_t)(it + 1) << 1) | (uint32_t)done, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        // (A launched run's caller gate opens behind the rollback launch that follows
        // the loop -- cle_run_locked -- not here: the lagged schedule's next
        // iteration may be running speculatively beside this stop rule.)
    }
}

// The metric tiles (+ the next iteration's ranges) with the chunk combine and the
// stop rule folded in: the block that finishes a chunk's last tile sums that
// chunk, and the block that finishes the last chunk runs the stop rule -- two
// launches fewer per iteration.  Hand-offs between blocks go through
// agent-coherent stores / loads and monotone arrival counters (cnt: one per
// chunk, then one for the launch; zeroed by plan_run, iteration i's target is
// (i + 1) x members); the ordering of the hand-offs: handoff_arrive.
// Arrival on a block-to-block hand-off counter (chunk tiles -> chunk sum -> stop
// rule).  The words handed over (level-1 sums, chunk tails, chunk sums) are
// written with agent-coherent stores (st_coh) and read with agent-coherent loads
// (ld_coh), and the caller has drained its stores (s_waitcnt vmcnt(0)) first.
// The sc1 hand-off form MI355X_MICROARCH.md lists as valid (section "visibility",
// Valid forms, table row 1; cdna_hip_programming.md Guideline 16): every
// handed-off word stored sc1 and drained by every storing wave before ONE lane's
// agent-scope counter add (behind the workgroup barrier), the workgroup whose add
// came last told by the returned value, and every load of the words an sc1 load to
// registers issued after that add returned (the other waves after a workgroup
// barrier).  No L2 write-back.  (The memory model's release / acquire form gave the
// same results 50 % slower: each release writes the arriving block's XCD L2 back,
// profiles/r03/cle_ab_d.jsonl.)
__device__ __forceinline__ bool handoff_arrive(uint32_t* c, uint32_t target) {
    return __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == target;
}

// Blocks of the lagged schedule's stop rule: one wave per chunk sum (host and kernel).
__host__ __device__ inline int64_t cle_stop_blocks(int64_t nchunks) {
    return nchunks > 0 ? (nchunks + kThreads / 64 - 1) / (kThreads / 64) : 1;
}

struct CleFin {
    uint32_t* cnt;
    float* part;
    double* means;
    double* hist;
    int64_t nchunks, nbig;   // all chunks / chunks with tiles (len >= 8)
    int32_t S, nl;
    int32_t last;            // the round-4 schedule's tiles-only launch (the stop rule's block without tiles)
    uint32_t* hflag;         // pinned host word: (iterations << 1) | done, or null
    int32_t stop_arrival;    // 1: the stop rule runs at the iteration's last tile arrival (round-4 schedule);
                             // 0: as a block of its own (lagged schedule, stop_it)
};

// One launch of iteration group g.  The group's launches k < steps run the
// rescale tasks of chain step k of iteration g (blocks [0, nab)); beside them run
// metric tiles and next-iteration range tasks placed in this launch by the
// planner (dfq_cle_plan_create): "own" ones of iteration g and "prev" ones of
// iteration g - 1 (the lagged schedule: a tensor's tiles and ranges go anywhere
// after its last rescale of iteration g-1 and before its first rescale of
// iteration g).  Blocks: [0, nab) rescale, then nto own tiles, ntp prev tiles,
// nro own ranges, nrp prev ranges.
//
// Lagged schedule: iteration g's first steps run before iteration g-1's stop
// rule (the last tile arrival) has decided -- speculatively.  When that stop rule
// says done, iteration g is discarded: its rescale blocks skip from then on
// (st->done) and cle_loop_rollback_kernel restores the weights from the snapshots
// (= iteration g-1's weights: every tile of g-1 ran before any rescale of g
// touched its tensor) and the per-channel vectors from the saves of iteration g.
// Tiles of iteration i are placed after every tile of i-1 (the planner's band),
// so they start only after stop(i-1): a tile never runs for a discarded
// iteration, and its snapshot writes and arrivals are always real.  Every block
// takes its iteration, parity and arrival round from the launch argument g,
// never from st (the stop rule advances st mid-launch).
static_assert(kCleTilesLds - kCleTile >= kNpStackFloats, "np_pairwise's frame stack after the tile area");
union CleStepLds {
    CleApplyLds apply;
    float tiles[kCleTilesLds > kCleRangeLds ? kCleTilesLds : kCleRangeLds];
};

// Block order of a step launch: metric tiles (the launch's longest blocks: 8,192
// elements, 12 B each), rescale tasks, the stop rule, range tasks.  MobileNetV2's
// first launch holds 1,994 blocks, about two rounds of resident ones; with the tiles
// last they started in the second round and set the launch's tail.  CLE 2.27-2.29
// against 2.39-2.40 ms, ResNet-50 (tiles in a launch of their own) unchanged
// (profiles/r06/cle_ab_tiles_first_r06t/u.jsonl; tiles then ranges first: 2.36).
// DFQ_CLE_TILES_FIRST=0 (diagnostics): the round-6 order, tiles after the stop rule.
constexpr bool kCleTilesFirst = true;
#ifdef DFQ_DIAGNOSTICS
__device__ int g_cle_tiles_first = kCleTilesFirst ? 1 : 0;
#endif

// POS = false (no position-parallel 3x3 rescale tiles): capped at 128 VGPRs,
// 4 waves per SIMD like the rescale body alone
// (POS capped at 3 waves per SIMD -- 168 VGPRs, 124 B of spills -- measured slower:
// profiles/r04/cle_ab_r04t.jsonl)
template <bool POS>
#ifndef DFQ_CLE_POS_WAVES   // waves per SIMD asked of the POS kernel (1: no cap); A/B as above
#define DFQ_CLE_POS_WAVES 1
#endif
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(POS ? DFQ_CLE_POS_WAVES : 4)))
cle_loop_step_kernel(const CleRel* __restrict__ rels, const CleTask* __restrict__ atasks, int64_t a0, int64_t a1,
                     int64_t nab, uint32_t* __restrict__ rng, int64_t M, int is_signed, float eps, double smin,
                     double smax, const CleLayer* __restrict__ layers, const CleChunk* __restrict__ chunks,
                     const int64_t* __restrict__ b1off, const CleUnit* __restrict__ units, int64_t uo, int64_t nuo,
                     int64_t nto, int64_t up, int64_t nup, int64_t ntp, float* __restrict__ b1buf,
                     float* __restrict__ tailbuf, const CleTask* __restrict__ rtasks, int64_t ro, int64_t nro_t,
                     int64_t nro, int64_t rp, int64_t nrp_t, int64_t nrp, CleFin F, CleState* __restrict__ st,
                     int32_t g, float* __restrict__ vsave, int32_t* __restrict__ vtag, int32_t stop_it) {
    __shared__ CleStepLds L;
    __shared__ int flag;
    if (st->done) return;
    int64_t blk = blockIdx.x;
#ifdef DFQ_DIAGNOSTICS
    const bool tiles_first = g_cle_tiles_first != 0;   // DFQ_CLE_TILES_FIRST (A/B)
#else
    constexpr bool tiles_first = kCleTilesFirst;
#endif
    // lagged schedule: the stop rule of iteration stop_it takes cle_stop_blocks blocks
    // (its chunk sums, then the stop rule at their last arrival)
    const int64_t nstop = stop_it >= 0 ? cle_stop_blocks(F.nchunks) : 0;
    if (tiles_first) {   // block order: metric tiles, rescale tasks, the stop rule, ranges
        const int64_t ns = nab + nstop, ntl = nto + ntp;
        if (blk < ntl) blk += ns;
        else if (blk < ntl + ns) blk -= ntl;
    }
    if (blk < nab) {   // this step's rescale tasks (iteration g)
        cle_apply_body<POS>(rels, atasks, a0, a1, rng, M, g & 1, g == 0, is_signed, eps, smin, smax, blk, nab, L.apply,
                            vsave, vtag, g);
        return;
    }
    blk -= nab;
#ifdef DFQ_DIAGNOSTICS
    const bool tl2 = g_cle_tl2 != nullptr && blk < kCleTl2Fin && (g_cle_tl2_a0 < 0 || (a0 == g_cle_tl2_a0 && nab > 0));
    const uint64_t tl2_start = tl2 ? __builtin_amdgcn_s_memrealtime() : 0;
    auto tl2_rec = [&](int role) {
        if (tl2 && threadIdx.x == 0) {
            uint64_t* r = g_cle_tl2 + 4 * blk;
            r[0] = tl2_start;
            r[1] = __builtin_amdgcn_s_memrealtime();
            r[2] = (uint64_t)role;
        }
    };
#else
    auto tl2_rec = [](int) {};
#endif
    float* lds = L.tiles;
    // The last arrival of the iteration: tiny chunks' sums, then the per-layer
    // means, the history and the stop rule.
    auto finish = [&]() {
#ifdef DFQ_DIAGNOSTICS
        const uint64_t tf0 = __builtin_amdgcn_s_memrealtime();
#endif
        if (threadIdx.x == 0 && F.nchunks > F.nbig)   // tiny chunks exist (fallback schedule only)
            for (int64_t k = 0; k < F.nchunks; ++k) {
                const CleChunk c2 = chunks[k];
                if (c2.len < 8) st_coh(F.part + (int64_t)c2.layer * F.S + c2.t, 0.f + cle_tiny_chunk_sum(layers, c2));
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // the chunk sums, layer sizes and state words (cle_final_body) after the means
        const bool stage_part = (int64_t)F.nl * (F.S + 2) + (int64_t)(sizeof(CleState) / 4) + 2048 <= kCleTile;
        if (F.nl <= 128)   // numpy's pairwise sum over the layer means is one leaf
            cle_final_body<true, true>(layers, F.nl, F.part, F.S, F.means, F.hist, st, reinterpret_cast<double*>(lds),
                                       stage_part ? lds + 2048 : nullptr, nullptr, F.hflag);
        else   // the frame stack after the metric tile area (free: this block's units are done)
            cle_final_body<false, true>(layers, F.nl, F.part, F.S, F.means, F.hist, st,
                                        reinterpret_cast<double*>(lds), stage_part ? lds + 2048 : nullptr,
                                        lds + kCleTile, F.hflag);
#ifdef DFQ_DIAGNOSTICS
        if (tl2 && threadIdx.x == 0) {
            uint64_t* r = g_cle_tl2 + 4 * kCleTl2Fin;
            r[0] = tf0;
            r[1] = __builtin_amdgcn_s_memrealtime();
        }
#endif
    };
    if (stop_it >= 0) {   // lagged schedule: the stop rule of iteration stop_it
        if (blk < nstop) {
            // The iteration's chunk sums, one wave per chunk, from the level-1 sums and
            // tail words its tiles wrote in earlier launches (no tile of any iteration
            // runs in this launch: the stop rule's offset follows its iteration's
            // band and precedes the next iteration's; host structure checker); the
            // last block to arrive runs the stop rule.  The tiles themselves no longer
            // arrive anywhere (their chunk's last arrival summed the chunk: a store
            // drain, an arrival and a staged sum on the launch's longest blocks).
            // (Staging each wave's level-1 sums through LDS first measured the same:
            // profiles/r06/cle_lib_ab_stop_chunk_sums_staged_r06z.jsonl.)
            const int64_t c = blk * (kThreads / 64) + (threadIdx.x >> 6);
            if (c < F.nchunks) {
                const CleChunk ch = chunks[c];
                if (ch.len >= 8) {   // (tiny chunks: finish, thread 0)
                    const float fa = cle_chunk_sum(ch, b1buf + b1off[c], tailbuf + c * kCleTailWords, threadIdx.x & 63);
                    if ((threadIdx.x & 63) == 0) st_coh(F.part + (int64_t)ch.layer * F.S + ch.t, 0.f + fa);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0)
                flag = handoff_arrive(F.cnt + F.nchunks, ((uint32_t)stop_it + 1u) * (uint32_t)nstop - 1u);
            __syncthreads();
            if (flag) finish();
            return;
        }
        blk -= nstop;
    }
    const int64_t ntiles = nto + ntp;
    if (blk >= ntiles) {   // next-iteration ranges of tensors final by now
        blk -= ntiles;
        const bool own = blk < nro;
        const int64_t b = own ? blk : blk - nro;
        // own: iteration g's tasks (ranges of g + 1); prev: iteration g - 1's (ranges of g)
        cle_range_body(rels, rtasks, own ? ro : rp, (own ? ro : rp) + (own ? nro_t : nrp_t), rng, M,
                       own ? (g + 1) & 1 : g & 1, b, own ? nro : nrp, L.tiles);
        tl2_rec(2);
        return;
    }
    const bool own = blk < nto;
    const int32_t it = own ? g : g - 1;                    // the tiles' iteration
    const int64_t tb = own ? blk : blk - nto;
    const int64_t tnb = own ? nto : ntp;
    const uint32_t round = (uint32_t)it + 1u;
    // Arrival on counter c (handoff_arrive); returns whether this block arrived last.
    auto arrive = [&](uint32_t* c, uint32_t members) -> bool {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) flag = handoff_arrive(c, round * members - 1u);
        __syncthreads();
        return flag != 0;
    };
    if (F.nbig == 0) {   // no chunk has tiles (tiny or no target layers): the fallback launch's one block finishes
        if (own && tb == 0 && F.last) finish();
        return;
    }
    const uint32_t fin_members = (uint32_t)F.nbig;
    auto hook = [&](const CleUnit& un, const CleChunk& ch, int64_t nb1) {
        if (!arrive(F.cnt + un.chunk, (uint32_t)(nb1 + 1))) return;   // not the chunk's last tile
        {
            // the chunk's level-1 sums and tail words in one parallel pass of coherent
            // loads into LDS (free again: the unit is done), then one wave sums them
            const float* gb1 = b1buf + b1off[un.chunk];
            const float* gtb = tailbuf + (int64_t)un.chunk * kCleTailWords;
            const int64_t nw = 32 * nb1;
            const bool staged = nw + kCleTailWords <= kCleTile;
            if (staged) {
                DFQ_LDS float* ll = (DFQ_LDS float*)lds;
                const DFQ_GLOBAL float* g1 = (const DFQ_GLOBAL float*)gb1;
                for (int64_t i = threadIdx.x; i < nw; i += kThreads) ll[i] = ld_coh(g1 + i);
                if (threadIdx.x < kCleTailWords) ll[nw + threadIdx.x] = ld_coh((const DFQ_GLOBAL float*)gtb + threadIdx.x);
            }
            __syncthreads();
            if (threadIdx.x < 64) {
                const float fa = staged ? cle_chunk_sum_with(ch, [&](int64_t i) { return lds[i]; },
                                                             [&](int64_t i) { return lds[nw + i]; }, threadIdx.x)
                                        : cle_chunk_sum(ch, gb1, gtb, threadIdx.x);
                if (threadIdx.x == 0) st_coh(F.part + (int64_t)ch.layer * F.S + ch.t, 0.f + fa);
            }
        }
        if (F.stop_arrival && arrive(F.cnt + F.nchunks, fin_members)) finish();   // the iteration's last arrival
    };
    if (F.stop_arrival)   // round-4 schedule: chunk sums and the stop rule at the tiles' arrivals
        cle_tiles_body<decltype(hook)>(layers, chunks, b1off, units + (own ? uo : up), own ? nuo : nup, b1buf, tailbuf,
                                       tb, tnb, lds, lds + kCleTile + kCleTailWords, hook);
    else   // lagged schedule: the stop rule's launch sums the chunks (above)
        cle_tiles_body(layers, chunks, b1off, units + (own ? uo : up), own ? nuo : nup, b1buf, tailbuf, tb, tnb, lds,
                       lds + kCleTile + kCleTailWords);
#ifdef DFQ_DIAGNOSTICS
    if (tl2) {   // role 3: the block's unit was a chunk's tail tile
        const CleUnit un0 = units[(own ? uo : up) + tb];
        tl2_rec(un0.tile >= (chunks[un0.chunk].len / 32) / 256 ? 3 : 1);
    }
#else
    tl2_rec(1);
#endif
}

// After the loop: undo a speculative iteration (the lagged schedule's iteration
// A = st->iters, started before stop(A - 1) said done).  Weights: every target
// layer := its snapshot (iteration A - 1's weights; the tiles of A - 1 wrote it
// before any rescale of A touched the tensor).  Vectors (B1, BN fake weight / bias,
// S): restored from the saves of every per-channel task that ran in iteration A.
// Correct whether or not iteration A started: without it the weights equal their
// snapshots already and no save carries A.
__global__ void __launch_bounds__(kThreads)
cle_loop_rollback_kernel(const CleLayer* __restrict__ layers, int32_t nl, const CleRel* __restrict__ rels,
                         const CleTask* __restrict__ atasks, int64_t n_at, const float* __restrict__ vsave,
                         const int32_t* __restrict__ vtag, const CleState* __restrict__ st) {
    const int32_t A = st->iters;
    const int64_t gt = (int64_t)blockIdx.x * kThreads + threadIdx.x, gs = (int64_t)gridDim.x * kThreads;
    for (int32_t l = 0; l < nl; ++l) {
        const CleLayer Ly = layers[l];
        for (int64_t i = gt; i < Ly.n; i += gs) Ly.w[i] = Ly.snap[i];
    }
    for (int64_t t = blockIdx.x; t < n_at; t += gridDim.x) {
        const CleTask tk = atasks[t];
        if (tk.kind != kApplyChannels || vtag[t] != A) continue;
        const CleRel& R = rels[tk.rel];
        const float* v = vsave + 2 * R.moff;
        for (int64_t c = tk.a + threadIdx.x; c < tk.b; c += kThreads) {
            if (R.b1) R.b1[c] = v[c];
            if (R.bnw) R.bnw[c] = v[R.c1 + c];
            if (R.bnb) R.bnb[c] = v[2 * R.c1 + c];
            if (R.sacc) R.sacc[c] = v[3 * R.c1 + c];
        }
    }
}

}  // namespace dfq

constexpr int32_t kCleHistCap = 1025;   // per-iteration diffs kept in the plan's tables

struct dfq_cle_plan {
    CleRel* d_rels = nullptr;
    CleTask* d_rtasks = nullptr;
    CleTask* d_atasks = nullptr;
    CleLayer* d_layers = nullptr;
    CleChunk* d_chunks = nullptr;
    uint32_t* d_rng = nullptr;      // [2 parities][mins M | maxs M]
    float* d_part = nullptr;        // [layers][slots]
    int32_t slots = 8;              // torch.mean's thread buffer (the reference run's thread count)
    double* d_means = nullptr;
    double* d_hist = nullptr;       // this run's history (the tables' kCleHistCap slots, or the context's)
    double* d_hist_tables = nullptr;
    CleState* d_state = nullptr;
    CleState* h_state = nullptr;    // pinned (the device context's, set by run)
    uint32_t* d_flag = nullptr;     // the stop rule's host word (the device context's, set by run)
    uint64_t* d_sig = nullptr;      // a launched run: the caller's gate word and its generation
    uint64_t gen = 0;
    hipStream_t st = nullptr;       // the loop's stream (the device context's)
    std::vector<int64_t> rstep, astep;   // task offsets per step (size steps + 1)
    std::vector<char> step_pos;          // per step: position-parallel W2 tiles (the POS rescale kernel)
    int64_t M = 0, nchunks = 0;
    int32_t nl = 0, chains = 0, steps = 0;
    bool fused = false;   // one range launch per iteration (see dfq_cle_plan_create)
    CleUnit* d_units = nullptr;
    int64_t* d_b1off = nullptr;
    float* d_b1 = nullptr;          // level-1 sums, [chunk][nb1][32]
    float* d_tail = nullptr;        // [chunk][kCleTailWords]
    int64_t nunits = 0;
    double smin = 1e-8, smax = 1e8;
    int32_t is_signed = 0;
    float eps = 0.f;
    void* d_tables = nullptr;       // every device table above: ONE allocation (unless pooled)
    bool pooled = false;            // the tables live in the device context's pool
    void* d_snap_owned = nullptr;   // snapshots when the caller passed no workspace
    uint32_t* d_cnt = nullptr;      // tiles_fin arrival counters [nchunks + 1]
    int64_t nbig = 0;               // chunks with tiles
    int64_t ri0 = 0, ri1 = 0;       // fused: each iteration's range tasks (the rest come from the rescales)
    std::vector<int64_t> uoffs, roffs;   // per offset k < 2 nlaunch: units / range tasks [v[k], v[k + 1])
    int32_t nlaunch = 0;                 // launches per iteration group (steps, + 1 for a tiles-only launch)
    int32_t stop_off = -1;               // lagged: the stop rule's block offset (else the last tile arrival)
    bool lagged = false;                 // some tiles run in the next group (speculative iterations)
    float* d_vsave = nullptr;            // lagged: per-channel vectors before the iteration's multiply [2 M]
    int32_t* d_vtag = nullptr;           // ... and the iteration that saved them, per rescale task
    int64_t n_at = 0;                    // rescale tasks
    int dev = 0;
    struct CleAsync* async = nullptr;   // dfq_cle_plan_launch's worker and result
    bool abandoned = false;             // join gave up waiting for the launched loop
    int64_t bytes[3] = {0, 0, 0};       // algorithmic bytes per iteration: rescale, metric, ranges
    bool timed = false;                 // dfq_cle_plan_set_timing: HIP events around the loop
    float loop_ms = -1.f;               // the last run's device time, first launch to last (timed runs)
    int32_t launched = 0;               // iteration groups the last run enqueued
#ifdef DFQ_DIAGNOSTICS
    std::vector<CleRel> h_rels;
    std::vector<CleTask> h_atasks;
#endif
};

// DFQ_CLE_TIMING: host-side phase times of create / run / destroy on stderr.
static bool cle_timing() {
    static const bool on = ab_env("DFQ_CLE_TIMING") != nullptr;
    return on;
}
static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Per-device loop stream and pinned state word, shared by every plan of the
// process (creating and destroying them per call cost ~0.6 ms); plan_run holds
// the device's lock while it uses them.
struct CleDeviceCtx {
    std::mutex mu;
    hipStream_t st = nullptr;
    CleState* h_state = nullptr;   // pinned: the run's state
    uint32_t* h_flag = nullptr;    // pinned, written by the stop rule: (iterations << 1) | done
    uint32_t* d_flag = nullptr;    // its device address
    // Table pool: one plan at a time keeps its tables here (device + pinned upload
    // mirror), so a plan costs no hipMalloc / hipFree (hipFree waits for the whole
    // device) and its upload is an async DMA on the loop stream.
    char* d_pool = nullptr;
    size_t pool_cap = 0;
    char* h_pool = nullptr;
    size_t hpool_cap = 0;
    bool pool_busy = false;
    uint64_t pool_struct = 0;                      // CleStructure::id whose address-free tables the pool holds
    hipEvent_t pool_ev = nullptr;                  // behind the last upload from h_pool
    double* d_hist = nullptr;                      // histories longer than the tables' kCleHistCap
    int64_t hist_cap = 0;
    double* h_hist = nullptr;                      // pinned: the run's history comes back here
    int64_t h_hist_cap = 0;
    // asynchronous runs (dfq_cle_plan_launch): the signal word callers' streams
    // wait on, its last generation, the launched plan not yet joined
    void* sig = nullptr;
    int sig_state = 0;                             // -1: the device cannot wait on a value
    uint64_t gen = 0;
    struct dfq_cle_plan* pending = nullptr;
    hipEvent_t in_ev = nullptr;                    // the caller's producers, for the loop stream
    struct CleWorker* worker = nullptr;            // drives launched runs
};
static CleDeviceCtx& cle_device_ctx(int dev) {
    static CleDeviceCtx ctx[64];
    return ctx[dev & 63];
}
// The loop stream and the pinned state word (caller holds ctx.mu).  Creating a
// stream can take milliseconds the first time, so dfq_preload does it up front.
static hipError_t cle_ctx_ready(CleDeviceCtx& ctx) {
    hipError_t e = hipSuccess;
    if (!ctx.st) {   // high priority: a hardware queue of its own (see dfq_cle_plan_launch)
        int least = 0, greatest = 0;
        e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&ctx.st, hipStreamNonBlocking, greatest);
    }
    if (e == hipSuccess && !ctx.h_state) e = hipHostMalloc(&ctx.h_state, sizeof(CleState));
    if (e == hipSuccess && !ctx.h_flag) {
        e = hipHostMalloc(&ctx.h_flag, 64, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx.d_flag), ctx.h_flag, 0);
    }
    if (e == hipSuccess && !ctx.pool_ev) e = hipEventCreateWithFlags(&ctx.pool_ev, hipEventDisableTiming);
    if (e == hipSuccess && !ctx.in_ev) e = hipEventCreateWithFlags(&ctx.in_ev, hipEventDisableTiming);
    return e;
}

static void cle_plan_free(dfq_cle_plan* p) {
    const double t0 = now_us();
    if (p->pooled) {   // hand the pool back (a run has synchronised its stream; an unrun
                       // plan's upload is waited for by the next user of the pool)
        CleDeviceCtx& ctx = cle_device_ctx(p->dev);
        std::lock_guard<std::mutex> lock(ctx.mu);
        ctx.pool_busy = false;
    } else {
        (void)hipFree(p->d_tables);
    }
    (void)hipFree(p->d_snap_owned);
    if (cle_timing()) fprintf(stderr, "DFQ_CLE_TIMING free: %.1f us\n", now_us() - t0);
    delete p;
}

static int64_t snap_bytes(int64_t n) { return ceil_div(n * (int64_t)sizeof(float), (int64_t)256) * 256; }

// Byte layout of the plan's device tables (one allocation, one host->device copy).
struct TableLayout {
    int64_t total = 0;
    template <typename T>
    int64_t add(int64_t count) {
        const int64_t off = total;
        total += ceil_div((int64_t)sizeof(T) * std::max<int64_t>(count, 1), (int64_t)256) * 256;
        return off;
    }
};

extern "C" int64_t dfq_cle_plan_ws_bytes(const int64_t* target_n, int32_t n_targets) {
    if (n_targets < 0 || (n_targets > 0 && !target_n)) return -1;
    int64_t b = 0;
    for (int32_t l = 0; l < n_targets; ++l) {
        if (target_n[l] < 0) return -1;
        b += snap_bytes(target_n[l]);
    }
    return b;
}

// Everything dfq_cle_plan_create derives from the relations' and targets' shapes
// and tensor identities -- chains, steps, tasks, metric chunks and units, the
// placement -- but no address: a plan of the same structure reuses it and binds
// its own tensors (cle_structure_key / the cache in dfq_cle_plan_create).
struct CleStructure {
    std::vector<CleRel> R;   // fused / depthwise / self-range flags set (addresses: the first plan's)
    int64_t M = 0;
    int32_t chains = 0, steps = 0;
    bool fused = false;
    std::vector<CleTask> rt, at;
    std::vector<int64_t> rstep, astep;
    int64_t ri0 = 0, ri1 = 0;
    std::vector<CleLayer> layers;   // n, nt (w / snap bound per plan)
    std::vector<CleChunk> chunks;
    std::vector<CleUnit> units;
    std::vector<int64_t> b1off;
    int64_t nb1_total = 0;
    std::vector<int64_t> uoffs, roffs;
    int32_t nlaunch = 0, stop_off = -1;
    bool lagged = false;
    double t_chains = 0, t_tasks = 0, t_chunks = 0, t_place = 0;
    // algorithmic HBM bytes of one iteration (dfq_cle_plan_stats): the rescales
    // (8 B per weight element and per channel of each per-channel vector: read +
    // write; a depthwise pair's filter once), the metric tiles (12 B per target
    // element: W and the snapshot read, the snapshot written) and the range tasks
    // that read weights (4 B per element; self ranges are free)
    int64_t bytes_rescale = 0, bytes_metric = 0, bytes_range = 0;
    uint64_t id = 0;   // unique per built structure: the device pool remembers whose tables it holds
};
static std::atomic<uint64_t> g_struct_ids{0};

static int cle_build_structure(std::vector<CleRel> R, int64_t M, int32_t n_rel, float* const* targets,
                               const int64_t* target_n, int32_t n_targets, int32_t ref_threads, CleStructure& S) {
    const double tp1 = now_us();
    // chains: connected components over the tensors a relation touches
    std::vector<int32_t> parent(n_rel);
    std::iota(parent.begin(), parent.end(), 0);
    auto find = [&](int32_t x) {
        while (parent[x] != x) x = parent[x] = parent[parent[x]];
        return x;
    };
    for (int32_t a = 0; a < n_rel; ++a) {
        const void* pa[5] = {R[a].w1, R[a].w2, R[a].b1, R[a].bnw, R[a].bnb};
        for (int32_t b = 0; b < a; ++b) {
            const void* pb[5] = {R[b].w1, R[b].w2, R[b].b1, R[b].bnw, R[b].bnb};
            bool share = false;
            for (int i = 0; i < 5 && !share; ++i)
                for (int j = 0; j < 5 && !share; ++j) share = pa[i] && pa[i] == pb[j];
            if (share) parent[find(a)] = find(b);
        }
    }
    std::vector<int32_t> step_of(n_rel), comp_len(n_rel, 0);
    int32_t chains = 0, steps = 0;
    for (int32_t r = 0; r < n_rel; ++r) {
        const int32_t c = find(r);
        if (comp_len[c] == 0) ++chains;
        step_of[r] = comp_len[c]++;
        steps = std::max(steps, step_of[r] + 1);
    }
    // Fused schedule: a relation's W2 must be untouched by the earlier relations of
    // its chain (its column range can be taken at the start of the iteration), and
    // its W1 untouched too, or the W2 of the immediately preceding relation -- whose
    // rescale then produces the W1 row ranges.  Otherwise: per-step range launches.
    std::vector<int32_t> w1_src(n_rel, -1);
    bool fused = true;
    {
        const char* fe = ab_env("DFQ_CLE_FUSED");   // diagnostics A/B: per-step range launches
        if (fe && fe[0] == '0') fused = false;
        std::vector<std::vector<int32_t>> chain_of(n_rel);
        for (int32_t r = 0; r < n_rel; ++r) chain_of[find(r)].push_back(r);
        for (const auto& L : chain_of) {
            for (size_t j = 0; j < L.size() && fused; ++j) {
                const CleRel& cr = R[L[j]];
                for (size_t i = 0; i < j && fused; ++i) {
                    const CleRel& cq = R[L[i]];
                    if (cq.w1 == cr.w2 || cq.w2 == cr.w2) fused = false;
                    if (cq.w1 == cr.w1 || cq.w2 == cr.w1) {
                        const bool ok = i + 1 == j && cq.w2 == cr.w1 && cq.w1 != cr.w1 && w1_src[L[j]] < 0 &&
                                        (cq.i2 > 1 || cq.o2g == 1) && cr.c1 == cq.o2 && cr.len1 == cq.i2 * cq.khw2;
                        if (ok) w1_src[L[j]] = L[i];
                        else fused = false;
                    }
                }
            }
        }
        if (fused)
            for (int32_t r = 0; r < n_rel; ++r)
                if (w1_src[r] >= 0) R[w1_src[r]].fuse_next = r;
    }
    // Depthwise pairs (fused schedule): relation r whose W1 is the depthwise W2 of
    // the relation q right before it in its chain runs in q's launch: its W1 row
    // ranges are derived from q's W2 range words (cle_rel_scale), q's filter
    // rescale and r's W1 rescale become ONE task (kApplyDwBoth), and r no longer
    // needs W1 range words.  MobileNetV2: 5 rescale launches per iteration -> 3.
    std::vector<int32_t> dw_next(n_rel, -1);
    if (fused) {
        for (int32_t r = 0; r < n_rel; ++r) {
            const int32_t q = w1_src[r];
            if (q < 0 || R[q].dw_prev >= 0 || dw_next[q] >= 0) continue;
            const CleRel& cq = R[q];
            const CleRel& cr = R[r];
            const bool dw = cq.i2 == 1 && cq.o2g == 1 && cq.o2 == cq.c1 && cr.c1 == cq.o2 && cr.len1 == cq.khw2;
            if (!dw) continue;
            R[r].dw_prev = q;
            R[q].fuse_next = -1;   // no range words to produce for r's W1
            dw_next[q] = r;
        }
        // steps again: a depthwise-paired relation shares its predecessor's step
        std::vector<int32_t> cur(n_rel, 0);
        steps = 0;
        for (int32_t r = 0; r < n_rel; ++r) {
            const int32_t c = find(r);
            step_of[r] = R[r].dw_prev >= 0 ? step_of[R[r].dw_prev] : cur[c]++;
            steps = std::max(steps, step_of[r] + 1);
        }
    }
    const double tp2 = now_us();
    // tasks: per-step range + rescale launches, or (fused) one range launch for
    // every relation's W2 (and untouched W1) followed by the rescale launches
    std::vector<CleTask> rt, at;
    std::vector<CleTask>* rout = &rt;   // where the range-task builders emit
    std::vector<int64_t> rstep(1, 0), astep(1, 0);
    auto w2_range_tasks = [&](int32_t r) {
        const CleRel& c = R[r];
        if (c.i2 == 1) {
            const int64_t k = rows_per_task(c.o2g * c.khw2);
            for (int64_t a = 0; a < c.c1; a += k)
                rout->push_back({r, kRangeW2Contig, a, std::min<int64_t>(a + k, c.c1), 0, 0});
        } else {
            for (int64_t a = 0; a < c.o2; a += kColTileRows)
                for (int64_t i0 = 0; i0 < c.i2; i0 += kThreads)
                    rout->push_back({r, kRangeW2Tile, a, std::min<int64_t>(a + kColTileRows, c.o2), i0,
                                     std::min<int64_t>(i0 + kThreads, c.i2)});
            for (int64_t a = 0; a < c.c1; a += kCleChansPerTask)
                rout->push_back({r, kRangeReset, a, std::min<int64_t>(a + kCleChansPerTask, c.c1), 0, 0});
        }
    };
    auto w1_range_tasks = [&](int32_t r) {
        const CleRel& c = R[r];
        if (c.dw_prev >= 0) return;   // derived from the depthwise predecessor's W2 words
        if (fused && w1_src[r] >= 0) {   // produced by the previous relation's rescale: reset the next parity
            for (int64_t a = 0; a < c.c1; a += kCleChansPerTask)
                rout->push_back({r, kRangeResetW1, a, std::min<int64_t>(a + kCleChansPerTask, c.c1), 0, 0});
        } else {
            const int64_t k = rows_per_task(c.len1);
            for (int64_t a = 0; a < c.c1; a += k)
                rout->push_back({r, kRangeW1, a, std::min<int64_t>(a + k, c.c1), 0, 0});
        }
    };
    // rows per W1 / depthwise-pair rescale task: rows_per_task (one row per wave)
    // times a factor (diagnostics A/B: DFQ_CLE_W1_ROWS / DFQ_CLE_DW_ROWS)
    // 0: the default rule (twice the rows for tasks of short rows, below)
    const int64_t w1_mult = [] {
        const char* e = ab_env("DFQ_CLE_W1_ROWS");
        return e && *e ? std::max<int64_t>(1, atoll(e)) : int64_t(0);
    }();
    auto w1_rows = [&](int64_t len1) {
        const int64_t k = rows_per_task(len1);
        if (w1_mult > 0) return w1_mult * k;
        return k * len1 < kCleW1SmallElems ? 2 * k : k;
    };
    const int64_t dw_mult = [] {
        const char* e = ab_env("DFQ_CLE_DW_ROWS");
        return e && *e ? std::max<int64_t>(1, atoll(e)) : kCleDwRowsMult;
    }();
    auto apply_tasks = [&](int32_t r, std::vector<CleTask>& out) {
        const CleRel& c = R[r];
        if (c.dw_prev < 0)   // else the predecessor's kApplyDwBoth rescales this W1
            for (int64_t a = 0, k = w1_rows(c.len1); a < c.c1; a += k)
                out.push_back({r, kApplyW1, a, std::min<int64_t>(a + k, c.c1), 0, 0});
        if (dw_next[r] >= 0) {
            for (int64_t a = 0, k = dw_mult * rows_per_task(c.o2g * c.khw2); a < c.c1; a += k)
                out.push_back({r, kApplyDwBoth, a, std::min<int64_t>(a + k, c.c1), dw_next[r], 0});
        } else if (c.i2 == 1) {
            for (int64_t a = 0, k = rows_per_task(c.o2g * c.khw2); a < c.c1; a += k)
                out.push_back({r, kApplyW2Contig, a, std::min<int64_t>(a + k, c.c1), 0, 0});
        } else {
            // KH*KW > 1 tiles go position-parallel, a row at a time: fewer rows per
            // task, more tasks in flight (ResNet-50's 3x3 W2 tiles: 16 rows took
            // ~70 us, DFQ_CLE_TL); 1x1 tiles keep kColTileRows (loads issued together)
            const int64_t rows = (c.khw2 > 1 && c.khw2 <= kTileMaxKhw) ? kPosTileMaxRows : kColTileRows;
            for (int64_t a = 0; a < c.o2; a += rows)
                for (int64_t i0 = 0; i0 < c.i2; i0 += kThreads)
                    out.push_back({r, kApplyW2Tile, a, std::min<int64_t>(a + rows, c.o2), i0,
                                   std::min<int64_t>(i0 + kThreads, c.i2)});
        }
        // one channel per thread: each channel's scale is a chain of dependent loads
        // and fp32 divides, and 1,024-channel tasks (4 channels a thread, one after
        // the other) were the slowest of their steps (6-9 us, DFQ_CLE_TL)
        for (int64_t a = 0; a < c.c1; a += kThreads)
            out.push_back({r, kApplyChannels, a, std::min<int64_t>(a + kThreads, c.c1), 0, 0});
    };
    int64_t ri0 = 0, ri1 = 0;
    if (fused) {
        for (int32_t r = 0; r < n_rel; ++r) {
            w1_range_tasks(r);
            w2_range_tasks(r);
        }
        rstep.push_back((int64_t)rt.size());
        // Self ranges: a W1 that no earlier relation of its chain touches is final
        // once its own row rescale ran, so that task writes the row's next range
        // (no kRangeW1 task); likewise a depthwise W2 after kApplyDwBoth.  The
        // first iteration's ranges still come from the full list [rstep0, rstep1);
        // each iteration's tiles launch runs the rest, [ri0, ri1).
        for (int32_t r = 0; r < n_rel; ++r) {
            if (w1_src[r] < 0 && R[r].dw_prev < 0) R[r].w1_self = 1;
            if (dw_next[r] >= 0) R[r].w2_self = 1;
        }
        ri0 = (int64_t)rt.size();
        for (int64_t t = rstep[0]; t < rstep[1]; ++t) {
            const CleTask tk = rt[t];
            if (tk.kind == kRangeW1 && R[tk.rel].w1_self) continue;
            if (tk.kind == kRangeW2Contig && R[tk.rel].w2_self) continue;
            rt.push_back(tk);
        }
        ri1 = (int64_t)rt.size();
    }
    for (int32_t k = 0; k < steps; ++k) {
        for (int32_t r = 0; r < n_rel; ++r) {
            if (step_of[r] != k) continue;
            if (!fused) {
                w1_range_tasks(r);
                w2_range_tasks(r);
            }
            apply_tasks(r, at);
        }
        // The step's slowest tasks first (its span is the last task's end): W2 row
        // tiles (strided columns, their loads and stores a row at a time), the
        // per-channel vectors (each a chain of dependent loads), then the depthwise
        // pairs, W1 rows and contiguous W2 channels (profiles/r03/cle_tl_*.log: tile
        // tasks started up to 10 us into a step and ran ~10 us)
        auto prio = [](int32_t kind) {
            switch (kind) {
                case kApplyW2Tile: return 0;
                case kApplyChannels: return 1;
                case kApplyDwBoth: return 2;
                case kApplyW1: return 3;
                default: return 4;
            }
        };
        std::stable_sort(at.begin() + astep.back(), at.end(),
                         [&](const CleTask& x, const CleTask& y) { return prio(x.kind) < prio(y.kind); });
        if (!fused) rstep.push_back((int64_t)rt.size());
        astep.push_back((int64_t)at.size());
    }
    const double tp3 = now_us();
    // metric chunks: torch.mean = sum / n; the sum is two_pass_reduction over
    // min(threads, ceil(n / 32768)) equal chunks when n >= 32768 (serial below)
    std::vector<CleLayer> layers(n_targets);
    std::vector<CleChunk> chunks;
    std::vector<CleUnit> units;
    std::vector<int64_t> b1off;
    int64_t nb1_total = 0;
    for (int32_t l = 0; l < n_targets; ++l) {
        const int64_t n = target_n[l];
        if (!targets[l] || n <= 0) return DFQ_ERR_INVALID;
        layers[l] = CleLayer{nullptr, nullptr, n, 1};   // the tensor and its snapshot: bound per plan
        int64_t nt = 1;
        if (n >= 32768 && ref_threads > 1) nt = std::min<int64_t>(ref_threads, ceil_div(n, (int64_t)32768));
        layers[l].nt = nt;
        const int64_t chunk = ceil_div(n, nt);
        for (int64_t t = 0; t < nt; ++t) {
            const int64_t b = t * chunk;
            if (b >= n) break;
            const int64_t len = std::min<int64_t>(n, b + chunk) - b;
            const int64_t sz = len / 32;
            if (aten_ceil_log2(sz) / 4 > 4) return DFQ_ERR_UNSUPPORTED;   // > 16M / chunk
            const int32_t ci = (int32_t)chunks.size();
            chunks.push_back(CleChunk{l, (int32_t)t, b, len});
            const int64_t nb1 = sz / 256;
            b1off.push_back(32 * nb1_total);   // float offset of this chunk's [nb1][32] level-1 sums
            nb1_total += nb1;
            if (len >= 8)
                for (int64_t g = 0; g <= nb1; ++g) units.push_back(CleUnit{ci, (int32_t)g});
        }
    }
    const double tp4 = now_us();
    // Placement of the metric tiles and the next iteration's range tasks.  An
    // iteration group has nlaunch launches: the steps' rescale launches (and, in the
    // round-4 schedule, one tiles-only launch after them).  Every tile unit and
    // range task gets an OFFSET in [0, 2 nlaunch): offset k < nlaunch runs in
    // launch k of its own iteration's group, offset nlaunch + k in launch k of the
    // next group.  A tensor's tiles and ranges must run after its last rescale of
    // iteration i and before its first rescale of iteration i + 1: offsets
    // [last + 1, nlaunch + first - 1].  Resets of a relation's range words go after
    // that relation's own step and before the next accumulation.
    // Lagged schedule (nlaunch = steps: no tiles-only launch): the tiles of one
    // iteration sit in a band of nlaunch - 1 offsets and the stop rule runs as a
    // block of its own one offset after the band (it reads the chunk sums the
    // tiles' last arrivals left, after a launch boundary): iteration i's stop rule
    // runs beside the rescale tasks of iteration i + 1 instead of after a serial
    // tile -> chunk-combine -> stop-rule chain in a launch of its own, and every
    // tile of iteration i + 1 starts after it (cle_loop_step_kernel).
    // MobileNetV2: 4 -> 3 launches per iteration.  Needs the fused range schedule
    // and no tiny chunks (the stop rule takes their sums from the live weights);
    // where no band fits (ResNet-50: a tensor rescaled at both steps) or without
    // lag (DFQ_CLE_LAG=0, diagnostics): the round-4 schedule, everything in the
    // tiles-only launch and the stop rule at the last tile arrival.
    const bool tiny = std::any_of(chunks.begin(), chunks.end(), [](const CleChunk& c) { return c.len < 8; });
    const bool have_tiles = std::any_of(chunks.begin(), chunks.end(), [](const CleChunk& c) { return c.len >= 8; });
    bool lag_ok = fused && !tiny && have_tiles && steps > 0;
    if (const char* e = ab_env("DFQ_CLE_LAG")) lag_ok = lag_ok && e[0] != '0';
    int32_t band_force = -1;   // diagnostics A/B: the tiles' band start
    // diagnostics A/B: the lagged schedule's stop rule at the last tile arrival
    // (band of nlaunch offsets) instead of as a block of its own after the band
    const bool stop_arrival = [] {
        const char* e = ab_env("DFQ_CLE_STOP");
        return e && e[0] == 'a';
    }();
    if (const char* e = ab_env("DFQ_CLE_BAND")) band_force = atoi(e);
    // (first, last) step of every tensor the relations rescale: a linear table (a few
    // hundred tensors at most), looked up once per relation and target layer
    std::vector<const float*> sp_w;
    std::vector<std::pair<int32_t, int32_t>> sp_v;
    auto sp_find = [&](const float* w) -> int32_t {
        for (size_t i = 0; i < sp_w.size(); ++i)
            if (sp_w[i] == w) return (int32_t)i;
        return -1;
    };
    std::vector<int32_t> rel_t1(n_rel), rel_t2(n_rel);
    for (int32_t r = 0; r < n_rel; ++r)
        for (int side = 0; side < 2; ++side) {
            const float* w = side ? R[r].w2 : R[r].w1;
            int32_t i = sp_find(w);
            if (i < 0) {
                i = (int32_t)sp_w.size();
                sp_w.push_back(w);
                sp_v.push_back({step_of[r], step_of[r]});
            } else {
                sp_v[i] = {std::min(sp_v[i].first, step_of[r]), std::max(sp_v[i].second, step_of[r])};
            }
            (side ? rel_t2 : rel_t1)[r] = i;
        }
    std::vector<int32_t> lay_t(n_targets);
    for (int32_t l = 0; l < n_targets; ++l) lay_t[l] = lag_ok ? sp_find(targets[l]) : -1;
    std::vector<int32_t> layer_off(n_targets, 0);
    int32_t stop_off = -1;   // lagged: the stop rule's own block at this offset (else: the last tile arrival)
    std::vector<int32_t> rt_off;   // per task of [ri0, ri1)
    int32_t nlaunch = steps + 1;
    bool lagged = false;
    // placement (lagged schedule only): loads in bytes per launch position of a
    // group -- the steps' rescale traffic, then greedy by size: each range task and
    // each layer's tiles to the least-loaded admissible offset
    int32_t lag_max = -1;   // the placement's largest tile offset
    auto place = [&](int32_t nl_) -> bool {
        auto window = [&](int32_t ti) -> std::pair<int32_t, int32_t> {   // [lo, hi] offsets (untouched: anywhere)
            if (ti < 0) return {0, 2 * nl_ - 1};
            return {sp_v[ti].second + 1, std::min(2 * nl_ - 1, nl_ + sp_v[ti].first - 1)};
        };
        std::vector<double> base_load(nl_, 0.0);
        for (int32_t k = 0; k < steps && k < nl_; ++k)
            for (int64_t t = astep[k]; t < astep[k + 1]; ++t) {
                const CleTask& tk = at[t];
                const CleRel& q = R[tk.rel];
                double n = 0;
                if (tk.kind == kApplyW1) n = (double)(tk.b - tk.a) * q.len1;
                else if (tk.kind == kApplyW2Tile) n = (double)(tk.b - tk.a) * (tk.c1 - tk.c0) * q.khw2;
                else if (tk.kind != kApplyChannels) n = (double)(tk.b - tk.a) * q.o2g * q.khw2;
                base_load[k] += 8.0 * n;
            }
        // range tasks: their own windows and bytes
        const int64_t nr = ri1 - ri0;
        std::vector<std::pair<int32_t, int32_t>> rwin((size_t)nr);
        std::vector<double> rbytes((size_t)nr);
        for (int64_t x = 0; x < nr; ++x) {
            const CleTask& tk = rt[ri0 + x];
            const CleRel& q = R[tk.rel];
            std::pair<int32_t, int32_t> w;
            switch (tk.kind) {
                case kRangeW1:
                    w = window(rel_t1[tk.rel]);
                    rbytes[x] = 4.0 * (tk.b - tk.a) * q.len1;
                    break;
                case kRangeW2Contig:
                    w = window(rel_t2[tk.rel]);
                    rbytes[x] = 4.0 * (tk.b - tk.a) * q.o2g * q.khw2;
                    break;
                case kRangeW2Tile:
                    w = window(rel_t2[tk.rel]);
                    rbytes[x] = 4.0 * (tk.b - tk.a) * (tk.c1 - tk.c0) * q.khw2;
                    break;
                case kRangeReset:   // after the consumer step, before the next accumulation (>= nl_ + last + 1)
                    w = {step_of[tk.rel] + 1, std::min(2 * nl_ - 1, nl_ + sp_v[rel_t2[tk.rel]].second)};
                    rbytes[x] = 64.0;
                    break;
                default:            // kRangeResetW1: after the consumer step, before the producer's step two groups on
                    w = {step_of[tk.rel] + 1, 2 * nl_ - 1};
                    rbytes[x] = 64.0;
            }
            if (w.first > w.second) return false;
            rwin[x] = w;
        }
        // tiles: a band [B0, B0 + nl_ - 2] meeting every layer's window; the stop
        // rule one offset after the band's last used offset
        int32_t maxlo = 0, minhi = 2 * nl_ - 1;
        std::vector<std::pair<int32_t, int32_t>> lwin(n_targets);
        for (int32_t l = 0; l < n_targets; ++l) {
            lwin[l] = window(lay_t[l]);
            if (lwin[l].first > lwin[l].second) return false;
            maxlo = std::max(maxlo, lwin[l].first);
            minhi = std::min(minhi, lwin[l].second);
        }
        const int32_t bw = stop_arrival ? nl_ : nl_ - 1;   // band width
        if (bw < 1) return false;
        const int32_t b_lo = std::max(0, maxlo - bw + 1), b_hi = std::min(minhi, 2 * nl_ - 1 - bw);
        if (b_lo > b_hi) return false;
        std::vector<int32_t> lord(n_targets);
        std::iota(lord.begin(), lord.end(), 0);
        std::sort(lord.begin(), lord.end(),
                  [&](int32_t x, int32_t y) { return target_n[x] != target_n[y] ? target_n[x] > target_n[y] : x < y; });
        std::vector<int64_t> rord((size_t)nr);
        std::iota(rord.begin(), rord.end(), 0);
        std::sort(rord.begin(), rord.end(),
                  [&](int64_t x, int64_t y) { return rbytes[x] != rbytes[y] ? rbytes[x] > rbytes[y] : x < y; });
        double best = 1e300;
        std::vector<int32_t> roff((size_t)nr), loff(n_targets);
        for (int32_t B0 = b_lo; B0 <= b_hi; ++B0) {
            if (band_force >= 0 && B0 != band_force && band_force >= b_lo && band_force <= b_hi) continue;
            std::vector<double> load = base_load;
            auto pick = [&](int32_t lo, int32_t hi, double bytes) {
                int32_t bo = lo;
                for (int32_t o = lo; o <= hi; ++o)
                    if (load[o % nl_] < load[bo % nl_]) bo = o;
                load[bo % nl_] += bytes;
                return bo;
            };
            for (int64_t x : rord) roff[x] = pick(rwin[x].first, rwin[x].second, rbytes[x]);
            int32_t maxoff = 0;
            for (int32_t l : lord) {
                loff[l] = pick(std::max(lwin[l].first, B0), std::min(lwin[l].second, B0 + bw - 1), 12.0 * target_n[l]);
                maxoff = std::max(maxoff, loff[l]);
            }
            if (!stop_arrival && maxoff + 1 > 2 * nl_ - 1) continue;
            double cost = *std::max_element(load.begin(), load.end());
            if (cost < best) {
                best = cost;
                layer_off = loff;
                rt_off = roff;
                stop_off = stop_arrival ? -1 : maxoff + 1;
                lag_max = maxoff;
            }
        }
        return best < 1e300;
    };
    if (lag_ok && place(steps) && (stop_arrival ? lag_max >= steps : stop_off >= steps)) {
        nlaunch = steps;
        lagged = true;
    } else {   // everything in the tiles-only launch after the steps (offset steps), the stop rule at the last arrival
        nlaunch = steps + 1;
        stop_off = -1;
        layer_off.assign(n_targets, steps);
        rt_off.assign((size_t)(ri1 - ri0), steps);
    }
    std::vector<int64_t> uoffs(2 * nlaunch + 1, 0), roffs(2 * nlaunch + 1, 0);
    {
        std::vector<std::vector<CleUnit>> ub(2 * nlaunch);
        for (const CleUnit& u : units) ub[layer_off[chunks[u.chunk].layer]].push_back(u);
        units.clear();
        for (int32_t k = 0; k < 2 * nlaunch; ++k) {
            uoffs[k] = (int64_t)units.size();
            units.insert(units.end(), ub[k].begin(), ub[k].end());
        }
        uoffs[2 * nlaunch] = (int64_t)units.size();
        if (fused) {   // (the unfused schedule's range tasks are per step: rstep; roffs stay empty)
            std::vector<std::vector<CleTask>> rb(2 * nlaunch);
            for (int64_t t = ri0; t < ri1; ++t) rb[rt_off[t - ri0]].push_back(rt[t]);
            rt.resize(ri0);
            for (int32_t k = 0; k < 2 * nlaunch; ++k) {
                roffs[k] = (int64_t)rt.size();
                rt.insert(rt.end(), rb[k].begin(), rb[k].end());
            }
            roffs[2 * nlaunch] = (int64_t)rt.size();
            ri1 = (int64_t)rt.size();
        }
    }
    S.R = std::move(R);
    S.M = M;
    S.chains = chains;
    S.steps = steps;
    S.fused = fused;
    S.rt = std::move(rt);
    S.at = std::move(at);
    S.rstep = std::move(rstep);
    S.astep = std::move(astep);
    S.ri0 = ri0;
    S.ri1 = ri1;
    S.layers = std::move(layers);
    S.chunks = std::move(chunks);
    S.units = std::move(units);
    S.b1off = std::move(b1off);
    S.nb1_total = nb1_total;
    S.uoffs = std::move(uoffs);
    S.roffs = std::move(roffs);
    S.nlaunch = nlaunch;
    S.stop_off = stop_off;
    S.lagged = lagged;
    S.id = ++g_struct_ids;
    for (const CleTask& tk : S.at) {
        const CleRel& q = S.R[tk.rel];
        const int64_t n = tk.b - tk.a;
        switch (tk.kind) {
            case kApplyW1: S.bytes_rescale += 8 * n * q.len1; break;
            case kApplyW2Contig:
            case kApplyDwBoth: S.bytes_rescale += 8 * n * q.o2g * q.khw2; break;
            case kApplyW2Tile: S.bytes_rescale += 8 * n * (tk.c1 - tk.c0) * q.khw2; break;
            default:
                S.bytes_rescale += 8 * n * ((q.b1 ? 1 : 0) + (q.bnw ? 1 : 0) + (q.bnb ? 1 : 0) + (q.sacc ? 1 : 0));
        }
    }
    for (int32_t l = 0; l < n_targets; ++l) S.bytes_metric += 12 * target_n[l];
    {
        const int64_t r0 = fused ? S.ri0 : 0, r1 = fused ? S.ri1 : (int64_t)S.rt.size();
        for (int64_t t = r0; t < r1; ++t) {
            const CleTask& tk = S.rt[t];
            const CleRel& q = S.R[tk.rel];
            const int64_t n = tk.b - tk.a;
            if (tk.kind == kRangeW1) S.bytes_range += 4 * n * q.len1;
            else if (tk.kind == kRangeW2Contig) S.bytes_range += 4 * n * q.o2g * q.khw2;
            else if (tk.kind == kRangeW2Tile) S.bytes_range += 4 * n * (tk.c1 - tk.c0) * q.khw2;
        }
    }
    const double tp5 = now_us();
    S.t_chains = tp2 - tp1;
    S.t_tasks = tp3 - tp2;
    S.t_chunks = tp4 - tp3;
    S.t_place = tp5 - tp4;
    return DFQ_OK;
}

// The structure key: shapes, flags and the identity pattern of every tensor
// address (which relation / target slots share a tensor), the metric's thread
// count and the diagnostics library's schedule switches.  Two calls with equal
// keys get equal structures.
static std::vector<int64_t> cle_structure_key(const std::vector<CleRel>& R, int64_t M, float* const* targets,
                                              const int64_t* target_n, int32_t n_targets, int32_t ref_threads) {
    std::vector<std::pair<uintptr_t, int32_t>> ps;
    ps.reserve(5 * R.size() + n_targets);
    for (const CleRel& c : R)
        for (const void* q : {(const void*)c.w1, (const void*)c.w2, (const void*)c.b1, (const void*)c.bnw,
                              (const void*)c.bnb})
            ps.push_back({reinterpret_cast<uintptr_t>(q), (int32_t)ps.size()});
    for (int32_t l = 0; l < n_targets; ++l) ps.push_back({reinterpret_cast<uintptr_t>(targets[l]), (int32_t)ps.size()});
    std::vector<int32_t> id(ps.size());
    std::vector<std::pair<uintptr_t, int32_t>> srt = ps;
    std::sort(srt.begin(), srt.end());
    for (size_t i = 0; i < srt.size();) {   // every slot -> the first slot holding the same address
        size_t j = i;
        while (j < srt.size() && srt[j].first == srt[i].first) ++j;
        for (size_t k = i; k < j; ++k) id[srt[k].second] = srt[i].first ? srt[i].second : -1;
        i = j;
    }
    std::vector<int64_t> key;
    key.reserve(16 * R.size() + 2 * n_targets + 16);
    key.push_back((int64_t)R.size());
    key.push_back(M);
    key.push_back(n_targets);
    key.push_back(ref_threads);
    for (const char* sw : {"DFQ_CLE_FUSED", "DFQ_CLE_LAG", "DFQ_CLE_BAND", "DFQ_CLE_STOP",
                           "DFQ_CLE_W1_ROWS", "DFQ_CLE_DW_ROWS"}) {   // diagnostics library only
        const char* v = ab_env(sw);
        int64_t h = v ? 1 : 0;
        for (int k = 0; v && v[k] && k < 8; ++k) h = h * 131 + (unsigned char)v[k];
        key.push_back(h);
    }
    size_t q = 0;
    for (const CleRel& c : R) {
        key.insert(key.end(), {c.c1, c.len1, c.o2, c.i2, c.khw2, (int64_t)c.sacc_init, (int64_t)c.vec1, (int64_t)c.vec2,
                               (int64_t)(c.sacc != nullptr)});
        for (int k = 0; k < 5; ++k) key.push_back(id[q++]);
    }
    for (int32_t l = 0; l < n_targets; ++l) {
        key.push_back(target_n[l]);
        key.push_back(id[q++]);
    }
    return key;
}

// The relations' descriptors as the device's records: shapes checked as
// dfq_cle_relation; each relation's [W1 | W2] range words at moff (M in all).
static int cle_rels_from_desc(const dfq_cle_rel* rels, int32_t n_rel, std::vector<CleRel>& R, int64_t& M) {
    R.assign(n_rel, CleRel{});
    M = 0;
    for (int32_t r = 0; r < n_rel; ++r) {
        const dfq_cle_rel& d = rels[r];
        if (!d.w1 || !d.w2 || !d.b1 || d.c1 <= 0 || d.len1 <= 0 || d.o2 <= 0 || d.i2 <= 0 || d.khw2 <= 0)
            return DFQ_ERR_INVALID;
        int64_t groups = 1;
        if (d.c1 != d.i2) {
            groups = d.c1 / d.i2;
            if (groups <= 0 || groups * d.i2 != d.c1) return DFQ_ERR_SHAPE;
        }
        if (d.o2 % groups != 0) return DFQ_ERR_SHAPE;
        CleRel c{};
        c.w1 = d.w1; c.w2 = d.w2; c.b1 = d.b1; c.bnw = d.bn_w; c.bnb = d.bn_b; c.sacc = d.s_acc;
        c.c1 = d.c1; c.len1 = d.len1; c.o2 = d.o2; c.i2 = d.i2; c.khw2 = d.khw2; c.o2g = d.o2 / groups;
        c.moff = M;
        c.sacc_init = d.s_acc_init;
        c.vec1 = (d.len1 % 4 == 0 && reinterpret_cast<uintptr_t>(d.w1) % 16 == 0) ? 1 : 0;
        c.vec2 = (d.i2 == 1 && (c.o2g * d.khw2) % 4 == 0 && reinterpret_cast<uintptr_t>(d.w2) % 16 == 0) ? 1 : 0;
        c.fuse_next = -1;
        c.dw_prev = -1;
        c.w1_self = 0;
        c.w2_self = 0;
        M += 2 * d.c1;
        R[r] = c;
    }
    return DFQ_OK;
}

static std::mutex g_struct_mu;
static std::list<std::pair<std::vector<int64_t>, std::shared_ptr<const CleStructure>>> g_struct_cache;
constexpr size_t kStructCacheCap = 8;

extern "C" int dfq_cle_plan_create(const dfq_cle_rel* rels, int32_t n_rel, float* const* targets,
                                   const int64_t* target_n, int32_t n_targets, double s_min, double s_max,
                                   int32_t is_signed, float eps, int32_t ref_threads, void* ws, int64_t ws_bytes,
                                   dfq_cle_plan** out) {
    if (!out || n_rel < 0 || n_targets < 0 || (n_rel > 0 && !rels) || (n_targets > 0 && (!targets || !target_n)))
        return DFQ_ERR_INVALID;
    const double tc0 = now_us();
    const int64_t need_ws = dfq_cle_plan_ws_bytes(target_n, n_targets);
    if (need_ws < 0) return DFQ_ERR_INVALID;
    if (ws && (ws_bytes < need_ws || reinterpret_cast<uintptr_t>(ws) % 256 != 0)) return DFQ_ERR_INVALID;
    *out = nullptr;
    std::vector<CleRel> R;
    int64_t M = 0;
    if (const int rc = cle_rels_from_desc(rels, n_rel, R, M); rc != DFQ_OK) return rc;
    const double tp1 = now_us();
    // the structure (chains, tasks, chunks, placement) from the cache when a plan of
    // the same shapes and tensor-sharing pattern was built before
    std::shared_ptr<const CleStructure> S;
    bool cached = false;
    const std::vector<int64_t> key = cle_structure_key(R, M, targets, target_n, n_targets, ref_threads);
    {
        std::lock_guard<std::mutex> lock(g_struct_mu);
        for (auto it = g_struct_cache.begin(); it != g_struct_cache.end(); ++it)
            if (it->first == key) {
                S = it->second;
                g_struct_cache.splice(g_struct_cache.begin(), g_struct_cache, it);   // most recent first
                cached = true;
                break;
            }
    }
    if (!S) {
        auto built = std::make_shared<CleStructure>();
        const int rc = cle_build_structure(R, M, n_rel, targets, target_n, n_targets, ref_threads, *built);
        if (rc != DFQ_OK) return rc;
        S = built;
        std::lock_guard<std::mutex> lock(g_struct_mu);
        g_struct_cache.emplace_front(key, S);
        if (g_struct_cache.size() > kStructCacheCap) g_struct_cache.pop_back();
    }
    const double tp5 = now_us();
    // this plan's addresses into its copy of the relations and layers
    std::vector<CleRel> Rb = S->R;
    for (int32_t r = 0; r < n_rel; ++r) {
        Rb[r].w1 = R[r].w1; Rb[r].w2 = R[r].w2; Rb[r].b1 = R[r].b1;
        Rb[r].bnw = R[r].bnw; Rb[r].bnb = R[r].bnb; Rb[r].sacc = R[r].sacc;
    }
    dfq_cle_plan* p = new (std::nothrow) dfq_cle_plan();
    if (!p) return DFQ_ERR_NOMEM;
    std::vector<CleLayer> layers = S->layers;
    {
        char* snap_base = static_cast<char*>(ws);
        if (!snap_base && need_ws > 0) {   // no caller workspace: the plan owns its snapshots
            hipError_t e = hipMalloc(&p->d_snap_owned, need_ws);
            if (e != hipSuccess) { set_last_hip_error(e); cle_plan_free(p); return DFQ_ERR_HIP; }
            snap_base = static_cast<char*>(p->d_snap_owned);
        }
        int64_t snap_off = 0;
        for (int32_t l = 0; l < n_targets; ++l) {
            layers[l].w = targets[l];
            layers[l].snap = reinterpret_cast<float*>(snap_base + snap_off);
            snap_off += snap_bytes(target_n[l]);
        }
    }
    const std::vector<CleTask>& rt = S->rt;
    const std::vector<CleTask>& at = S->at;
    const std::vector<CleChunk>& chunks = S->chunks;
    const std::vector<CleUnit>& units = S->units;
    const std::vector<int64_t>& b1off = S->b1off;
    const std::vector<int64_t>& rstep = S->rstep;
    const std::vector<int64_t>& astep = S->astep;
    const int64_t nb1_total = S->nb1_total, ri0 = S->ri0, ri1 = S->ri1;
    const int32_t steps = S->steps, chains = S->chains, nlaunch = S->nlaunch, stop_off = S->stop_off;
    const bool fused = S->fused, lagged = S->lagged;
    if (cle_timing() && !cached) {   // the schedule: per offset, tile units and range tasks
        fprintf(stderr, "DFQ_CLE_TIMING plan: steps %d nlaunch %d lagged %d stop %d; offsets (units/ranges):", steps,
                nlaunch, (int)lagged, stop_off);
        for (int32_t k = 0; k < 2 * nlaunch; ++k)
            fprintf(stderr, " %d:%lld/%lld", k, (long long)(S->uoffs[k + 1] - S->uoffs[k]),
                    (long long)(S->roffs[k + 1] - S->roffs[k]));
        fprintf(stderr, "; rescale tasks per step:");
        for (int32_t k = 0; k < steps; ++k) fprintf(stderr, " %lld", (long long)(astep[k + 1] - astep[k]));
        fprintf(stderr, "\n");
    }
    (void)hipGetDevice(&p->dev);
    p->uoffs = S->uoffs;
    p->roffs = S->roffs;
    p->nlaunch = nlaunch;
    p->lagged = lagged;
    p->stop_off = stop_off;
    p->nunits = (int64_t)units.size();
    p->M = M;
    p->nl = n_targets;
    p->nchunks = (int64_t)chunks.size();
    p->chains = chains;
    p->steps = steps;
    p->fused = fused;
    p->rstep = rstep;
    p->astep = astep;
    p->step_pos.assign(std::max<int32_t>(steps, 1), 0);
    for (int32_t k = 0; k < steps; ++k)
        for (int64_t t = astep[k]; t < astep[k + 1]; ++t)
            if (at[t].kind == kApplyW2Tile && Rb[at[t].rel].khw2 > 1) p->step_pos[k] = 1;
    p->ri0 = ri0;
    p->ri1 = ri1;
    p->bytes[0] = S->bytes_rescale;
    p->bytes[1] = S->bytes_metric;
    p->bytes[2] = S->bytes_range;
#ifdef DFQ_DIAGNOSTICS
    if (ab_env("DFQ_CLE_TL")) {   // for the timeline report (copies cost ~0.2 ms: only when asked)
        p->h_rels = R;
        p->h_atasks = at;
    }
#endif
    p->smin = s_min; p->smax = s_max; p->is_signed = is_signed; p->eps = eps;
    hipError_t e;
    auto fail = [&](hipError_t err) { set_last_hip_error(err); cle_plan_free(p); return DFQ_ERR_HIP; };
    // every table in one allocation; the host-built ones in one copy
    TableLayout T;
    const int64_t o_rels = T.add<CleRel>((int64_t)R.size());
    const int64_t o_rt = T.add<CleTask>((int64_t)rt.size());
    const int64_t o_at = T.add<CleTask>((int64_t)at.size());
    const int64_t o_layers = T.add<CleLayer>((int64_t)layers.size());
    const int64_t o_chunks = T.add<CleChunk>((int64_t)chunks.size());
    const int64_t o_units = T.add<CleUnit>((int64_t)units.size());
    const int64_t o_b1off = T.add<int64_t>((int64_t)b1off.size());
    p->slots = std::max<int32_t>(ref_threads, 1);
    // the chunk sums [layers][slots] (zeroed per run), then per layer {(float)n,
    // nt == 1}: the stop rule stages both in one pass of loads
    const int64_t o_part = T.add<float>((int64_t)(p->slots + 2) * n_targets);
    const int64_t host_bytes = T.total;   // the tables above are built on the host (and the group tables)
    const int64_t o_b1 = T.add<float>(32 * nb1_total);
    const int64_t o_tail = T.add<float>(kCleTailWords * (int64_t)chunks.size());
    const int64_t o_rng = T.add<uint32_t>(4 * M);
    const int64_t o_means = T.add<double>(n_targets);
    const int64_t o_state = T.add<CleState>(1);
    const int64_t o_hist = T.add<double>(kCleHistCap);
    const int64_t o_cnt = T.add<uint32_t>((int64_t)chunks.size() + 1);
    const int64_t o_vsave = T.add<float>(lagged ? 2 * M : 0);
    const int64_t o_vtag = T.add<int32_t>(lagged ? (int64_t)at.size() : 0);
    const double tm0 = now_us();
    char* base = nullptr;
    char* hblob = nullptr;
    CleDeviceCtx& ctx = cle_device_ctx(p->dev);
    e = hipSuccess;   // a busy pool leaves it untouched: the private path follows
    {   // the pool
        std::lock_guard<std::mutex> lock(ctx.mu);
        if (!ctx.pool_busy && (e = cle_ctx_ready(ctx)) == hipSuccess &&
            (e = hipEventSynchronize(ctx.pool_ev)) == hipSuccess) {
            if (ctx.pool_cap < (size_t)T.total) {
                (void)hipFree(ctx.d_pool);
                ctx.d_pool = nullptr;
                ctx.pool_cap = 0;
                ctx.pool_struct = 0;
                const size_t cap = (size_t)T.total + (size_t)T.total / 2;
                if ((e = hipMalloc(&ctx.d_pool, cap)) == hipSuccess) ctx.pool_cap = cap;
            }
            if (e == hipSuccess && ctx.hpool_cap < (size_t)host_bytes) {
                (void)hipHostFree(ctx.h_pool);
                ctx.h_pool = nullptr;
                ctx.hpool_cap = 0;
                const size_t cap = (size_t)host_bytes + (size_t)host_bytes / 2;
                if ((e = hipHostMalloc(&ctx.h_pool, cap, hipHostMallocDefault)) == hipSuccess) ctx.hpool_cap = cap;
            }
            if (e == hipSuccess) {
                ctx.pool_busy = true;
                p->pooled = true;
                base = ctx.d_pool;
                hblob = ctx.h_pool;
            }
        }
        if (e != hipSuccess) return fail(e);
    }
    std::vector<char> blob;
    // The pool already holding this structure's address-free tables (tasks,
    // chunks, units, level-1 offsets, layer sizes: a plan of the same structure
    // came before, and the tables are read-only on the device): only the records
    // that carry addresses -- relations and layers -- are written and uploaded.
    const bool resident = p->pooled && ctx.pool_struct == S->id;
    if (!p->pooled) {
        if ((e = hipMalloc(&p->d_tables, T.total)) != hipSuccess) return fail(e);
        base = static_cast<char*>(p->d_tables);
        blob.assign(host_bytes, 0);
        hblob = blob.data();
    } else if (!resident) {
        std::memset(hblob, 0, host_bytes);
    }
    const double tm1 = now_us();
    auto put = [&](int64_t off, const auto& v) {
        if (!v.empty()) std::memcpy(hblob + off, v.data(), sizeof(v[0]) * v.size());
    };
    put(o_rels, Rb);
    put(o_layers, layers);
    if (!resident) {
        put(o_rt, rt); put(o_at, at); put(o_chunks, chunks); put(o_units, units); put(o_b1off, b1off);
        float* lm = reinterpret_cast<float*>(hblob + o_part) + (int64_t)p->slots * n_targets;
        for (int64_t l = 0; l < n_targets; ++l) {
            lm[2 * l] = (float)layers[l].n;
            lm[2 * l + 1] = layers[l].nt == 1 ? 1.f : 0.f;
        }
    }
    if (p->pooled) {   // async on the loop stream, which every launch of the plan uses
        if (resident) {
            const size_t nr = sizeof(CleRel) * Rb.size(), nly = sizeof(CleLayer) * layers.size();
            if (nr && (e = hipMemcpyAsync(base + o_rels, hblob + o_rels, nr, hipMemcpyHostToDevice, ctx.st)) != hipSuccess)
                return fail(e);
            if (nly && (e = hipMemcpyAsync(base + o_layers, hblob + o_layers, nly, hipMemcpyHostToDevice, ctx.st)) !=
                           hipSuccess)
                return fail(e);
        } else if ((e = hipMemcpyAsync(base, hblob, host_bytes, hipMemcpyHostToDevice, ctx.st)) != hipSuccess) {
            return fail(e);
        }
        if ((e = hipEventRecord(ctx.pool_ev, ctx.st)) != hipSuccess) return fail(e);
        ctx.pool_struct = S->id;
    } else if ((e = hipMemcpy(base, hblob, host_bytes, hipMemcpyHostToDevice)) != hipSuccess) {
        return fail(e);
    }
    if (cle_timing())
        fprintf(stderr, "DFQ_CLE_TIMING create: plan %.1f us (relations %.1f, structure %s %.1f: chains %.1f, tasks %.1f, "
                "chunks %.1f, placement %.1f), tables %lld B %.1f us, copy %lld B %.1f us\n", tm0 - tc0, tp1 - tc0,
                cached ? "cached" : "built", tp5 - tp1, S->t_chains, S->t_tasks, S->t_chunks, S->t_place,
                (long long)T.total, tm1 - tm0, (long long)host_bytes, now_us() - tm1);
    p->d_rels = reinterpret_cast<CleRel*>(base + o_rels);
    p->d_rtasks = reinterpret_cast<CleTask*>(base + o_rt);
    p->d_atasks = reinterpret_cast<CleTask*>(base + o_at);
    p->d_layers = reinterpret_cast<CleLayer*>(base + o_layers);
    p->d_chunks = reinterpret_cast<CleChunk*>(base + o_chunks);
    p->d_units = reinterpret_cast<CleUnit*>(base + o_units);
    p->d_b1off = reinterpret_cast<int64_t*>(base + o_b1off);
    p->d_b1 = reinterpret_cast<float*>(base + o_b1);
    p->d_tail = reinterpret_cast<float*>(base + o_tail);
    p->d_rng = reinterpret_cast<uint32_t*>(base + o_rng);
    p->d_part = reinterpret_cast<float*>(base + o_part);
    p->d_means = reinterpret_cast<double*>(base + o_means);
    p->d_state = reinterpret_cast<CleState*>(base + o_state);
    p->d_hist = p->d_hist_tables = reinterpret_cast<double*>(base + o_hist);
    p->d_cnt = reinterpret_cast<uint32_t*>(base + o_cnt);
    p->n_at = (int64_t)at.size();
    if (lagged) {
        p->d_vsave = reinterpret_cast<float*>(base + o_vsave);
        p->d_vtag = reinterpret_cast<int32_t*>(base + o_vtag);
    }
    for (const auto& c : chunks) p->nbig += c.len >= 8 ? 1 : 0;
    *out = p;
    return DFQ_OK;
}

// Iteration group g's launches on stream s: the rescale steps of iteration g
// (g < max_iters), the tiles and ranges of iteration g placed in this group and
// those of iteration g - 1 placed in the next group (cle_loop_step_kernel).
// Groups 0 .. max_iters are enqueued (the last only finishes iteration
// max_iters - 1).
static int cle_enqueue_iteration(dfq_cle_plan* p, hipStream_t s, int32_t g, int32_t max_iters) {
    // grid caps: 2,048 / 4,096 blocks (caps of 128-1,024 measured 4-150 % slower on MobileNetV2)
    // step / tile grid caps (A/B: DFQ_CLE_STEP_GRID / DFQ_CLE_TILE_GRID, diagnostics library;
    // read per call, not cached: cle_ab.py switches them between runs of one process)
    const int64_t kStepGrid = [] {
        const char* e = ab_env("DFQ_CLE_STEP_GRID");
        return e && *e ? std::max<int64_t>(1, atoll(e)) : int64_t(2048);
    }();
    const int64_t kTileGrid = [] {
        const char* e = ab_env("DFQ_CLE_TILE_GRID");
        return e && *e ? std::max<int64_t>(1, atoll(e)) : int64_t(4096);
    }();
    CleFin F{p->d_cnt, p->d_part, p->d_means, p->d_hist, p->nchunks, p->nbig, p->slots, p->nl, 0, p->d_flag,
             p->stop_off < 0 ? 1 : 0};
    const int32_t NL = p->nlaunch;
    const bool run_g = g < max_iters, prev = g >= 1;
    for (int32_t k = 0; k < NL; ++k) {
        const bool step = k < p->steps;
        const int64_t a0 = step ? p->astep[k] : 0, a1 = step ? p->astep[k + 1] : 0;
        if (step && run_g && !p->fused && p->rstep[k + 1] > p->rstep[k]) {   // unfused: this step's ranges first
            hipLaunchKernelGGL(cle_loop_range_kernel, dim3((int)std::min<int64_t>(p->rstep[k + 1] - p->rstep[k], kStepGrid)),
                               dim3(kThreads), 0, s, p->d_rels, p->d_rtasks, p->rstep[k], p->rstep[k + 1], p->d_rng,
                               p->M, p->d_state, 0);
            DFQ_LAUNCH_CHECK();
        }
        const int64_t nab = run_g ? std::min<int64_t>(a1 - a0, kStepGrid) : 0;
        const int64_t uo = p->uoffs[k], nuo = run_g ? p->uoffs[k + 1] - uo : 0;
        const int64_t up = p->uoffs[NL + k], nup = prev ? p->uoffs[NL + k + 1] - up : 0;
        const int64_t ro = p->roffs[k], nro_t = (g + 1 < max_iters) ? p->roffs[k + 1] - ro : 0;
        const int64_t rp = p->roffs[NL + k], nrp_t = (prev && run_g) ? p->roffs[NL + k + 1] - rp : 0;
        int64_t nto = std::min<int64_t>(nuo, kTileGrid);
        const int64_t ntp = std::min<int64_t>(nup, kTileGrid);
        F.last = (k == p->steps) ? 1 : 0;
        if (F.last && run_g && p->nbig == 0) nto = std::max<int64_t>(nto, 1);   // the stop rule's block without tiles
        const int64_t nro = std::min<int64_t>(nro_t, kStepGrid), nrp = std::min<int64_t>(nrp_t, kStepGrid);
        // lagged schedule: the stop rule's block (iteration g's, or g - 1's placed in this group)
        int32_t stop_it = -1;
        if (p->stop_off == k && run_g) stop_it = g;
        else if (p->stop_off == NL + k && prev) stop_it = g - 1;
        const int64_t nblk = nab + (stop_it >= 0 ? cle_stop_blocks(p->nchunks) : 0) + nto + ntp + nro + nrp;
        if (nblk == 0) continue;
        auto kern = (step && p->step_pos[k]) ? cle_loop_step_kernel<true> : cle_loop_step_kernel<false>;
        hipLaunchKernelGGL(kern, dim3((int)nblk), dim3(kThreads), 0, s, p->d_rels, p->d_atasks, a0, a1, nab, p->d_rng,
                           p->M, p->is_signed, p->eps, p->smin, p->smax, p->d_layers, p->d_chunks, p->d_b1off,
                           p->d_units, uo, nuo, nto, up, nup, ntp, p->d_b1, p->d_tail, p->d_rtasks, ro, nro_t, nro, rp,
                           nrp_t, nrp, F, p->d_state, g, p->d_vsave, p->d_vtag, stop_it);
        DFQ_LAUNCH_CHECK();
    }
    return DFQ_OK;
}

// Iterations the host keeps enqueued behind the running one.  Whatever is queued
// when the loop converges runs as no-op launches (every block returns at
// st->done), and a no-op launch of a full-size grid still costs ~9 us
// (profiles/r04/cle_trace_*): round 3's batches of 4 iterations, one batch
// ahead, wasted 16-28 of them per run.
constexpr int32_t kCleAhead = 1;
// How long the loop's host word may stay unchanged before the host asks the
// stream whether it has drained (hipStreamQuery: a marker packet in the queue).
constexpr double kClePollQuietUs = 1000.0;
// How long the caller's stream gate waits for a launched loop at most (it traps
// after that), and how long join waits on the host (then it reports the loop
// lost).  A launched run stops enqueueing iterations at half the gate's limit and
// fails cleanly (cle_run_locked's deadline), so a slowly converging loop on a busy
// GPU ends with an error at join, not with the gate's trap; blocking runs
// (dfq_cle_plan_run) have no deadline and stop at max_iters
// (Cross_layer_equal.DFQ_CLE_MAX_ITERS) with its warning.
static constexpr int kCleGateSeconds = 120;
static constexpr int kCleJoinSeconds = kCleGateSeconds + 30;
static constexpr double kCleLaunchDeadlineUs = 0.5e6 * kCleGateSeconds;
// The context's history buffer for caps above the tables' kCleHistCap slots,
// grown once (a launched run grows it before its caller's stream waits: hipFree
// synchronises the whole device).
static hipError_t cle_hist_ready(CleDeviceCtx& ctx, int32_t max_iters) {
    if (ctx.h_hist_cap < max_iters + 1) {   // the pinned copy-back buffer
        (void)hipHostFree(ctx.h_hist);
        ctx.h_hist = nullptr;
        ctx.h_hist_cap = 0;
        const hipError_t e = hipHostMalloc(&ctx.h_hist, sizeof(double) * (max_iters + 1), hipHostMallocDefault);
        if (e != hipSuccess) return e;
        ctx.h_hist_cap = max_iters + 1;
    }
    if (max_iters + 1 <= kCleHistCap || ctx.hist_cap >= max_iters + 1) return hipSuccess;
    (void)hipFree(ctx.d_hist);
    ctx.d_hist = nullptr;
    ctx.hist_cap = 0;
    const hipError_t e = hipMalloc(&ctx.d_hist, sizeof(double) * (max_iters + 1));
    if (e == hipSuccess) ctx.hist_cap = max_iters + 1;
    return e;
}

// Device -> host copy ordered on the loop stream.  Never a blocking hipMemcpy
// here: that runs on the null stream, which the caller of a launched run may be
// holding behind its wait for this very loop (dfq_cle_plan_launch).
static hipError_t cle_copy_back(void* dst, const void* src, size_t bytes, hipStream_t s) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s);
    return e == hipSuccess ? hipStreamSynchronize(s) : e;
}

// The loop on the device context's stream; the caller holds ctx.mu and has
// ordered the plan's producers before that stream.  iterations / hist: the run's
// result (hist resized to the iterations run).
static int cle_run_locked(dfq_cle_plan* p, CleDeviceCtx& ctx, double threshold, int32_t count, int32_t max_iters,
                          int32_t* iterations, std::vector<double>* hist, double deadline_us = -1.0) {
    DFQ_HIP_CHECK(cle_ctx_ready(ctx));
    p->st = ctx.st;
    p->h_state = ctx.h_state;
    *ctx.h_flag = 0;   // (no kernel of this context's stream is running: the caller holds ctx.mu)
    p->d_flag = ctx.d_flag;
    hipStream_t s = p->st;
    // the history: the tables' slots, or the context's buffer (grown once) for longer caps
    p->d_hist = p->d_hist_tables;
    DFQ_HIP_CHECK(cle_hist_ready(ctx, max_iters));
    if (max_iters + 1 > kCleHistCap) p->d_hist = ctx.d_hist;
    CleState init{};
    init.diff = 1e8;
    init.thr = threshold;
    init.iter_count = 0;
    init.iters = 0;
    init.count = count;
    init.max_iters = max_iters;
    init.done = !((init.diff > threshold) && (0 < count)) || max_iters == 0;
    // the range words, chunk sums, counters, rollback tags, the state and the
    // snapshots in one launch (cle_loop_init_kernel; round 5: six fills, a state
    // upload and the snapshot kernel)
    {
        const int64_t npart = (int64_t)p->slots * std::max(p->nl, 1), ncnt = p->nchunks + 1;
        const int64_t nvtag = p->d_vtag ? p->n_at : 0;
        const int64_t words = std::max({4 * p->M, npart, ncnt, nvtag});
        const int64_t grid = std::min<int64_t>(std::max<int64_t>({p->nunits, ceil_div(words, (int64_t)kThreads), 1}), 4096);
        hipLaunchKernelGGL(cle_loop_init_kernel, dim3((int)grid), dim3(kThreads), 0, s, p->d_layers, p->d_chunks,
                           p->nchunks, p->d_units, p->nunits, p->d_rng, p->M, p->d_part, npart, p->d_cnt, ncnt,
                           p->d_vtag, nvtag, p->d_state, init);
        DFQ_LAUNCH_CHECK();
    }
    // fused schedule: the first iteration's ranges (later ones ride with the tiles)
    if (p->fused && p->rstep[1] > p->rstep[0]) {
        hipLaunchKernelGGL(cle_loop_range_kernel, dim3((int)std::min<int64_t>(p->rstep[1] - p->rstep[0], 2048)),
                           dim3(kThreads), 0, s, p->d_rels, p->d_rtasks, p->rstep[0], p->rstep[1], p->d_rng, p->M,
                           p->d_state, 0);
        DFQ_LAUNCH_CHECK();
    }
#ifdef DFQ_DIAGNOSTICS
    uint64_t* d_tl = nullptr;   // DFQ_CLE_TL: per rescale task timestamps (cle_apply_body)
    uint64_t* d_tl2 = nullptr;  // ... and per block of the last launch
    const int64_t n_at = p->astep.empty() ? 0 : p->astep.back();
    const size_t n_tl2 = 4 * (size_t)(kCleTl2Fin + 1);
    {
        const char* e = ab_env("DFQ_CLE_TILES_FIRST");
        const int tf = e && *e ? (e[0] == '1' ? 1 : 0) : (kCleTilesFirst ? 1 : 0);
        DFQ_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_cle_tiles_first), &tf, sizeof(tf), 0, hipMemcpyHostToDevice, s));
    }
    if (ab_env("DFQ_CLE_TL") && n_at > 0) {
        DFQ_HIP_CHECK(hipMalloc(&d_tl, sizeof(uint64_t) * 4 * n_at));
        DFQ_HIP_CHECK(hipMemsetAsync(d_tl, 0, sizeof(uint64_t) * 4 * n_at, s));
        DFQ_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_cle_tl), &d_tl, sizeof(d_tl), 0, hipMemcpyHostToDevice, s));
        DFQ_HIP_CHECK(hipMalloc(&d_tl2, sizeof(uint64_t) * n_tl2));
        DFQ_HIP_CHECK(hipMemsetAsync(d_tl2, 0, sizeof(uint64_t) * n_tl2, s));
        DFQ_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_cle_tl2), &d_tl2, sizeof(d_tl2), 0, hipMemcpyHostToDevice, s));
        const char* ek = ab_env("DFQ_CLE_TL_STEP");
        const int kk = ek && *ek ? atoi(ek) : -1;
        const int64_t a0v = (kk >= 0 && kk < p->steps) ? p->astep[kk] : -1;
        DFQ_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_cle_tl2_a0), &a0v, sizeof(a0v), 0, hipMemcpyHostToDevice, s));
        DFQ_HIP_CHECK(hipStreamSynchronize(s));
    }
#endif
    // Iteration by iteration, kCleAhead of them queued behind the running one; the
    // stop rule writes (iterations << 1) | done into pinned host memory every
    // iteration (ctx.h_flag, a system-scope store), and this thread polls that word
    // both for the stop and for its pacing -- no copy, event or host round trip
    // sits between two iterations on the loop stream, and at convergence at most
    // kCleAhead iterations are left to run as no-ops.  (Pacing by an event behind
    // each iteration: its marker packet added ~3.7 us before every iteration's
    // first launch, profiles/r04/cle_trace_r04v_*.  Round 3 enqueued batches of 4
    // iterations a batch ahead and read the state back per batch.)
    // hipStreamQuery is NOT polled per iteration: the runtime answers it with a
    // marker packet in the loop's queue, which then sits between two iterations'
    // launches.  It is asked only when the word has not moved for kClePollQuietUs
    // (a kernel error, or everything launched has run).  A drained stream ends the
    // polling only when the word, re-read after the drain, says done, or every
    // allowed iteration was launched, or the word lags the launches (a lost
    // word): a stale read that held back the next enqueue just goes on enqueueing
    // (breaking there ended the loop early as DFQ_OK).
    // deadline_us > 0 (launched runs): past it no more iterations are enqueued and
    // the run fails cleanly, well before the caller's stream gate would trap.
    const double tc1 = now_us();
    int32_t launched = 0;
    bool deadline_hit = false;
    // timed runs (dfq_cle_plan_set_timing, measurement only): one event pair around
    // the loop's launches on its stream (two marker packets per run, none between
    // iterations)
    hipEvent_t tev[2] = {nullptr, nullptr};
    p->loop_ms = -1.f;
    if (p->timed) {
        DFQ_HIP_CHECK(hipEventCreate(&tev[0]));
        DFQ_HIP_CHECK(hipEventCreate(&tev[1]));
        DFQ_HIP_CHECK(hipEventRecord(tev[0], s));
    }
#ifdef DFQ_DIAGNOSTICS
    const char* pd = ab_env("DFQ_CLE_TEST_POLL_DELAY_US");
    const int poll_delay_us = pd ? atoi(pd) : 0;
    const double quiet_us = pd ? 0.0 : kClePollQuietUs;   // the query on every poll, as round 4 did
#else
    const double quiet_us = kClePollQuietUs;
#endif
    if (!init.done) {
        uint32_t last_f = ~0u;
        double t_moved = tc1;
        for (;;) {
            const uint32_t f = __atomic_load_n(ctx.h_flag, __ATOMIC_ACQUIRE);
            if (f & 1u) break;
            const int32_t ran = (int32_t)(f >> 1);   // iterations complete
            if (launched <= max_iters && !deadline_hit && launched - ran <= kCleAhead) {
                const int rc = cle_enqueue_iteration(p, s, launched, max_iters);
                if (rc != DFQ_OK) return rc;
                ++launched;
                continue;
            }
#ifdef DFQ_DIAGNOSTICS
            // test switch: the polling thread descheduled between its load of the word
            // and the stream query below (the stale-word race of ADVICE r04)
            if (poll_delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(poll_delay_us));
#endif
            const double t = now_us();
            if (f != last_f) {
                last_f = f;
                t_moved = t;
            } else if (t - t_moved >= quiet_us) {
                const hipError_t q = hipStreamQuery(s);
                if (q != hipErrorNotReady) {
                    if (q != hipSuccess) break;   // a device error: the synchronize below reports it
                    const uint32_t f2 = __atomic_load_n(ctx.h_flag, __ATOMIC_ACQUIRE);
                    if ((f2 & 1u) || launched > max_iters || deadline_hit || (int32_t)(f2 >> 1) + 1 < launched) break;
                }
                t_moved = t;
            }
            if (deadline_us > 0 && t - tc1 > deadline_us) deadline_hit = true;
            __builtin_ia32_pause();
        }
    }
    if (!init.done && p->lagged) {   // undo a speculative iteration, then release a launched run's caller
        hipLaunchKernelGGL(cle_loop_rollback_kernel, dim3(1024), dim3(kThreads), 0, s, p->d_layers, p->nl, p->d_rels,
                           p->d_atasks, p->n_at, p->d_vsave, p->d_vtag, p->d_state);
        DFQ_LAUNCH_CHECK();
    }
    if (tev[1]) DFQ_HIP_CHECK(hipEventRecord(tev[1], s));
    if (p->d_sig) DFQ_HIP_CHECK(hipStreamWriteValue64(s, p->d_sig, p->gen, 0));
    // the final state and the history (at most the groups launched: iterations run
    // <= groups) come back in the same drain -- one synchronize, not three
    DFQ_HIP_CHECK(hipMemcpyAsync(p->h_state, p->d_state, sizeof(CleState), hipMemcpyDeviceToHost, s));
    const int32_t hn = std::min(launched, max_iters);
    if (hist && hn > 0) DFQ_HIP_CHECK(hipMemcpyAsync(ctx.h_hist, p->d_hist, sizeof(double) * hn, hipMemcpyDeviceToHost, s));
    DFQ_HIP_CHECK(hipStreamSynchronize(s));
    p->launched = launched;
    if (tev[0]) {
        float ms = -1.f;
        if (hipEventElapsedTime(&ms, tev[0], tev[1]) == hipSuccess) p->loop_ms = ms;
        (void)hipEventDestroy(tev[0]);
        (void)hipEventDestroy(tev[1]);
    }
    if (cle_timing())
        fprintf(stderr, "DFQ_CLE_TIMING run: loop %.1f us (%d iterations launched)\n", now_us() - tc1, launched);
#ifdef DFQ_DIAGNOSTICS
    if (d_tl) {   // per step: span, task durations, the slowest tasks
        std::vector<uint64_t> tl(4 * (size_t)n_at);
        DFQ_HIP_CHECK(cle_copy_back(tl.data(), d_tl, sizeof(uint64_t) * tl.size(), s));
        uint64_t* null_tl = nullptr;
        DFQ_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_cle_tl), &null_tl, sizeof(null_tl), 0, hipMemcpyHostToDevice, s));
        std::vector<uint64_t> tl2(n_tl2);
        DFQ_HIP_CHECK(cle_copy_back(tl2.data(), d_tl2, sizeof(uint64_t) * n_tl2, s));
        DFQ_HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_cle_tl2), &null_tl, sizeof(null_tl), 0, hipMemcpyHostToDevice, s));
        DFQ_HIP_CHECK(hipStreamSynchronize(s));
        (void)hipFree(d_tl2);
        {   // the last launch: per role, when blocks started / ended (us after the first start)
            uint64_t t0 = ~0ull;
            for (int b = 0; b < kCleTl2Fin; ++b)
                if (tl2[4 * b]) t0 = std::min(t0, tl2[4 * b]);
            fprintf(stderr, "DFQ_CLE_TL last launch%s:", ab_env("DFQ_CLE_TL_STEP") ? " of DFQ_CLE_TL_STEP" : "");
            for (int role = 1; role <= 3; ++role) {
                std::vector<double> st, en, du;
                for (int b = 0; b < kCleTl2Fin; ++b) {
                    const uint64_t* r = &tl2[4 * b];
                    if (!r[0] || (int)r[2] != role) continue;
                    st.push_back((double)(r[0] - t0) * 0.01);
                    en.push_back((double)(r[1] - t0) * 0.01);
                    du.push_back((double)(r[1] - r[0]) * 0.01);
                }
                if (st.empty()) continue;
                std::sort(st.begin(), st.end());
                std::sort(en.begin(), en.end());
                double m = 0;
                for (double x : du) m += x;
                fprintf(stderr, " [%s: %zu blocks, start p50 %.2f max %.2f, end p50 %.2f max %.2f, dur mean %.2f]",
                        role == 1 ? "tiles" : role == 2 ? "ranges" : "tail tiles", st.size(), st[st.size() / 2], st.back(), en[en.size() / 2],
                        en.back(), m / du.size());
            }
            const uint64_t* f = &tl2[4 * kCleTl2Fin];
            if (f[0] && t0 != ~0ull)
                fprintf(stderr, " [stop rule: %.2f - %.2f, sums staged %.2f, means %.2f]", (double)(f[0] - t0) * 0.01,
                        (double)(f[1] - t0) * 0.01, f[2] ? (double)(f[2] - t0) * 0.01 : -1.0,
                        f[3] ? (double)(f[3] - t0) * 0.01 : -1.0);
            fprintf(stderr, "\n");
        }
        DFQ_HIP_CHECK(hipStreamSynchronize(s));
        (void)hipFree(d_tl);
        for (int32_t k = 0; k < p->steps; ++k) {
            const int64_t a0 = p->astep[k], a1 = p->astep[k + 1];
            uint64_t t_lo = ~0ull, t_hi = 0;
            double sum = 0;
            std::vector<std::pair<double, int64_t>> d;
            for (int64_t t = a0; t < a1; ++t) {
                const uint64_t* r = &tl[4 * t];
                if (!r[0]) continue;
                t_lo = std::min(t_lo, r[0]);
                t_hi = std::max(t_hi, r[1]);
                const double us = (double)(r[1] - r[0]) * 0.01;
                sum += us;
                d.push_back({us, t});
            }
            std::sort(d.rbegin(), d.rend());
            fprintf(stderr, "DFQ_CLE_TL step %d: %lld tasks, span %.2f us, task mean %.2f us, max %.2f us; slowest:",
                    k, (long long)(a1 - a0), t_hi > t_lo ? (double)(t_hi - t_lo) * 0.01 : 0.0,
                    d.empty() ? 0.0 : sum / d.size(), d.empty() ? 0.0 : d[0].first);
            for (size_t i = 0; i < d.size() && i < 6; ++i) {
                const uint64_t m = tl[4 * d[i].second + 3];
                const int rel = (int)((m >> 8) & 0xffff);
                const CleRel& q = p->h_rels[rel];
                const CleTask& tk = p->h_atasks[d[i].second];
                fprintf(stderr, " [%.2f us kind %d rel %d n %lld c1 %lld o2 %lld i2 %lld khw2 %lld o2g %lld fuse %d cols %lld",
                        d[i].first, (int)(m & 255), rel, (long long)(m >> 24), (long long)q.c1, (long long)q.o2,
                        (long long)q.i2, (long long)q.khw2, (long long)q.o2g, q.fuse_next, (long long)(tk.c1 - tk.c0));
                const uint64_t sub = tl[4 * d[i].second + 2];
                if (sub >> 63)   // phase marks (us after the task's start)
                    fprintf(stderr, q.khw2 > 1 ? " scales %.2f inv_pos %.2f rows %.2f" : " landed %.2f rows %.2f barrier %.2f",
                            (double)(sub & 0xffff) * 0.01, (double)((sub >> 16) & 0xffff) * 0.01,
                            (double)((sub >> 32) & 0xffff) * 0.01);
                fprintf(stderr, "]");
            }
            // start-time histogram: when the tasks began relative to the first
            fprintf(stderr, "\nDFQ_CLE_TL step %d starts (us after first):", k);
            std::vector<double> st;
            for (int64_t t = a0; t < a1; ++t)
                if (tl[4 * t]) st.push_back((double)(tl[4 * t] - t_lo) * 0.01);
            std::sort(st.begin(), st.end());
            for (double q : {0.1, 0.5, 0.9, 0.99, 1.0})
                if (!st.empty()) fprintf(stderr, " p%.0f %.2f", q * 100, st[std::min(st.size() - 1, (size_t)(q * st.size()))]);
            // per task kind: count, mean / max duration, mean start
            fprintf(stderr, "\nDFQ_CLE_TL step %d kinds:", k);
            for (int kind = 0; kind < 8; ++kind) {
                int64_t cnt = 0;
                double sum = 0, mx = 0, s0 = 0;
                for (int64_t t = a0; t < a1; ++t) {
                    const uint64_t* r = &tl[4 * t];
                    if (!r[0] || (int)(r[3] & 255) != kind) continue;
                    const double us = (double)(r[1] - r[0]) * 0.01;
                    ++cnt;
                    sum += us;
                    mx = std::max(mx, us);
                    s0 += (double)(r[0] - t_lo) * 0.01;
                }
                if (cnt)
                    fprintf(stderr, " [kind %d: %lld tasks, mean %.2f max %.2f us, start mean %.2f]", kind,
                            (long long)cnt, sum / cnt, mx, s0 / cnt);
            }
            fprintf(stderr, "\n");
        }
    }
#endif
    // the final state (a no-op iteration after convergence changed nothing)
    const CleState fin = *p->h_state;
    if (fin.error) {   // a range block saw the wrong parity: never expected
        set_last_hip_error(hipErrorLaunchTimeOut);
        return DFQ_ERR_HIP;
    }
    if (!fin.done) {   // the stop rule never said done: never report a partial loop as a result
        set_last_hip_error_text(deadline_hit ? "the launched CLE loop reached its time limit before converging"
                                             : "the CLE loop stopped before its stop rule said done");
        return DFQ_ERR_HIP;
    }
    if (ab_env("DFQ_CLE_DEBUG")) {   // per-layer chunk sums of the last iteration run
        std::vector<float> part((size_t)p->slots * std::max(p->nl, 1));
        DFQ_HIP_CHECK(cle_copy_back(part.data(), p->d_part, sizeof(float) * part.size(), s));
        for (int32_t l = 0; l < p->nl; ++l) {
            fprintf(stderr, "DFQ_CLE_DEBUG layer %d:", l);
            for (int t = 0; t < p->slots; ++t) fprintf(stderr, " %.9g", part[(size_t)p->slots * l + t]);
            fprintf(stderr, "\n");
        }
    }
    if (iterations) *iterations = fin.iters;
    if (hist) {
        hist->assign((size_t)std::max(fin.iters, 0), 0.0);
        if (fin.iters > 0) std::memcpy(hist->data(), ctx.h_hist, sizeof(double) * std::min(fin.iters, hn));
    }
    return DFQ_OK;
}

extern "C" int dfq_cle_plan_run(dfq_cle_plan* p, double threshold, int32_t count, int32_t max_iters,
                                int32_t* iterations, double* diffs, void* stream) {
    if (!p || max_iters < 0 || p->async) return DFQ_ERR_INVALID;   // a launched plan is joined instead
    // The loop runs on the device context's stream: wait for the caller's
    // producers first; the call is blocking.
    const double ts0 = now_us();
    DFQ_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    const double ts1 = now_us();
    int dev = 0;
    DFQ_HIP_CHECK(hipGetDevice(&dev));
    CleDeviceCtx& ctx = cle_device_ctx(dev);
    std::lock_guard<std::mutex> lock(ctx.mu);
    if (cle_timing()) fprintf(stderr, "DFQ_CLE_TIMING run: caller sync %.1f us, context %.1f us\n", ts1 - ts0,
                              now_us() - ts1);
    std::vector<double> h;
    const int rc = cle_run_locked(p, ctx, threshold, count, max_iters, iterations, diffs ? &h : nullptr);
    if (rc == DFQ_OK && diffs && !h.empty()) std::memcpy(diffs, h.data(), sizeof(double) * h.size());
    return rc;
}

namespace dfq {
// The caller's stream gate of a launched loop: one lane polls the signal word
// until the worker has written this run's generation behind the loop's last
// launch, sleeping between polls.  A CP wait packet (hipStreamWaitValue64) in
// the caller's queue measured 1.8x slower loops (MobileNetV2 CLE 2.73 -> 4.97 ms:
// the polling packet holds up the dispatch of the loop's queue), a running
// one-wave kernel costs nothing.  Bounded: past `limit` ticks of the 100 MHz
// clock (kCleGateSeconds: never reached by a loop that is running -- a
// MobileNetV2 loop takes milliseconds) it traps instead of returning, so a lost
// release cannot hang the queue and nothing queued behind the gate runs on weights
// a still-running loop is rescaling.  A loop that FAILS (a HIP error, the launch
// deadline) is not held back this way: the worker releases the gate behind
// whatever the loop enqueued, the caller's queued stages (absorption, the second
// fold, quantize, bias correction) run on the failed loop's weights, and the
// failure is raised at the join (Cross_layer_equal.wait(), which run_dfq,
// main_dfq and every read of the loop's results call), so those results are
// never returned as a success.
__global__ void __launch_bounds__(64) cle_caller_gate_kernel(const uint64_t* sig, uint64_t gen, uint64_t limit) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < gen) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > limit) __builtin_trap();
        __builtin_amdgcn_s_sleep(32);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
}
}  // namespace dfq

// ---- asynchronous run (dfq_cle_plan_launch / _join) -------------------------
// The loop needs the host between iterations (it polls the stop rule), so a
// worker thread drives it on the context's stream while the caller's thread goes
// on enqueueing the next stages on its own stream.  That stream waits, in the
// device, behind the gate kernel for a per-device signal word the worker writes
// behind the loop's last launch (hipStreamWriteValue64): no host sync between
// the stages, and nothing of the caller's stream runs before the loop is done.
// The loop stream is a high-priority stream: it gets a hardware queue of its own
// (queues are pooled per priority), so the caller's waiting queue can never hold
// the loop's launches back.
// (the gate's limit and the launched run's deadline: kCleGateSeconds, above)

struct CleAsync {
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    int rc = DFQ_OK;
    int32_t iters = 0;
    std::vector<double> hist;
    char err[128] = {0};
};

// One long-lived worker thread per device context: a thread created per run paid
// the HIP runtime's per-thread setup on every run.  Detached, never destroyed (a
// process ends with it idle: wait() / destroy join every launched run first).
struct CleWorker {
    std::mutex m;
    std::condition_variable cv;
    std::function<void()> job;
    bool has_job = false;
};
static void cle_worker_loop(CleWorker* w) {
    for (;;) {
        std::function<void()> j;
        {
            std::unique_lock<std::mutex> l(w->m);
            w->cv.wait(l, [w] { return w->has_job; });
            j = std::move(w->job);
            w->has_job = false;
        }
        j();
    }
}

// The context's signal word (lazily allocated as HIP signal memory: the gate
// kernel polls it, the worker writes it with hipStreamWriteValue64); when it
// cannot be allocated, callers run synchronously.
static hipError_t cle_signal_ready(CleDeviceCtx& ctx) {
    if (ctx.sig) return hipSuccess;
    if (ctx.sig_state < 0) return hipErrorNotSupported;
    hipError_t e = hipSuccess;
    void* sig = nullptr;
    if ((e = hipExtMallocWithFlags(&sig, sizeof(uint64_t), hipMallocSignalMemory)) != hipSuccess) {
        ctx.sig_state = -1;
        return e;
    }
    // generation 0, in stream order on the loop stream
    if ((e = hipStreamWriteValue64(ctx.st, sig, 0, 0)) != hipSuccess || (e = hipStreamSynchronize(ctx.st)) != hipSuccess) {
        (void)hipFree(sig);
        ctx.sig_state = -1;
        return e;
    }
    ctx.sig = sig;
    ctx.gen = 0;
    return hipSuccess;
}

// Waits for a launched run; false when it has not finished within `seconds`
// (< 0: no limit).
static bool cle_async_join(dfq_cle_plan* p, double seconds = -1.0) {
    if (!p || !p->async) return true;
    CleAsync* a = p->async;
    std::unique_lock<std::mutex> l(a->m);
    if (seconds < 0) {
        a->cv.wait(l, [a] { return a->done; });
        return true;
    }
    return a->cv.wait_for(l, std::chrono::duration<double>(seconds), [a] { return a->done; });
}

extern "C" int dfq_cle_plan_launch(dfq_cle_plan* p, double threshold, int32_t count, int32_t max_iters,
                                   void* stream) {
    if (!p || max_iters < 0 || p->async) return DFQ_ERR_INVALID;
    // The diagnostics task timeline allocates and frees inside the loop, which may
    // synchronise the whole device -- behind a caller's stream that waits for the
    // loop: it takes the blocking run (the product library reads no switches).
    if (ab_env("DFQ_CLE_TL")) return DFQ_ERR_UNSUPPORTED;
    hipStream_t caller = static_cast<hipStream_t>(stream);
    CleDeviceCtx& ctx = cle_device_ctx(p->dev);
    const double tl0 = now_us();
    // one launched loop per device at a time: the signal's generations then
    // complete in launch order
    if (ctx.pending && ctx.pending != p) cle_async_join(ctx.pending);
    ctx.pending = nullptr;
    uint64_t gen = 0;
    {
        std::lock_guard<std::mutex> lock(ctx.mu);
        DFQ_HIP_CHECK(hipSetDevice(p->dev));
        DFQ_HIP_CHECK(cle_ctx_ready(ctx));
        const hipError_t es = cle_signal_ready(ctx);
        if (es == hipErrorNotSupported) return DFQ_ERR_UNSUPPORTED;
        DFQ_HIP_CHECK(es);
        DFQ_HIP_CHECK(cle_hist_ready(ctx, max_iters));   // no hipFree in the worker
        // the caller's producers before the loop; the caller's later work after it
        DFQ_HIP_CHECK(hipEventRecord(ctx.in_ev, caller));
        DFQ_HIP_CHECK(hipStreamWaitEvent(ctx.st, ctx.in_ev, 0));
        gen = ctx.gen + 1;
        // the caller's stream waits behind a gate kernel (cle_caller_gate_kernel);
        // a CP wait packet (hipStreamWaitValue64) there measured 1.8x slower loops
        // (profiles/r03/async_ab/)
        hipLaunchKernelGGL(cle_caller_gate_kernel, dim3(1), dim3(64), 0, caller,
                           static_cast<const uint64_t*>(ctx.sig), gen, (uint64_t)kCleGateSeconds * 100000000ull);
        DFQ_LAUNCH_CHECK();
        ctx.gen = gen;
    }
    if (cle_timing()) fprintf(stderr, "DFQ_CLE_TIMING launch: gate and order %.1f us\n", now_us() - tl0);
    // from here on the caller's stream is held until the signal reaches gen: every
    // path below writes it
    CleAsync* a = new (std::nothrow) CleAsync();
    const double t_launch = now_us();
    auto body = [p, &ctx, threshold, count, max_iters, gen, t_launch](CleAsync* a) {
        std::lock_guard<std::mutex> lock(ctx.mu);
        int rc = DFQ_OK;
        if (hipSetDevice(p->dev) != hipSuccess) {
            rc = DFQ_ERR_HIP;
        } else {
            rc = cle_run_locked(p, ctx, threshold, count, max_iters, &a->iters, &a->hist, kCleLaunchDeadlineUs);
        }
        if (rc == DFQ_ERR_HIP) {
            const char* m = dfq_last_hip_error();
            for (size_t i = 0; m && m[i] && i + 1 < sizeof(a->err); ++i) a->err[i] = m[i];
        }
#ifdef DFQ_DIAGNOSTICS   // tests of the held caller stream (test_gpu_cle_plan.py): a late release
        if (const char* d = ab_env("DFQ_CLE_TEST_RELEASE_DELAY_MS"))
            std::this_thread::sleep_for(std::chrono::milliseconds(atoi(d)));
#endif
        // release the caller's stream behind everything the loop enqueued
        hipError_t e = hipStreamWriteValue64(ctx.st, ctx.sig, gen, 0);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx.st);
        if (e != hipSuccess) {   // never expected; the gate traps at its time limit
            fprintf(stderr, "dfq_cle_plan_launch: releasing the caller's stream failed (%s)\n", hipGetErrorString(e));
            if (rc == DFQ_OK) rc = DFQ_ERR_HIP;
        }
        if (rc == DFQ_OK && now_us() - t_launch > 0.9e6 * kCleGateSeconds) {   // the gate may have opened early
            set_last_hip_error(hipErrorLaunchTimeOut);
            const char* m = "CLE loop outlived the caller's stream gate";
            for (size_t i = 0; m[i] && i + 1 < sizeof(a->err); ++i) a->err[i] = m[i];
            rc = DFQ_ERR_HIP;
        }
        {
            std::lock_guard<std::mutex> l(a->m);
            a->rc = rc;
            a->done = true;
        }
        a->cv.notify_all();   // a is the joiner's from here on
    };
    if (!a) {   // no memory for the worker's record: run here, then release
        CleAsync tmp;
        body(&tmp);
        return tmp.rc;
    }
    p->async = a;
    ctx.pending = p;
    p->d_sig = static_cast<uint64_t*>(ctx.sig);   // released behind the loop's rollback (cle_run_locked)
    if (ab_env("DFQ_CLE_HOST_RELEASE")) p->d_sig = nullptr;   // diagnostics: only the worker's release, after the run
    p->gen = gen;
    bool posted = false;
    try {
        if (!ctx.worker) {
            CleWorker* w = new CleWorker();
            std::thread(cle_worker_loop, w).detach();
            ctx.worker = w;
        }
        {
            std::lock_guard<std::mutex> l(ctx.worker->m);
            ctx.worker->job = [body, a] { body(a); };
            ctx.worker->has_job = true;
        }
        ctx.worker->cv.notify_one();
        posted = true;
    } catch (...) {
    }
    if (!posted) body(a);   // no worker: run on this thread (blocking), which also releases
    if (cle_timing()) fprintf(stderr, "DFQ_CLE_TIMING launch: total %.1f us\n", now_us() - tl0);
    return DFQ_OK;
}

extern "C" int dfq_cle_plan_join(dfq_cle_plan* p, int32_t* iterations, double* diffs) {
    if (!p || !p->async) return DFQ_ERR_INVALID;
    if (p->abandoned) return DFQ_ERR_HIP;
    double limit = kCleJoinSeconds;
#ifdef DFQ_DIAGNOSTICS
    if (const char* j = ab_env("DFQ_CLE_TEST_JOIN_LIMIT_MS")) limit = atoi(j) * 1e-3;
#endif
    if (!cle_async_join(p, limit)) {
        // The loop has not finished: the caller's stream stays held behind the gate
        // (which traps at its own limit); the plan stays with the worker, which may
        // still use it (destroy leaves it alone).
        p->abandoned = true;
        set_last_hip_error_text("the launched CLE loop did not finish in time; the caller's stream stays held");
        return DFQ_ERR_HIP;
    }
    CleDeviceCtx& ctx = cle_device_ctx(p->dev);
    if (ctx.pending == p) ctx.pending = nullptr;
    const CleAsync& a = *p->async;
    if (a.rc == DFQ_ERR_HIP && a.err[0]) set_last_hip_error_text(a.err);
    if (a.rc != DFQ_OK) return a.rc;
    if (iterations) *iterations = a.iters;
    if (diffs && !a.hist.empty()) std::memcpy(diffs, a.hist.data(), sizeof(double) * a.hist.size());
    return DFQ_OK;
}

extern "C" int dfq_cle_plan_info(const dfq_cle_plan* p, int32_t* chains, int32_t* steps, int32_t* launches) {
    if (!p) return DFQ_ERR_INVALID;
    if (chains) *chains = p->chains;
    if (steps) *steps = p->steps;
    // per iteration: the rescale launches (+ per-step range launches when the
    // schedule is not fused), + a tiles-only launch unless the schedule is lagged
    if (launches) *launches = p->fused ? p->nlaunch : 2 * p->steps + 1;
    return DFQ_OK;
}

extern "C" int dfq_cle_plan_set_timing(dfq_cle_plan* p, int32_t on) {
    if (!p || p->async) return DFQ_ERR_INVALID;
    p->timed = on != 0;
    return DFQ_OK;
}

extern "C" int dfq_cle_plan_stats(const dfq_cle_plan* p, int64_t* bytes, double* loop_ms, int32_t* launched) {
    if (!p) return DFQ_ERR_INVALID;
    if (bytes) {
        bytes[0] = p->bytes[0];
        bytes[1] = p->bytes[1];
        bytes[2] = p->bytes[2];
    }
    if (loop_ms) *loop_ms = p->loop_ms;
    if (launched) *launched = p->launched;
    return DFQ_OK;
}

extern "C" int dfq_cle_plan_destroy(dfq_cle_plan* p) {
    if (!p) return DFQ_OK;
    if (p->abandoned) return DFQ_OK;   // its worker may still run it: left to the worker (leaked)
    if (p->async) {   // a launched run finishes first (its worker uses the plan)
        cle_async_join(p);
        CleDeviceCtx& ctx = cle_device_ctx(p->dev);
        if (ctx.pending == p) ctx.pending = nullptr;
        delete p->async;
        p->async = nullptr;
    }
    cle_plan_free(p);
    return DFQ_OK;
}


namespace dfq {
// What a first CLE run on a device would otherwise allocate inside the caller's
// timed region (a cold main_dfq run: plan create 314 against 55 us warm, launch 160
// against 20): the table pools at a size that holds the zoo models' tables, the
// iteration history for the default DFQ_CLE_MAX_ITERS, the signal word of launched
// runs and their worker thread.
constexpr size_t kClePreloadPool = size_t(4) << 20, kClePreloadHostPool = size_t(2) << 20;
constexpr int32_t kClePreloadHistIters = 100000;   // Cross_layer_equal.MAX_ITERS' default
hipError_t preload_cle() {   // see dfq_preload
    int dev = 0;
    hipError_t e0 = hipGetDevice(&dev);
    if (e0 != hipSuccess) return e0;
    {
        CleDeviceCtx& ctx = cle_device_ctx(dev);
        std::lock_guard<std::mutex> lock(ctx.mu);
        if ((e0 = cle_ctx_ready(ctx)) != hipSuccess) return e0;
        if (!ctx.pool_busy && ctx.pool_cap < kClePreloadPool) {
            (void)hipFree(ctx.d_pool);
            ctx.d_pool = nullptr;
            ctx.pool_cap = 0;
            ctx.pool_struct = 0;
            if ((e0 = hipMalloc(&ctx.d_pool, kClePreloadPool)) != hipSuccess) return e0;
            ctx.pool_cap = kClePreloadPool;
        }
        if (!ctx.pool_busy && ctx.hpool_cap < kClePreloadHostPool) {
            (void)hipHostFree(ctx.h_pool);
            ctx.h_pool = nullptr;
            ctx.hpool_cap = 0;
            if ((e0 = hipHostMalloc(&ctx.h_pool, kClePreloadHostPool, hipHostMallocDefault)) != hipSuccess) return e0;
            ctx.hpool_cap = kClePreloadHostPool;
        }
        if ((e0 = cle_hist_ready(ctx, kClePreloadHistIters)) != hipSuccess) return e0;
        (void)cle_signal_ready(ctx);   // unsupported: launched runs fall back to blocking ones
        if (!ctx.worker) {
            try {
                CleWorker* w = new CleWorker();
                std::thread(cle_worker_loop, w).detach();
                ctx.worker = w;
            } catch (...) {   // created at the first launch instead
            }
        }
    }
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(cle_loop_step_kernel<true>));
    if (e == hipSuccess) e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(cle_loop_step_kernel<false>));
    return e;
}
}  // namespace dfq

#ifdef DFQ_DIAGNOSTICS
#include "dfq_diag.h"   // default visibility for the entry point below
// ---- diagnostics: the plan structure's index invariants, on the host -----------
// Builds the structure dfq_cle_plan_create would (chains, tasks, metric chunks and
// units, the lagged placement) -- host code only, no device memory, so it runs on
// a machine without a GPU and with stand-in addresses -- and checks every index
// the step, range, tile, stop-rule and rollback blocks derive from it:
//  * task tables: step offsets monotone and inside the tables; every task's
//    relation, rows / channels / columns inside that relation's shapes;
//  * range words and rollback saves: moff + 2 c1 <= M (both parities' words) and
//    2 moff + 4 c1 <= 2 M (vsave: b1 | bn_w | bn_b | S per channel);
//  * metric chunks and units: layer, element span, level-1 slots inside the tables;
//  * placement: per launch offset the unit / range slices partition the tables;
//    a tensor's tiles and ranges sit after its last rescale of iteration i and
//    before its first rescale of iteration i + 1 (its window), range resets after
//    their relation's step; lagged plans: the stop rule one offset after every tile
//    of its iteration and before the next iteration's first tile.
// The round-5 fault of a development tree was in this code's
// domain; tests/test_cle_structure.py runs it on every zoo model and schedule
// switch and on fuzzed relation graphs.
// info[0..7] = steps, nlaunch, lagged, stop_off, rescale tasks, range tasks, units,
// chunks.  Returns DFQ_OK, or DFQ_ERR_INVALID with the first violation in msg.
extern "C" int dfq_diag_cle_check_structure(const dfq_cle_rel* rels, int32_t n_rel, float* const* targets,
                                            const int64_t* target_n, int32_t n_targets, int32_t ref_threads,
                                            int64_t* info, char* msg, int32_t msg_cap) {
    auto fail = [&](const char* fmt, long long a, long long b, long long c) {
        if (msg && msg_cap > 0) snprintf(msg, (size_t)msg_cap, fmt, a, b, c);
        return DFQ_ERR_INVALID;
    };
    if (n_rel < 0 || n_targets < 0 || (n_rel > 0 && !rels) || (n_targets > 0 && (!targets || !target_n)))
        return fail("bad arguments %lld %lld %lld", n_rel, n_targets, 0);
    std::vector<CleRel> R0;
    int64_t M = 0;
    if (const int rc = cle_rels_from_desc(rels, n_rel, R0, M); rc != DFQ_OK) return rc;
    CleStructure S;
    if (const int rc = cle_build_structure(R0, M, n_rel, targets, target_n, n_targets, ref_threads, S); rc != DFQ_OK)
        return rc;
    const std::vector<CleRel>& R = S.R;
    const int32_t steps = S.steps, NL = S.nlaunch;
    if (const char* e = getenv("DFQ_CLE_PLACE_DUMP"); e && *e) {
        // per launch offset: blocks and bytes of rescale tasks, metric tiles and range tasks
        fprintf(stderr, "DFQ_CLE_PLACE steps %d nlaunch %d lagged %d stop_off %d\n", steps, NL, (int)S.lagged,
                S.stop_off);
        for (int32_t k = 0; k < 2 * NL; ++k) {
            int64_t na = 0;
            double ba = 0;
            if (k < steps)
                for (int64_t t = S.astep[k]; t < S.astep[k + 1]; ++t, ++na) {
                    const CleTask& tk = S.at[t];
                    const CleRel& q = R[tk.rel];
                    const int64_t n = tk.b - tk.a;
                    if (tk.kind == kApplyW1) ba += 8.0 * n * q.len1;
                    else if (tk.kind == kApplyW2Tile) ba += 8.0 * n * (tk.c1 - tk.c0) * q.khw2;
                    else if (tk.kind != kApplyChannels) ba += 8.0 * n * q.o2g * q.khw2;
                }
            double bu = 0;
            for (int64_t u = S.uoffs[k]; u < S.uoffs[k + 1]; ++u) {
                const CleChunk& ch = S.chunks[S.units[u].chunk];
                const int64_t nb1 = ch.len / kCleTile;
                bu += 12.0 * (S.units[u].tile < nb1 ? kCleTile : ch.len - nb1 * kCleTile);
            }
            double br = 0;
            for (int64_t t = S.roffs[k]; t < S.roffs[k + 1]; ++t) {
                const CleTask& tk = S.rt[t];
                const CleRel& q = R[tk.rel];
                const int64_t n = tk.b - tk.a;
                if (tk.kind == kRangeW1) br += 4.0 * n * q.len1;
                else if (tk.kind == kRangeW2Contig) br += 4.0 * n * q.o2g * q.khw2;
                else if (tk.kind == kRangeW2Tile) br += 4.0 * n * (tk.c1 - tk.c0) * q.khw2;
            }
            fprintf(stderr, "DFQ_CLE_PLACE offset %d: rescale %lld blocks %.2f MB, tiles %lld blocks %.2f MB, ranges %lld blocks %.2f MB\n",
                    k, (long long)na, ba / 1e6, (long long)(S.uoffs[k + 1] - S.uoffs[k]), bu / 1e6,
                    (long long)(S.roffs[k + 1] - S.roffs[k]), br / 1e6);
        }
    }
    if (info) {
        const int64_t v[8] = {steps, NL, S.lagged ? 1 : 0, S.stop_off, (int64_t)S.at.size(), (int64_t)S.rt.size(),
                              (int64_t)S.units.size(), (int64_t)S.chunks.size()};
        std::memcpy(info, v, sizeof(v));
    }
    // relations: range words and rollback saves inside their tables, links valid
    for (int32_t r = 0; r < n_rel; ++r) {
        const CleRel& c = R[r];
        if (c.moff < 0 || c.moff + 2 * c.c1 > S.M) return fail("rel %lld: range words [%lld, +2 c1) past M %lld", r, c.moff, S.M);
        if (2 * c.moff + 4 * c.c1 > 2 * S.M) return fail("rel %lld: rollback saves past 2 M (moff %lld, c1 %lld)", r, c.moff, c.c1);
        if (c.fuse_next >= n_rel || c.dw_prev >= n_rel || c.fuse_next < -1 || c.dw_prev < -1)
            return fail("rel %lld: link out of range (fuse_next %lld, dw_prev %lld)", r, c.fuse_next, c.dw_prev);
        if (c.fuse_next >= 0 && R[c.fuse_next].moff + R[c.fuse_next].c1 > S.M)
            return fail("rel %lld: fused W1 words of rel %lld past M %lld", r, c.fuse_next, S.M);
    }
    // rescale tasks per step
    if ((int32_t)S.astep.size() != steps + 1 || S.astep[0] != 0 || S.astep.back() != (int64_t)S.at.size())
        return fail("astep: %lld entries for %lld steps, last %lld", (long long)S.astep.size(), steps,
                    S.astep.empty() ? -1 : S.astep.back());
    std::vector<int32_t> rel_step(n_rel, -1);
    std::vector<std::pair<const float*, int32_t>> touch;   // (tensor, step) of every weight rescale
    for (int32_t k = 0; k < steps; ++k) {
        if (S.astep[k + 1] < S.astep[k]) return fail("astep not monotone at step %lld: %lld > %lld", k, S.astep[k], S.astep[k + 1]);
        for (int64_t t = S.astep[k]; t < S.astep[k + 1]; ++t) {
            const CleTask& tk = S.at[t];
            if (tk.rel < 0 || tk.rel >= n_rel) return fail("rescale task %lld: relation %lld of %lld", t, tk.rel, n_rel);
            const CleRel& c = R[tk.rel];
            if (tk.a < 0 || tk.a >= tk.b) return fail("rescale task %lld: empty or negative span [%lld, %lld)", t, tk.a, tk.b);
            switch (tk.kind) {
                case kApplyW1:
                    if (tk.b > c.c1) return fail("W1 task %lld: rows to %lld of %lld", t, tk.b, c.c1);
                    touch.push_back({c.w1, k});
                    break;
                case kApplyW2Contig:
                    if (tk.b > c.c1 || c.i2 != 1) return fail("W2 contig task %lld: channels to %lld of %lld", t, tk.b, c.c1);
                    touch.push_back({c.w2, k});
                    break;
                case kApplyDwBoth:
                    if (tk.b > c.c1 || tk.c0 < 0 || tk.c0 >= n_rel || R[tk.c0].w1 != c.w2 || R[tk.c0].dw_prev != tk.rel)
                        return fail("depthwise pair task %lld: partner %lld, channels to %lld", t, tk.c0, tk.b);
                    touch.push_back({c.w2, k});
                    break;
                case kApplyW2Tile:
                    if (tk.b > c.o2 || tk.c0 < 0 || tk.c0 >= tk.c1 || tk.c1 > c.i2)
                        return fail("W2 tile task %lld: rows to %lld, columns to %lld", t, tk.b, tk.c1);
                    touch.push_back({c.w2, k});
                    break;
                case kApplyChannels:
                    if (tk.b > c.c1) return fail("channel task %lld: channels to %lld of %lld", t, tk.b, c.c1);
                    if (rel_step[tk.rel] >= 0 && rel_step[tk.rel] != k)
                        return fail("relation %lld: channel tasks in steps %lld and %lld", tk.rel, rel_step[tk.rel], k);
                    rel_step[tk.rel] = k;
                    break;
                default:
                    return fail("rescale task %lld: kind %lld", t, tk.kind, 0);
            }
        }
    }
    for (int32_t r = 0; r < n_rel; ++r)
        if (rel_step[r] < 0) return fail("relation %lld has no channel task", r, 0, 0);
    // range tasks
    const int64_t nrt = (int64_t)S.rt.size();
    if (S.ri0 < 0 || S.ri0 > S.ri1 || S.ri1 > nrt) return fail("range slice [%lld, %lld) of %lld tasks", S.ri0, S.ri1, nrt);
    for (int64_t t = 0; t < nrt; ++t) {
        const CleTask& tk = S.rt[t];
        if (tk.rel < 0 || tk.rel >= n_rel) return fail("range task %lld: relation %lld of %lld", t, tk.rel, n_rel);
        const CleRel& c = R[tk.rel];
        if (tk.a < 0 || tk.a >= tk.b) return fail("range task %lld: span [%lld, %lld)", t, tk.a, tk.b);
        const bool ok = tk.kind == kRangeW2Tile ? (tk.b <= c.o2 && tk.c0 >= 0 && tk.c0 < tk.c1 && tk.c1 <= c.i2)
                                                : (tk.kind >= kRangeW1 && tk.kind <= kRangeResetW1 && tk.b <= c.c1);
        if (!ok) return fail("range task %lld (kind %lld): span to %lld out of the relation's shape", t, tk.kind, tk.b);
    }
    // metric chunks and units
    int64_t nb1_seen = 0;
    for (size_t ci = 0; ci < S.chunks.size(); ++ci) {
        const CleChunk& ch = S.chunks[ci];
        if (ch.layer < 0 || ch.layer >= n_targets) return fail("chunk %lld: layer %lld of %lld", (long long)ci, ch.layer, n_targets);
        if (ch.c0 < 0 || ch.len <= 0 || ch.c0 + ch.len > target_n[ch.layer])
            return fail("chunk %lld: elements [%lld, +%lld) past its layer", (long long)ci, ch.c0, ch.len);
        const int64_t nb1 = ch.len / 32 / 256;
        if (S.b1off[ci] != 32 * nb1_seen) return fail("chunk %lld: level-1 offset %lld, expected %lld", (long long)ci, S.b1off[ci], 32 * nb1_seen);
        nb1_seen += nb1;
    }
    if (nb1_seen != S.nb1_total) return fail("level-1 slots %lld, table %lld", nb1_seen, S.nb1_total, 0);
    for (size_t u = 0; u < S.units.size(); ++u) {
        const CleUnit& un = S.units[u];
        if (un.chunk < 0 || un.chunk >= (int32_t)S.chunks.size()) return fail("unit %lld: chunk %lld", (long long)u, un.chunk, 0);
        const CleChunk& ch = S.chunks[un.chunk];
        if (ch.len < 8 || un.tile < 0 || un.tile > ch.len / 32 / 256)
            return fail("unit %lld: tile %lld of chunk %lld", (long long)u, un.tile, un.chunk);
        // cle_tiles_body's element ranges: a full tile is 8,192 elements inside the
        // chunk; a tail tile's [e0, len) (empty when 8,192 divides the chunk) fits the
        // LDS staging area below the b0 sums
        const int64_t nb1 = ch.len / 32 / 256, e0 = (int64_t)un.tile * kCleTile;
        if (un.tile < nb1 ? e0 + kCleTile > ch.len : (ch.len - e0 < 0 || ch.len - e0 > kCleTile + kCleTailWords))
            return fail("unit %lld: tile past chunk %lld (len %lld)", (long long)u, un.chunk, ch.len);
    }
    // placement tables
    if ((int32_t)S.uoffs.size() != 2 * NL + 1 || S.uoffs[0] != 0 || S.uoffs.back() != (int64_t)S.units.size())
        return fail("uoffs: %lld entries for %lld launches, last %lld", (long long)S.uoffs.size(), NL, S.uoffs.back());
    for (int32_t k = 0; k < 2 * NL; ++k)
        if (S.uoffs[k + 1] < S.uoffs[k]) return fail("uoffs not monotone at %lld", k, 0, 0);
    if (S.fused) {
        if ((int32_t)S.roffs.size() != 2 * NL + 1 || S.roffs[0] != S.ri0 || S.roffs.back() != S.ri1)
            return fail("roffs: %lld entries, [%lld, %lld)", (long long)S.roffs.size(), S.roffs.empty() ? -1 : S.roffs[0],
                        S.roffs.empty() ? -1 : S.roffs.back());
        for (int32_t k = 0; k < 2 * NL; ++k)
            if (S.roffs[k + 1] < S.roffs[k]) return fail("roffs not monotone at %lld", k, 0, 0);
    } else if ((int32_t)S.rstep.size() != steps + 1 || S.rstep.back() != nrt) {
        return fail("unfused rstep: %lld entries, last %lld of %lld", (long long)S.rstep.size(), S.rstep.back(), nrt);
    }
    if (NL != (S.lagged ? steps : steps + 1)) return fail("nlaunch %lld for %lld steps (lagged %lld)", NL, steps, S.lagged);
    // windows: a tensor's first / last rescale step
    auto span = [&](const float* w, int32_t& first, int32_t& last) {
        first = INT32_MAX;
        last = -1;
        for (const auto& x : touch)
            if (x.first == w) {
                first = std::min(first, x.second);
                last = std::max(last, x.second);
            }
        return last >= 0;
    };
    auto in_window = [&](const float* w, int32_t o) {
        int32_t f, l;
        if (!span(w, f, l)) return o >= 0 && o <= 2 * NL - 1;
        return o >= l + 1 && o <= std::min(2 * NL - 1, NL + f - 1);
    };
    int32_t umin = INT32_MAX, umax = -1;
    for (int32_t k = 0; k < 2 * NL; ++k)
        for (int64_t u = S.uoffs[k]; u < S.uoffs[k + 1]; ++u) {
            const int32_t l = S.chunks[S.units[u].chunk].layer;
            if (!S.lagged && k != steps) return fail("unit %lld of layer %lld at offset %lld outside the tiles-only launch", u, l, k);
            if (!in_window(targets[l], k)) return fail("unit %lld of layer %lld at offset %lld outside its tensor's window", u, l, k);
            umin = std::min(umin, k);
            umax = std::max(umax, k);
        }
    if (S.fused)
        for (int32_t k = 0; k < 2 * NL; ++k)
            for (int64_t t = S.roffs[k]; t < S.roffs[k + 1]; ++t) {
                const CleTask& tk = S.rt[t];
                const CleRel& c = R[tk.rel];
                bool ok = true;
                switch (tk.kind) {
                    case kRangeW1: ok = in_window(c.w1, k); break;
                    case kRangeW2Contig:
                    case kRangeW2Tile: ok = in_window(c.w2, k); break;
                    case kRangeReset: {
                        int32_t f, l;
                        span(c.w2, f, l);
                        ok = k >= rel_step[tk.rel] + 1 && k <= std::min(2 * NL - 1, NL + l);
                        break;
                    }
                    default: ok = k >= rel_step[tk.rel] + 1 && k <= 2 * NL - 1;   // kRangeResetW1
                }
                if (!S.lagged && k != steps) ok = false;
                if (!ok) return fail("range task %lld (kind %lld) at offset %lld outside its window", t, tk.kind, k);
            }
    if (S.lagged && S.stop_off >= 0) {
        if (S.stop_off < steps || S.stop_off > 2 * NL - 1) return fail("stop rule at offset %lld of [%lld, %lld]", S.stop_off, steps, 2 * NL - 1);
        if (umax >= 0 && S.stop_off <= umax) return fail("stop rule at offset %lld, not after the last tile offset %lld", S.stop_off, umax, 0);
        if (umax >= 0 && umin + NL <= S.stop_off)
            return fail("the next iteration's first tile (offset %lld + %lld) not after the stop rule at %lld", umin, NL, S.stop_off);
    } else if (!S.lagged && S.stop_off != -1) {
        return fail("unlagged plan with a stop-rule offset %lld", S.stop_off, 0, 0);
    }
    return DFQ_OK;
}
#endif
