// Graph-transform kernels of the DFQ path (gfx950): BatchNorm folding,
// cross-layer equalization, its convergence metric, high-bias absorption and the
// bias-correction combine.  All are HBM/latency-bound elementwise or row/column
// reductions: no MFMA.  fp32 arithmetic is ordered exactly as the reference's
// torch CPU ops (one rounding per op; -ffp-contract=off, IEEE div/sqrt).
#include "dfq_common.h"

#include <algorithm>
#include <cmath>
#include <new>
#include <vector>

namespace dfq {

constexpr int kThreads = 256;

static int blocks_for(int64_t n, int per_thread = 1) {
    const int64_t b = ceil_div(std::max<int64_t>(n, 1), (int64_t)kThreads * per_thread);
    return (int)std::min<int64_t>(b, 256 * 8);
}

// ---------------------------------------------------------------------------
// BatchNorm folding: utils/layer_transform.py:255-281
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bn_factor(float g, float v, float eps) {
    // bn_weight / torch.sqrt(bn_var + bn_eps)
    return g / sqrtf(v + eps);
}

__global__ void bn_fold_weight_kernel(float* __restrict__ w, const float* __restrict__ g,
                                      const float* __restrict__ v, float eps, int64_t rows, int64_t len) {
    const int64_t n = rows * len;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = i / len;
        w[i] = w[i] * bn_factor(g[o], v[o], eps);
    }
}

__global__ void bn_fold_channel_kernel(float* __restrict__ bias, float* __restrict__ g, float* __restrict__ b,
                                       float* __restrict__ m, float* __restrict__ v, float* __restrict__ fake_w,
                                       float* __restrict__ fake_b, float eps, int64_t rows) {
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < rows; o += (int64_t)gridDim.x * blockDim.x) {
        const float go = g[o], bo = b[o], mo = m[o], vo = v[o];
        const float f = bn_factor(go, vo, eps);
        // conv_bias.mul(f).add(bn_bias - (bn_weight * bn_mean) / sqrt(bn_var + eps))
        const float shift = bo - (go * mo) / sqrtf(vo + eps);
        bias[o] = bias[o] * f + shift;
        if (fake_w) fake_w[o] = fabsf(go);
        if (fake_b) fake_b[o] = bo;
        g[o] = 1.0f;
        v[o] = 1.0f;
        b[o] = 0.0f;
        m[o] = 0.0f;
    }
}

// ---------------------------------------------------------------------------
// clip_weight: clip_weight.py:29  (layer.weight.data.clamp_(lo, hi))
// ---------------------------------------------------------------------------
__global__ void clamp_kernel(float* __restrict__ w, int64_t n, float lo, float hi) {
    const int64_t n4 = n >> 2;
    float4* w4 = reinterpret_cast<float4*>(w);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        float4 v = w4[i];
        v.x = fminf(fmaxf(v.x, lo), hi);
        v.y = fminf(fmaxf(v.y, lo), hi);
        v.z = fminf(fmaxf(v.z, lo), hi);
        v.w = fminf(fmaxf(v.w, lo), hi);
        w4[i] = v;
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        w[i] = fminf(fmaxf(w[i], lo), hi);
}

// ---------------------------------------------------------------------------
// Cross-layer equalization: Cross_layer_equal.py:11-59
//   ws layout: [mins1 | mins2] (2*c1 uint32, memset 0xFF)  [maxs1 | maxs2] (2*c1, memset 0)
// ---------------------------------------------------------------------------
struct CleShape {
    int64_t c1, len1, o2, i2, khw2, groups, o2g;
};

// W1 rows: one wave per row.
__global__ void cle_range_w1_kernel(const float* __restrict__ w1, CleShape sh, uint32_t* __restrict__ mins,
                                    uint32_t* __restrict__ maxs) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t c = wave; c < sh.c1; c += nwaves) {
        const float* row = w1 + c * sh.len1;
        float vmin = INFINITY, vmax = -INFINITY;
        for (int64_t i = lane; i < sh.len1; i += 64) {
            const float x = row[i];
            vmin = fminf(vmin, x);
            vmax = fmaxf(vmax, x);
        }
        vmin = wave_min(vmin);
        vmax = wave_max(vmax);
        if (lane == 0) {
            mins[c] = enc_ord(vmin);
            maxs[c] = enc_ord(vmax);
        }
    }
}

// W2 "columns" W2[g*o2g:(g+1)*o2g, i, :] for channel c = g*i2 + i.
// i2 == 1 (depthwise-style groups): the column is contiguous -> one wave per channel.
__global__ void cle_range_w2_contig_kernel(const float* __restrict__ w2, CleShape sh,
                                           uint32_t* __restrict__ mins, uint32_t* __restrict__ maxs) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    const int64_t seg = sh.o2g * sh.khw2;
    for (int64_t c = wave; c < sh.c1; c += nwaves) {
        const float* col = w2 + c * seg;   // channel c = group c, rows [c*o2g, (c+1)*o2g)
        float vmin = INFINITY, vmax = -INFINITY;
        for (int64_t i = lane; i < seg; i += 64) {
            const float x = col[i];
            vmin = fminf(vmin, x);
            vmax = fmaxf(vmax, x);
        }
        vmin = wave_min(vmin);
        vmax = wave_max(vmax);
        if (lane == 0) {
            mins[c] = enc_ord(vmin);
            maxs[c] = enc_ord(vmax);
        }
    }
}

// i2 > 1: each block takes a tile of W2 rows; a thread owns column i and reduces it
// over the tile's rows, then one ordered-uint atomic per (block, column).
constexpr int kColTileRows = 16;
__global__ void cle_range_w2_cols_kernel(const float* __restrict__ w2, CleShape sh,
                                         uint32_t* __restrict__ mins, uint32_t* __restrict__ maxs) {
    const int64_t ntiles = ceil_div(sh.o2, kColTileRows);
    const int64_t rowlen = sh.i2 * sh.khw2;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tile * kColTileRows;
        const int64_t r1 = std::min<int64_t>(r0 + kColTileRows, sh.o2);
        for (int64_t i = threadIdx.x; i < sh.i2; i += blockDim.x) {
            float vmin = INFINITY, vmax = -INFINITY;
            int64_t g_prev = -1;
            for (int64_t o = r0; o < r1; ++o) {
                const int64_t g = o / sh.o2g;
                if (g != g_prev && g_prev >= 0) {   // tile straddles groups: flush
                    const int64_t c = g_prev * sh.i2 + i;
                    atomicMin(&mins[c], enc_ord(vmin));
                    atomicMax(&maxs[c], enc_ord(vmax));
                    vmin = INFINITY; vmax = -INFINITY;
                }
                g_prev = g;
                const float* p = w2 + o * rowlen + i * sh.khw2;
                for (int64_t k = 0; k < sh.khw2; ++k) {
                    const float x = p[k];
                    vmin = fminf(vmin, x);
                    vmax = fmaxf(vmax, x);
                }
            }
            if (g_prev >= 0) {
                const int64_t c = g_prev * sh.i2 + i;
                atomicMin(&mins[c], enc_ord(vmin));
                atomicMax(&maxs[c], enc_ord(vmax));
            }
        }
    }
}

struct CleScale {
    float s;    // stored in S and multiplied into W1 rows, B1, bn_w, bn_b
    float inv;  // multiplied into W2 columns
};

// s = (1 / (r1 + eps)) * sqrt(r1 * r2 + eps); s = max(smin, min(smax, s))  (Python builtins)
__device__ __forceinline__ CleScale cle_scale(const uint32_t* mins, const uint32_t* maxs, int64_t c1, int64_t c,
                                              int is_signed, float eps, double smin, double smax) {
    const float mn1 = dec_ord(mins[c]), mx1 = dec_ord(maxs[c]);
    const float mn2 = dec_ord(mins[c1 + c]), mx2 = dec_ord(maxs[c1 + c]);
    float r1, r2;
    if (is_signed) {
        r1 = fmaxf(fabsf(mn1), fabsf(mx1));
        r2 = fmaxf(fabsf(mn2), fabsf(mx2));
    } else {
        r1 = mx1 - mn1;
        r2 = mx2 - mn2;
    }
    const float s = (1.0f / (r1 + eps)) * sqrtf(r1 * r2 + eps);
    CleScale out;
    if (s < (float)smax) {
        if (s > (float)smin) {
            out.s = s;
            out.inv = 1.0f / s;
        } else {
            out.s = (float)smin;
            out.inv = (float)(1.0 / smin);
        }
    } else {   // includes NaN (dead channel: 0 * inf)
        const double v = (smax > smin) ? smax : smin;
        out.s = (float)v;
        out.inv = (float)(1.0 / v);
    }
    return out;
}

__global__ void cle_apply_kernel(float* __restrict__ w1, float* __restrict__ w2, float* __restrict__ b1,
                                 float* __restrict__ bn_w, float* __restrict__ bn_b, float* __restrict__ S,
                                 float* __restrict__ S_acc, int s_acc_init, CleShape sh,
                                 const uint32_t* __restrict__ mins, const uint32_t* __restrict__ maxs,
                                 int is_signed, float eps, double smin, double smax) {
    const int64_t n1 = sh.c1 * sh.len1;
    const int64_t n2 = sh.o2 * sh.i2 * sh.khw2;
    const int64_t total = n1 + n2 + sh.c1;
    const int64_t rowlen2 = sh.i2 * sh.khw2;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        if (e < n1) {
            const int64_t c = e / sh.len1;
            const CleScale cs = cle_scale(mins, maxs, sh.c1, c, is_signed, eps, smin, smax);
            w1[e] = w1[e] * cs.s;
        } else if (e < n1 + n2) {
            const int64_t f = e - n1;
            const int64_t o = f / rowlen2;
            const int64_t i = (f - o * rowlen2) / sh.khw2;
            const int64_t c = (o / sh.o2g) * sh.i2 + i;
            const CleScale cs = cle_scale(mins, maxs, sh.c1, c, is_signed, eps, smin, smax);
            w2[f] = w2[f] * cs.inv;
        } else {
            const int64_t c = e - n1 - n2;
            const CleScale cs = cle_scale(mins, maxs, sh.c1, c, is_signed, eps, smin, smax);
            if (b1) b1[c] = b1[c] * cs.s;
            if (bn_w) bn_w[c] = bn_w[c] * cs.s;
            if (bn_b) bn_b[c] = bn_b[c] * cs.s;
            if (S) S[c] = cs.s;
            if (S_acc) S_acc[c] = s_acc_init ? cs.s : S_acc[c] * cs.s;
        }
    }
}

// ---------------------------------------------------------------------------
// CLE convergence metric: Cross_layer_equal.py:83,107-108
// ---------------------------------------------------------------------------
struct DiffLayer {
    float* w;
    float* snap;
    int64_t n;
    int64_t block0;   // first partial slot of this layer
    int64_t nblocks;
};
constexpr int kDiffPerBlock = 8192;

__global__ void diff_partial_kernel(const DiffLayer* __restrict__ layers, const int32_t* __restrict__ block_layer,
                                    int64_t nblk, double* __restrict__ partial) {
    __shared__ double red[kThreads / 64];
    for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const DiffLayer Ly = layers[block_layer[b]];
        const int64_t lo = (b - Ly.block0) * kDiffPerBlock;
        const int64_t hi = std::min<int64_t>(lo + kDiffPerBlock, Ly.n);
        double acc = 0.0;
        for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
            const float w = Ly.w[i];
            acc += (double)fabsf(w - Ly.snap[i]);
            Ly.snap[i] = w;
        }
        acc = wave_sum_d(acc);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int k = 0; k < (int)(blockDim.x / 64); ++k) t += red[k];
            partial[b] = t;
        }
        __syncthreads();
    }
}

__global__ void diff_final_kernel(const DiffLayer* __restrict__ layers, int32_t nl, const double* __restrict__ partial,
                                  double* __restrict__ out) {
    for (int l = blockIdx.x * blockDim.x + threadIdx.x; l < nl; l += gridDim.x * blockDim.x) {
        const DiffLayer Ly = layers[l];
        double t = 0.0;
        for (int64_t k = 0; k < Ly.nblocks; ++k) t += partial[Ly.block0 + k];   // fixed order
        out[l] = Ly.n > 0 ? (double)(float)(t / (double)Ly.n) : 0.0;
    }
}

__global__ void copy_kernel(const DiffLayer* __restrict__ layers, const int32_t* __restrict__ block_layer,
                            int64_t nblk) {
    for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const DiffLayer Ly = layers[block_layer[b]];
        const int64_t lo = (b - Ly.block0) * kDiffPerBlock;
        const int64_t hi = std::min<int64_t>(lo + kDiffPerBlock, Ly.n);
        for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) Ly.snap[i] = Ly.w[i];
    }
}

// ---------------------------------------------------------------------------
// High-bias absorption: bias_absorption.py:147-197
// ---------------------------------------------------------------------------
__device__ __forceinline__ float absorb_c(float beta, float gamma, float n_sigma) {
    float c = beta - n_sigma * gamma;   // bn_beta - N * bn_gamma
    return (c < 0.0f) ? 0.0f : c;       // clamp_(0), NaN kept
}

// b2[o] += sum_i (sum_k W2[o,i,k]) * c[g*i2 + i]: one wave per output row.
__global__ void absorb_gemv_kernel(const float* __restrict__ w2, float* __restrict__ b2,
                                   const float* __restrict__ bn_w, const float* __restrict__ bn_b,
                                   int64_t o2, int64_t i2, int64_t khw2, int64_t o2g, float n_sigma) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t o = wave; o < o2; o += nwaves) {
        const int64_t g = o / o2g;
        const float* row = w2 + o * i2 * khw2;
        float acc = 0.f;
        for (int64_t i = lane; i < i2; i += 64) {
            float ssum = 0.f;
            for (int64_t k = 0; k < khw2; ++k) ssum += row[i * khw2 + k];
            const int64_t ch = g * i2 + i;
            acc += ssum * absorb_c(bn_b[ch], bn_w[ch], n_sigma);
        }
        acc = wave_sum_f(acc);
        if (lane == 0) b2[o] = b2[o] + acc;
    }
}

__global__ void absorb_channel_kernel(float* __restrict__ b1, float* __restrict__ bn_b, const float* __restrict__ bn_w,
                                      int64_t c1, float n_sigma) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < c1; c += (int64_t)gridDim.x * blockDim.x) {
        const float cc = absorb_c(bn_b[c], bn_w[c], n_sigma);
        b1[c] = b1[c] + (-cc);
        bn_b[c] = bn_b[c] + (-cc);
    }
}

// ---------------------------------------------------------------------------
// Bias correction: bias_correction.py:15-106,170-172,206-213
// ---------------------------------------------------------------------------
// scipy.stats.norm: pdf = exp(-x^2/2)/sqrt(2 pi); cdf = cephes ndtr (erf below
// |x|/sqrt2 < 1/sqrt2, erfc above), both in float64 on the fp32 argument.
__device__ __forceinline__ double ndtr_d(double a) {
    const double x = a * 0.70710678118654752440;
    const double z = fabs(x);
    if (z < 0.70710678118654752440) return 0.5 + 0.5 * erf(x);
    const double y = 0.5 * erfc(z);
    return x > 0.0 ? 1.0 - y : y;
}

__global__ void bc_expect_kernel(const float* __restrict__ w, const float* __restrict__ b, int64_t n, int relu,
                                 int accumulate, float* __restrict__ out) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const float wj = w[j], bj = b[j];
        float ex;
        if (relu) {
            const float x = (-bj) / wj;               // -bias/weight (fp32)
            const double xd = (double)x;
            const float pdf = (float)(exp(-(xd * xd) / 2.0) / 2.5066282746310002);
            const float cdf = (float)ndtr_d(xd);
            ex = wj * pdf + bj * (1.0f - cdf);        // torch finishes in fp32
            if (ex < 0.0f) ex = 0.0f;                  // expect[expect < 0] = 0
        } else {
            ex = bj;
        }
        out[j] = accumulate ? out[j] + ex : ex;
    }
}

// One thread per output row: bias_vec[r, :] = E (+) expect, bias[r] += mean in
// ATen's order (bias.view(O, -1).mean(dim=1)).
__global__ void bc_apply_kernel(const float* __restrict__ E, int64_t o, int64_t i2, const float* __restrict__ ex,
                                int64_t f, int64_t bcols, float* __restrict__ bias, float* __restrict__ bias_vec) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < o; r += (int64_t)gridDim.x * blockDim.x) {
        auto get = [&](int64_t j) { return E[r * i2 + (i2 > 1 ? j : 0)] + ex[f > 1 ? j : 0]; };
        if (bias_vec)
            for (int64_t j = 0; j < bcols; ++j) bias_vec[r * bcols + j] = get(j);
        const float sum = aten_inner_sum(get, bcols);
        bias[r] = bias[r] + sum / (float)bcols;
    }
}

// One thread per BN channel: fake_b[c] += mean_r(-bias_vec[r*f + c]) in ATen's
// order for bias_prev.view(-1, F).mean(0) with `threads` intra-op threads.
__global__ void bc_propagate_kernel(const float* __restrict__ bias_vec, int64_t nrows, int64_t f, int threads,
                                    float* __restrict__ fake_b) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < f; c += (int64_t)gridDim.x * blockDim.x) {
        const float s = -aten_outer_col_sum(bias_vec, nrows, f, c, threads);   // sum(-v) == -sum(v) exactly
        fake_b[c] = fake_b[c] + s / (float)nrows;
    }
}

}  // namespace dfq

using namespace dfq;

// ============================================================================
// C ABI
// ============================================================================
extern "C" int dfq_bn_fold(float* w, float* bias, float* bn_w, float* bn_b, float* bn_mean, float* bn_var,
                           float* fake_w, float* fake_b, float eps, int64_t rows, int64_t row_len, void* stream) {
    if (!w || !bias || !bn_w || !bn_b || !bn_mean || !bn_var || rows < 0 || row_len < 0) return DFQ_ERR_INVALID;
    if (rows == 0) return DFQ_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(bn_fold_weight_kernel, dim3(blocks_for(rows * row_len, 4)), dim3(kThreads), 0, s,
                       w, bn_w, bn_var, eps, rows, row_len);
    DFQ_LAUNCH_CHECK();
    hipLaunchKernelGGL(bn_fold_channel_kernel, dim3(blocks_for(rows)), dim3(kThreads), 0, s,
                       bias, bn_w, bn_b, bn_mean, bn_var, fake_w, fake_b, eps, rows);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_clamp(float* w, int64_t n, float lo, float hi, void* stream) {
    if (!w || n < 0) return DFQ_ERR_INVALID;
    if (reinterpret_cast<uintptr_t>(w) % 16) return DFQ_ERR_INVALID;
    if (n == 0) return DFQ_OK;
    hipLaunchKernelGGL(clamp_kernel, dim3(blocks_for(n, 16)), dim3(kThreads), 0, static_cast<hipStream_t>(stream), w,
                       n, lo, hi);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" size_t dfq_cle_ws_bytes(int64_t c1) { return (size_t)(c1 > 0 ? c1 : 0) * 4 * sizeof(uint32_t); }

extern "C" int dfq_cle_relation(float* w1, float* w2, float* b1, float* bn_w, float* bn_b, int64_t c1, int64_t len1,
                                int64_t o2, int64_t i2, int64_t khw2, double s_min, double s_max, int32_t is_signed,
                                float eps, float* S, float* S_acc, int32_t s_acc_init, void* ws, size_t ws_bytes,
                                void* stream) {
    if (!w1 || !w2 || c1 <= 0 || len1 <= 0 || o2 <= 0 || i2 <= 0 || khw2 <= 0) return DFQ_ERR_INVALID;
    if (!ws || ws_bytes < dfq_cle_ws_bytes(c1)) return DFQ_ERR_WORKSPACE;
    // grouping as Cross_layer_equal.py:12-18
    int64_t groups = 1;
    if (c1 != i2) {
        groups = c1 / i2;
        if (groups <= 0 || groups * i2 != c1) return DFQ_ERR_SHAPE;
    }
    if (o2 % groups != 0) return DFQ_ERR_SHAPE;
    CleShape sh{c1, len1, o2, i2, khw2, groups, o2 / groups};
    hipStream_t s = static_cast<hipStream_t>(stream);
    uint32_t* mins = static_cast<uint32_t*>(ws);
    uint32_t* maxs = mins + 2 * c1;
    DFQ_HIP_CHECK(hipMemsetAsync(mins, 0xFF, sizeof(uint32_t) * 2 * c1, s));
    DFQ_HIP_CHECK(hipMemsetAsync(maxs, 0x00, sizeof(uint32_t) * 2 * c1, s));
    const int wave_blocks = (int)std::min<int64_t>(ceil_div(c1, kThreads / 64), 2048);
    hipLaunchKernelGGL(cle_range_w1_kernel, dim3(wave_blocks), dim3(kThreads), 0, s, w1, sh, mins, maxs);
    DFQ_LAUNCH_CHECK();
    if (i2 == 1) {
        hipLaunchKernelGGL(cle_range_w2_contig_kernel, dim3(wave_blocks), dim3(kThreads), 0, s, w2, sh, mins + c1,
                           maxs + c1);
    } else {
        const int nt = (int)std::min<int64_t>(ceil_div(o2, kColTileRows), 2048);
        hipLaunchKernelGGL(cle_range_w2_cols_kernel, dim3(nt), dim3(kThreads), 0, s, w2, sh, mins + c1, maxs + c1);
    }
    DFQ_LAUNCH_CHECK();
    const int64_t total = c1 * len1 + o2 * i2 * khw2 + c1;
    hipLaunchKernelGGL(cle_apply_kernel, dim3(blocks_for(total, 4)), dim3(kThreads), 0, s, w1, w2, b1, bn_w, bn_b,
                       S, S_acc, s_acc_init, sh, mins, maxs, is_signed, eps, s_min, s_max);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

struct dfq_diff_plan {
    DiffLayer* d_layers = nullptr;
    int32_t* d_block_layer = nullptr;
    double* d_partial = nullptr;
    double* d_out = nullptr;
    double* h_out = nullptr;   // pinned
    int32_t n = 0;
    int64_t nblk = 0;
};

extern "C" int dfq_diff_plan_create(float* const* w, float* const* snap, const int64_t* n, int32_t count,
                                    dfq_diff_plan** out) {
    if (!out || count < 0 || (count > 0 && (!w || !snap || !n))) return DFQ_ERR_INVALID;
    *out = nullptr;
    std::vector<DiffLayer> layers(count);
    std::vector<int32_t> block_layer;
    int64_t nb = 0;
    for (int32_t l = 0; l < count; ++l) {
        if (!w[l] || !snap[l] || n[l] < 0) return DFQ_ERR_INVALID;
        const int64_t k = ceil_div(n[l], kDiffPerBlock);
        layers[l] = DiffLayer{w[l], snap[l], n[l], nb, k};
        for (int64_t b = 0; b < k; ++b) block_layer.push_back(l);
        nb += k;
    }
    dfq_diff_plan* p = new (std::nothrow) dfq_diff_plan();
    if (!p) return DFQ_ERR_NOMEM;
    p->n = count;
    p->nblk = nb;
    auto fail = [&](hipError_t e) {
        set_last_hip_error(e);
        (void)hipFree(p->d_layers); (void)hipFree(p->d_block_layer); (void)hipFree(p->d_partial); (void)hipFree(p->d_out);
        if (p->h_out) (void)hipHostFree(p->h_out);
        delete p;
        return DFQ_ERR_HIP;
    };
    hipError_t e;
    if ((e = hipMalloc(&p->d_layers, sizeof(DiffLayer) * std::max(count, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&p->d_block_layer, sizeof(int32_t) * std::max<int64_t>(nb, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&p->d_partial, sizeof(double) * std::max<int64_t>(nb, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&p->d_out, sizeof(double) * std::max(count, 1))) != hipSuccess) return fail(e);
    if ((e = hipHostMalloc(&p->h_out, sizeof(double) * std::max(count, 1))) != hipSuccess) return fail(e);
    if (count > 0 && (e = hipMemcpy(p->d_layers, layers.data(), sizeof(DiffLayer) * count, hipMemcpyHostToDevice)) != hipSuccess)
        return fail(e);
    if (nb > 0 && (e = hipMemcpy(p->d_block_layer, block_layer.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice)) != hipSuccess)
        return fail(e);
    *out = p;
    return DFQ_OK;
}

extern "C" int dfq_diff_plan_snapshot(dfq_diff_plan* p, void* stream) {
    if (!p) return DFQ_ERR_INVALID;
    if (p->nblk == 0) return DFQ_OK;
    hipLaunchKernelGGL(copy_kernel, dim3((int)std::min<int64_t>(p->nblk, 4096)), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), p->d_layers, p->d_block_layer, p->nblk);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_diff_plan_execute(dfq_diff_plan* p, double* out_mean, void* stream) {
    if (!p || (p->n > 0 && !out_mean)) return DFQ_ERR_INVALID;
    if (p->n == 0) return DFQ_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (p->nblk > 0) {
        hipLaunchKernelGGL(diff_partial_kernel, dim3((int)std::min<int64_t>(p->nblk, 4096)), dim3(kThreads), 0, s,
                           p->d_layers, p->d_block_layer, p->nblk, p->d_partial);
        DFQ_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(diff_final_kernel, dim3((int)ceil_div(p->n, kThreads)), dim3(kThreads), 0, s, p->d_layers, p->n,
                       p->d_partial, p->d_out);
    DFQ_LAUNCH_CHECK();
    DFQ_HIP_CHECK(hipMemcpyAsync(p->h_out, p->d_out, sizeof(double) * p->n, hipMemcpyDeviceToHost, s));
    DFQ_HIP_CHECK(hipStreamSynchronize(s));
    for (int32_t l = 0; l < p->n; ++l) out_mean[l] = p->h_out[l];
    return DFQ_OK;
}

extern "C" int dfq_diff_plan_destroy(dfq_diff_plan* p) {
    if (!p) return DFQ_OK;
    (void)hipFree(p->d_layers); (void)hipFree(p->d_block_layer); (void)hipFree(p->d_partial); (void)hipFree(p->d_out);
    if (p->h_out) (void)hipHostFree(p->h_out);
    delete p;
    return DFQ_OK;
}

extern "C" int dfq_bias_absorb(const float* w2, float* b1, float* b2, float* bn_w, float* bn_b, int64_t c1,
                               int64_t o2, int64_t i2, int64_t khw2, float n_sigma, void* stream) {
    if (!w2 || !b1 || !b2 || !bn_w || !bn_b || c1 <= 0 || o2 <= 0 || i2 <= 0 || khw2 <= 0) return DFQ_ERR_INVALID;
    const int64_t groups = c1 / i2;   // bias_absorption.py:159
    if (groups <= 0 || o2 % groups != 0) return DFQ_ERR_SHAPE;
    const int64_t o2g = o2 / groups;
    if (groups * i2 > c1) return DFQ_ERR_SHAPE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int wave_blocks = (int)std::min<int64_t>(ceil_div(o2, kThreads / 64), 2048);
    hipLaunchKernelGGL(absorb_gemv_kernel, dim3(wave_blocks), dim3(kThreads), 0, s, w2, b2, bn_w, bn_b, o2, i2, khw2,
                       o2g, n_sigma);
    DFQ_LAUNCH_CHECK();
    hipLaunchKernelGGL(absorb_channel_kernel, dim3(blocks_for(c1)), dim3(kThreads), 0, s, b1, bn_b, bn_w, c1, n_sigma);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_bc_expect(const float* fake_w, const float* fake_b, int64_t n, int32_t relu, int32_t accumulate,
                             float* out, void* stream) {
    if (!fake_w || !fake_b || !out || n < 0) return DFQ_ERR_INVALID;
    if (n == 0) return DFQ_OK;
    hipLaunchKernelGGL(bc_expect_kernel, dim3(blocks_for(n)), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                       fake_w, fake_b, n, relu, accumulate, out);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_bc_apply(const float* E, int64_t o, int64_t i2, const float* expect, int64_t f, float* bias,
                            float* bias_vec, int64_t* bcols_out, void* stream) {
    if (!E || !expect || !bias || o <= 0 || i2 <= 0 || f <= 0) return DFQ_ERR_INVALID;
    // torch broadcasting of [o, i2] + [f]
    int64_t bcols;
    if (i2 == f || f == 1) bcols = i2;
    else if (i2 == 1) bcols = f;
    else return DFQ_ERR_SHAPE;
    if (bcols_out) *bcols_out = bcols;
    // _apply_bias_correction: sizes never equal (2-D vs 1-D); numel must exceed o
    if (o * bcols <= o) return DFQ_ERR_SHAPE;
    hipLaunchKernelGGL(bc_apply_kernel, dim3(blocks_for(o)), dim3(kThreads), 0, static_cast<hipStream_t>(stream), E,
                       o, i2, expect, f, bcols, bias, bias_vec);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_bc_propagate(const float* bias_vec, int64_t numel, float* fake_b, int64_t f, int32_t ref_threads,
                                void* stream) {
    if (!bias_vec || !fake_b || numel <= 0 || f <= 0 || ref_threads < 1) return DFQ_ERR_INVALID;
    if (numel % f != 0) return DFQ_ERR_SHAPE;   // .view(-1, F) fails
    hipLaunchKernelGGL(bc_propagate_kernel, dim3(blocks_for(f)), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                       bias_vec, numel / f, f, (int)ref_threads, fake_b);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}
