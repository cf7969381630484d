// Graph-transform kernels of the DFQ path (gfx950): BatchNorm folding, weight
// clipping, high-bias absorption and the
// bias-correction combine.  All are HBM/latency-bound elementwise or row/column
// reductions: no MFMA.  fp32 arithmetic is ordered exactly as the reference's
// torch CPU ops (one rounding per op; -ffp-contract=off, IEEE div/sqrt).
#include "dfq_common.h"

#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <mutex>
#include <new>
#include <string>
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

__device__ __forceinline__ float bc_expect_value(float wj, float bj, int relu) {
    if (!relu) return bj;
    const float x = (-bj) / wj;               // -bias/weight (fp32)
    const double xd = (double)x;
    const float pdf = (float)(exp(-(xd * xd) / 2.0) / 2.5066282746310002);
    const float cdf = (float)ndtr_d(xd);
    float ex = wj * pdf + bj * (1.0f - cdf);  // torch finishes in fp32
    if (ex < 0.0f) ex = 0.0f;                  // expect[expect < 0] = 0
    return ex;
}

__global__ void bc_expect_kernel(const float* __restrict__ w, const float* __restrict__ b, int64_t n, int relu,
                                 int accumulate, float* __restrict__ out) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const float ex = bc_expect_value(w[j], b[j], relu);
        out[j] = accumulate ? out[j] + ex : ex;
    }
}

// One wave per output row: bias_vec[r, :] = E (+) expect, bias[r] += mean in
// ATen's order (bias.view(O, -1).mean(dim=1)): the 32 (vector lane, ILP) streams
// of the row run on 32 lanes, the combine on lane 0 (wave_inner_sum).
__global__ void __launch_bounds__(kThreads)
bc_apply_kernel(const float* __restrict__ E, int64_t o, int64_t i2, const float* __restrict__ ex, int64_t f,
                int64_t bcols, float* __restrict__ bias, float* __restrict__ bias_vec) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (kThreads / 64);
    for (int64_t r = wave; r < o; r += nwaves) {
        auto get = [&](int64_t j) { return E[r * i2 + (i2 > 1 ? j : 0)] + ex[f > 1 ? j : 0]; };
        if (bias_vec)
            for (int64_t j = lane; j < bcols; j += 64) bias_vec[r * bcols + j] = get(j);
        const float sum = wave_inner_sum(get, bcols, lane);
        if (lane == 0) bias[r] = bias[r] + sum / (float)bcols;
    }
}

// One wave per BN channel: fake_b[c] += mean_r(-bias_vec[r*f + c]) in ATen's
// order for bias_prev.view(-1, F).mean(0) with `threads` intra-op threads (the
// column's cascade or ILP row_sum as a wave-parallel tree).
constexpr int64_t kBcScratch = 1024;
__global__ void __launch_bounds__(kThreads)
bc_propagate_kernel(const float* __restrict__ bias_vec, int64_t nrows, int64_t f, int threads,
                    float* __restrict__ fake_b) {
    __shared__ float scratch[kThreads / 64][kBcScratch + kBcScratch / 16];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    float* b0s = scratch[wv];
    float* b1s = b0s + kBcScratch;
    const int64_t wave = (int64_t)blockIdx.x * (kThreads / 64) + wv;
    const int64_t nwaves = (int64_t)gridDim.x * (kThreads / 64);
    for (int64_t c = wave; c < f; c += nwaves) {
        auto get = [&](int64_t r) { return bias_vec[r * f + c]; };
        const float sum = aten_outer_col_is_cascade(nrows, f, c, threads)
                              ? wave_cascade(get, nrows, lane, b0s, b1s, kBcScratch)
                              : wave_row_sum(get, nrows, lane, b0s, b1s, kBcScratch);
        if (lane == 0) fake_b[c] = fake_b[c] + (-sum) / (float)nrows;   // sum(-v) == -sum(v) exactly
    }
}



// One target layer of the bias-correction walk in ONE launch: the op group
// EXPECT+ -> APPLY (-> PROPAGATE) that dfq_bc_chain records per layer
// (bias_correction.py:170-172,196-213,231-251).  Every block first evaluates the
// layer's expectation vector (the branch's BN terms summed in op order) into
// LDS; blocks [0, apply_blocks) then take the APPLY rows (bias += mean_j
// (E (+) expect)[o, j], bias_vec written), the rest the PROPAGATE columns of
// bias_vec.view(-1, F) -- recomputing each element fl(E + expect) instead of
// reading what the apply blocks store, so the two run in the same launch.
// Same per-element values and the same reduction trees as bc_expect_kernel /
// bc_apply_kernel / bc_propagate_kernel: bit-identical, one dependent launch
// per layer instead of three (MobileNetV2: 173 -> 55 launches).
constexpr int kBcMaxTerms = 8;
constexpr int64_t kBcMaxExpect = 4096;
struct BcLayerJob {
    const float* ew[kBcMaxTerms];
    const float* eb[kBcMaxTerms];
    int32_t relu[kBcMaxTerms];
    int32_t nterms;
    int32_t threads;            // PROPAGATE: the reference run's intra-op threads
    float* expect_out;          // the EXPECT ops' slot (written by block 0, as they would)
    int64_t f;                  // expect numel
    const float* E;
    int64_t o, i2, bcols;
    float* bias;
    float* vec;                 // APPLY's bias_vec (may be null)
    float* fake_b;              // PROPAGATE target (null: no PROPAGATE in the group)
    int64_t F, nrows;
    int64_t apply_blocks;
};

// Rows / columns of at most kBcStage values are first staged into LDS by all 64
// lanes of the wave (independent loads in flight together), then summed in
// ATen's order from LDS: the order's lane-serial parts (cascade tails, the
// 32-stream inner sums) read LDS instead of issuing one dependent global load
// per element (a 96-row propagate column took ~50 us that way, DFQ trace
// profiles/r04/r04i_bc).
constexpr int64_t kBcStage = 2048;
__global__ void __launch_bounds__(kThreads) bc_layer_kernel(BcLayerJob J) {
    __shared__ float ex[kBcMaxExpect];
    __shared__ float scratch[kThreads / 64][kBcScratch + kBcScratch / 16];
    __shared__ float stage[kThreads / 64][kBcStage];
    for (int64_t j = threadIdx.x; j < J.f; j += kThreads) {
        float v = bc_expect_value(J.ew[0][j], J.eb[0][j], J.relu[0]);
        for (int t = 1; t < J.nterms; ++t) v = v + bc_expect_value(J.ew[t][j], J.eb[t][j], J.relu[t]);
        ex[j] = v;
        if (blockIdx.x == 0) J.expect_out[j] = v;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const bool ebc = J.i2 > 1, xbc = J.f > 1;
    if ((int64_t)blockIdx.x < J.apply_blocks) {
        const int64_t wave = (int64_t)blockIdx.x * (kThreads / 64) + wv;
        const int64_t nwaves = J.apply_blocks * (kThreads / 64);
        float* rowv = stage[wv];
        for (int64_t r = wave; r < J.o; r += nwaves) {
            auto get = [&](int64_t j) { return J.E[r * J.i2 + (ebc ? j : 0)] + ex[xbc ? j : 0]; };
            for (int64_t j = lane; j < J.bcols; j += 64) {   // bcols <= kBcStage (bc_layer_group)
                const float v = get(j);
                rowv[j] = v;
                if (J.vec) J.vec[r * J.bcols + j] = v;
            }
            wave_lds_sync();
            const float sum = wave_inner_sum([&](int64_t j) { return rowv[j]; }, J.bcols, lane);
            wave_lds_sync();   // rowv is rewritten by the next row
            if (lane == 0) J.bias[r] = J.bias[r] + sum / (float)J.bcols;
        }
        return;
    }
    float* b0s = scratch[wv];
    float* b1s = b0s + kBcScratch;
    const int64_t wave = ((int64_t)blockIdx.x - J.apply_blocks) * (kThreads / 64) + wv;
    const int64_t nwaves = ((int64_t)gridDim.x - J.apply_blocks) * (kThreads / 64);
    float* colv = stage[wv];
    for (int64_t c = wave; c < J.F; c += nwaves) {
        auto get = [&](int64_t r) {   // 32-bit index math: o * bcols < 2^31 (bc_layer_group)
            const uint32_t idx = (uint32_t)r * (uint32_t)J.F + (uint32_t)c;
            const uint32_t row = idx / (uint32_t)J.bcols, j = idx - row * (uint32_t)J.bcols;
            return J.E[(int64_t)row * J.i2 + (ebc ? j : 0)] + ex[xbc ? j : 0];
        };
        const bool cascade = aten_outer_col_is_cascade(J.nrows, J.F, c, J.threads);
        for (int64_t r = lane; r < J.nrows; r += 64) colv[r] = get(r);   // nrows <= kBcStage (bc_layer_group)
        wave_lds_sync();
        auto lds = [&](int64_t r) { return colv[r]; };
        const float sum = cascade ? wave_cascade(lds, J.nrows, lane, b0s, b1s, kBcScratch)
                                  : wave_row_sum(lds, J.nrows, lane, b0s, b1s, kBcScratch);
        wave_lds_sync();   // colv is rewritten by the next column
        if (lane == 0) J.fake_b[c] = J.fake_b[c] + (-sum) / (float)J.nrows;
    }
}

// ---------------------------------------------------------------------------
// Activation ranges from BN statistics: set_quant_minmax,
// utils/layer_transform.py:356-618.  Rectified-Gaussian moments with scipy's
// pdf / ndtr in float64 on the fp32 argument, every fp32 op in the reference's
// expression order (:396-410).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float std_pdf(float x) {
    const double xd = (double)x;
    return (float)(exp(-(xd * xd) / 2.0) / 2.5066282746310002);
}
__device__ __forceinline__ float std_cdf(float x) { return (float)ndtr_d((double)x); }

// kind 0: mean = b, var = w*w; 1: calculate_mean / calculate_var (ReLU);
// 2: calculate_mean_6 / calculate_var_6 (ReLU6).  sqrt_w: w := sqrt(w + eps)
// (torch.sqrt(var + eps)).  accumulate: mean += m, var += v.  mean/var may alias w/b.
__global__ void act_moments_kernel(const float* w_in, const float* b_in, int64_t n, int kind, int sqrt_w, float eps,
                                   int accumulate, float* mean, float* var) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const float w = sqrt_w ? sqrtf(w_in[j] + eps) : w_in[j];
        const float b = b_in[j];
        float m, v;
        if (kind == 0) {
            m = b;
            v = w * w;
        } else if (kind == 1) {
            const float x0 = (-b) / w;
            const float P0 = std_pdf(x0), C0 = std_cdf(x0);
            m = w * P0 + b * (1.0f - C0);
            const float B = ((b * b + w * w) + m * m) - (2.0f * m) * b;
            v = ((1.0f - C0) * B + (w * (b - 2.0f * m)) * P0) + (m * m) * C0;
        } else {
            const float x0 = (-b) / w, x6 = (6.0f - b) / w;
            const float P0 = std_pdf(x0), C0 = std_cdf(x0), P6 = std_pdf(x6), C6 = std_cdf(x6);
            m = (w * (P0 - P6) + b * (C6 - C0)) + 6.0f * (1.0f - C6);
            const float B = ((b * b + w * w) + m * m) - (2.0f * m) * b;
            const float d6 = 6.0f - m;
            v = ((((C6 - C0) * B + (w * -6.0f) * P6) + (w * (b - 2.0f * m)) * (P0 - P6)) + (m * m) * C0) +
                (d6 * d6) * (1.0f - C6);
        }
        if (accumulate) {
            m = mean[j] + m;
            v = var[j] + v;
        }
        mean[j] = m;
        var[j] = v;
    }
}

// out = {min(a - N*w), max(a + N*w)} (get_min_value / get_max_value, :391-392);
// w_is_var: w := sqrt(w + eps).  One block.
__global__ void act_minmax_kernel(const float* a, const float* w_in, int64_t n, int w_is_var, float eps, float nsig,
                                  float* out) {
    __shared__ float smin[4], smax[4];
    float vmin = INFINITY, vmax = -INFINITY;
    for (int64_t j = threadIdx.x; j < n; j += blockDim.x) {
        const float w = w_is_var ? sqrtf(w_in[j] + eps) : w_in[j];
        const float nw = nsig * w;
        vmin = fminf(vmin, a[j] - nw);
        vmax = fmaxf(vmax, a[j] + nw);
    }
    vmin = wave_min(vmin);
    vmax = wave_max(vmax);
    if ((threadIdx.x & 63) == 0) {
        smin[threadIdx.x >> 6] = vmin;
        smax[threadIdx.x >> 6] = vmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x / 64); ++k) {
            vmin = fminf(vmin, smin[k]);
            vmax = fmaxf(vmax, smax[k]);
        }
        out[0] = fminf(smin[0], vmin);
        out[1] = fmaxf(smax[0], vmax);
    }
}

// Case (d.) of set_quant_minmax (:470-481): a BN statistic vector pushed through a
// conv (weights summed over KH*KW, ATen order) or linear layer with its bias:
// out[o] = sum_i Wsum[o, i] * x[g*I + i] (+ bias[o]).  One wave per output.
__global__ void act_affine_kernel(const float* x, const float* w, const float* bias, int64_t o, int64_t i2,
                                  int64_t khw, int64_t og, float* out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t r = wave; r < o; r += nwaves) {
        const int64_t g = r / og;
        float acc = 0.f;
        for (int64_t i = lane; i < i2; i += 64) {
            const float* p = w + (r * i2 + i) * khw;
            const float ws = khw == 1 ? p[0] : aten_inner_sum([&](int64_t k) { return p[k]; }, khw);
            acc += ws * x[g * i2 + i];
        }
        acc = wave_sum_f(acc);
        if (lane == 0) out[r] = bias ? acc + bias[r] : acc;
    }
}


// Batched BN fold: every (BN, producer layer) pair of a model in two launches.
struct BnFoldJob {
    float* w;
    float* bias;
    float* g;
    float* b;
    float* m;
    float* v;
    float* fake_w;
    float* fake_b;
    float eps;
    int32_t flags;    // DFQ_BN_FOLD_ZERO_BIAS
    int64_t rows, row_len;
    uint32_t* range_enc;
};
struct BnFoldChunk {
    int32_t job;
    int32_t pad;
    int64_t e0, e1;   // element range of the job's weight
};

// The fold factor of row o (bn_factor), without the divide and square root for
// an identity BatchNorm (weight 1, var + eps == 1: the factor is exactly 1).
__device__ __forceinline__ float fold_factor(const BnFoldJob& J, int64_t o) {
    const float go = ((const DFQ_GLOBAL float*)J.g)[o], ve = ((const DFQ_GLOBAL float*)J.v)[o] + J.eps;
    return (go == 1.0f && ve == 1.0f) ? 1.0f : go / sqrtf(ve);
}

// w <- w * factor(row) over one chunk; w * 1 == w, so a factor of exactly 1
// (merge_batchnorm #2, whose BN is the identity the first fold left) rewrites
// nothing.  Row of element i: chunk-local index times 1/row_len in fp32, exact
// after a +-1 correction (chunk-local indices stay below 2^24).
__device__ __forceinline__ int64_t fold_row(const BnFoldJob& J, int64_t r0, int64_t base, float inv, int64_t i,
                                            int* rem_out) {
    const int li = (int)(i - base);
    const int len = (int)J.row_len;
    int q = (int)((float)li * inv);
    int rem = li - q * len;
    if (rem < 0) {
        --q;
        rem += len;
    } else if (rem >= len) {
        ++q;
        rem -= len;
    }
    *rem_out = rem;
    return r0 + q;
}

__device__ __forceinline__ float fold_one(const BnFoldJob& J, int64_t r0, int64_t base, float inv, int64_t i,
                                          float w) {
    int rem;
    const float f = fold_factor(J, fold_row(J, r0, base, inv, i, &rem));
    return f != 1.0f ? w * f : w;
}

__global__ void __launch_bounds__(kThreads)
bn_fold_weight_batch_kernel(const BnFoldJob* __restrict__ jobs, const BnFoldChunk* __restrict__ chunks,
                            int64_t nchunks) {
    __shared__ float smn[kThreads / kWave], smx[kThreads / kWave];
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const BnFoldChunk ch = chunks[c];
        const BnFoldJob J = jobs[ch.job];
        const int64_t r0 = ch.e0 / J.row_len, base = r0 * J.row_len;
        const float inv = 1.0f / (float)J.row_len;
        float a = INFINITY, b = -INFINITY;
        const int64_t n = ch.e1 - ch.e0;
        int64_t done = 0;
        // every row of the chunk with a factor of exactly 1 (merge_batchnorm #2): a
        // read-only stream for the range, 4 x 16 B in flight per thread
        int ident = 1;
        for (int64_t r = r0 + threadIdx.x; r <= (ch.e1 - 1) / J.row_len; r += blockDim.x)
            ident &= fold_factor(J, r) == 1.0f;
        ident = __syncthreads_and(ident);
        if (ident && (reinterpret_cast<uintptr_t>(J.w + ch.e0) & 15) == 0) {
            const DFQ_GLOBAL f32x4* w4 = (const DFQ_GLOBAL f32x4*)(J.w + ch.e0);   // global, not flat
            const int64_t n4 = n >> 2;
            for (int64_t k = threadIdx.x; k < n4; k += 4 * (int64_t)blockDim.x) {
                f32x4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k + u * (int64_t)blockDim.x < n4) v[u] = w4[k + u * blockDim.x];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k + u * (int64_t)blockDim.x < n4) {
                        a = fminf(a, fminf(fminf(v[u].x, v[u].y), fminf(v[u].z, v[u].w)));
                        b = fmaxf(b, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)));
                    }
            }
            done = 4 * n4;
        } else if ((reinterpret_cast<uintptr_t>(J.w + ch.e0) & 15) == 0) {   // 16-B groups
            DFQ_GLOBAL f32x4* w4 = (DFQ_GLOBAL f32x4*)(J.w + ch.e0);
            const int64_t n4 = n >> 2;
            for (int64_t k = threadIdx.x; k < n4; k += blockDim.x) {
                const f32x4 v = w4[k];
                const int64_t i = ch.e0 + 4 * k;
                f32x4 o;
                int rem;
                const float f = fold_factor(J, fold_row(J, r0, base, inv, i, &rem));
                if (rem + 3 < (int)J.row_len) {   // the 4 elements share a row: one factor
                    o.x = f != 1.0f ? v.x * f : v.x;
                    o.y = f != 1.0f ? v.y * f : v.y;
                    o.z = f != 1.0f ? v.z * f : v.z;
                    o.w = f != 1.0f ? v.w * f : v.w;
                } else {
                    o.x = f != 1.0f ? v.x * f : v.x;
                    o.y = fold_one(J, r0, base, inv, i + 1, v.y);
                    o.z = fold_one(J, r0, base, inv, i + 2, v.z);
                    o.w = fold_one(J, r0, base, inv, i + 3, v.w);
                }
                if (__float_as_uint(o.x) != __float_as_uint(v.x) || __float_as_uint(o.y) != __float_as_uint(v.y) ||
                    __float_as_uint(o.z) != __float_as_uint(v.z) || __float_as_uint(o.w) != __float_as_uint(v.w))
                    w4[k] = o;
                a = fminf(a, fminf(fminf(o.x, o.y), fminf(o.z, o.w)));
                b = fmaxf(b, fmaxf(fmaxf(o.x, o.y), fmaxf(o.z, o.w)));
            }
            done = 4 * n4;
        }
        DFQ_GLOBAL float* wg = (DFQ_GLOBAL float*)J.w;
        for (int64_t k = done + threadIdx.x; k < n; k += blockDim.x) {
            const int64_t i = ch.e0 + k;
            const float v = wg[i];
            const float o = fold_one(J, r0, base, inv, i, v);
            if (__float_as_uint(o) != __float_as_uint(v)) wg[i] = o;
            a = fminf(a, o);
            b = fmaxf(b, o);
        }
        if (J.range_enc) {   // the folded weight's (min, max), dfq_range's encoding
            a = wave_min(a);
            b = wave_max(b);
            const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
            if (lane == 0) {
                smn[wv] = a;
                smx[wv] = b;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                for (int k = 1; k < kThreads / kWave; ++k) {
                    a = fminf(a, smn[k]);
                    b = fmaxf(b, smx[k]);
                }
                atomicMax(&J.range_enc[0], ~enc_ord(a));
                atomicMax(&J.range_enc[1], enc_ord(b));
            }
            __syncthreads();   // smn / smx are rewritten by the next chunk
        }
    }
}

// One block per job: the per-channel bias / fake-stat / BN-reset update (after
// every weight has used the old BN parameters: a separate launch).
__global__ void bn_fold_channel_batch_kernel(const BnFoldJob* __restrict__ jobs, int32_t njobs) {
    for (int32_t j = blockIdx.x; j < njobs; j += gridDim.x) {
        const BnFoldJob J = jobs[j];
        typedef DFQ_GLOBAL float* G;   // global, not flat
        const G g = (G)J.g, b = (G)J.b, m = (G)J.m, v = (G)J.v, bias = (G)J.bias, fw = (G)J.fake_w, fb = (G)J.fake_b;
        for (int64_t o = threadIdx.x; o < J.rows; o += blockDim.x) {
            const float go = g[o], bo = b[o], mo = m[o], vo = v[o];
            const float f = bn_factor(go, vo, J.eps);
            const float shift = bo - (go * mo) / sqrtf(vo + J.eps);
            // a layer without a bias gets torch.zeros first (layer_transform.py:262-263)
            const float b0 = (J.flags & DFQ_BN_FOLD_ZERO_BIAS) ? 0.0f : bias[o];
            bias[o] = b0 * f + shift;
            if (J.fake_w) fw[o] = fabsf(go);
            if (J.fake_b) fb[o] = bo;
            g[o] = 1.0f;
            v[o] = 1.0f;
            b[o] = 0.0f;
            m[o] = 0.0f;
        }
    }
}

// ---------------------------------------------------------------------------
// Activation fake quant with a given range (QuantMeasure.forward at inference,
// utils/quantize.py:112-126 -> quantize(input, b, float(min), float(max))):
// elementwise, async, no workspace.  The range may live in device memory (the
// observer's running_min / running_max), read as the exact doubles float()
// would produce, so no host round trip is needed.
// ---------------------------------------------------------------------------
// A NaN element stays NaN (torch's clamp_ propagates it; qdq's fminf / fmaxf
// clamp would map it to qmin).
__device__ __forceinline__ float qdq_nan(float x, const QParams& p, float& q) {
    const float y = qdq(x, p, q);
    return x != x ? x : y;
}

__global__ void __launch_bounds__(kThreads)
fq_given_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, int bits, int sym, int flags,
                const float* __restrict__ min_dev, const float* __restrict__ max_dev,
                const uint32_t* __restrict__ range_enc, double gmin, double gmax, int vec4) {
    if (min_dev) gmin = (double)min_dev[0];
    if (max_dev) gmax = (double)max_dev[0];
    if (range_enc) {   // dfq_range's {~enc(min), enc(max)}
        gmin = (double)dec_ord(~range_enc[0]);
        gmax = (double)dec_ord(range_enc[1]);
    }
    const QParams p = make_qparams((float)gmin, (float)gmax, bits, sym != 0, flags | DFQ_GIVEN_RANGE, gmin, gmax);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float q;
    if (vec4) {
        const int64_t n4 = n >> 2;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
            const float4 v = reinterpret_cast<const float4*>(x)[i];
            float4 o;
            o.x = qdq_nan(v.x, p, q);
            o.y = qdq_nan(v.y, p, q);
            o.z = qdq_nan(v.z, p, q);
            o.w = qdq_nan(v.w, p, q);
            reinterpret_cast<float4*>(y)[i] = o;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
            y[i] = qdq_nan(x[i], p, q);
    }
}

// ---------------------------------------------------------------------------
// The Quant* layers' weight / bias fake quant in one call (dfq_fake_quant_tensor):
// y = quantize(x, b, float(x.min()), float(x.max())) -- the given-range fake quant
// of fq_given_kernel on the tensor's own range, without the fill and the separate
// range launch of dfq_range.  words[8]: caller scratch, zero once; every call leaves
// it armed again.
// ---------------------------------------------------------------------------
constexpr int64_t kFqSmall = 16384;   // one workgroup does range and fake quant

// One workgroup: the range (fminf / fmaxf, as range_enc_kernel), then the fake quant.
__global__ void __launch_bounds__(kThreads)
fq_tensor_small_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, int bits, int sym, int flags) {
    __shared__ float smn[kThreads / kWave], smx[kThreads / kWave];
    float a = INFINITY, b = -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += kThreads) {
        const float v = x[i];
        a = fminf(a, v);
        b = fmaxf(b, v);
    }
    a = wave_min(a);
    b = wave_max(b);
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
    if (lane == 0) {
        smn[w] = a;
        smx[w] = b;
    }
    __syncthreads();
    for (int k = 0; k < kThreads / kWave; ++k) {   // every thread combines (same order as thread 0's)
        a = k ? fminf(a, smn[k]) : smn[0];
        b = k ? fmaxf(b, smx[k]) : smx[0];
    }
    // the range as dfq_range's encoding would give it back (the same float, read as a double)
    const double gmin = (double)dec_ord(~(~enc_ord(a))), gmax = (double)dec_ord(enc_ord(b));
    const QParams p = make_qparams((float)gmin, (float)gmax, bits, sym != 0, flags | DFQ_GIVEN_RANGE, gmin, gmax);
    float q;
    for (int64_t i = threadIdx.x; i < n; i += kThreads) y[i] = qdq_nan(x[i], p, q);
}

// Range launch of large tensors: range_enc_kernel's accumulation into words[0..1];
// each block's atomics return before its arrival on words[2] (returning atomics:
// the wave waits for them), and the last block to arrive takes the range with
// atomic exchanges (re-arming words[0..1]), publishes it in words[4..5] for the
// fake-quant launch and re-arms the counter.
__global__ void __launch_bounds__(kThreads)
fq_tensor_range_kernel(const float* __restrict__ x, int64_t n, uint32_t* __restrict__ words) {
    __shared__ float smn[kThreads / kWave], smx[kThreads / kWave];
    float a = INFINITY, b = -INFINITY;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = x[i];
        a = fminf(a, v);
        b = fmaxf(b, v);
    }
    a = wave_min(a);
    b = wave_max(b);
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
    if (lane == 0) {
        smn[w] = a;
        smx[w] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kThreads / kWave; ++k) {
            a = fminf(a, smn[k]);
            b = fmaxf(b, smx[k]);
        }
        const uint32_t o0 = __hip_atomic_fetch_max(&words[0], ~enc_ord(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t o1 = __hip_atomic_fetch_max(&words[1], enc_ord(b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(o0), "v"(o1) : "memory");   // both performed before the arrival
        const uint32_t last = gridDim.x - 1;
        if (__hip_atomic_fetch_add(&words[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == last) {
            const uint32_t r0 = __hip_atomic_exchange(&words[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t r1 = __hip_atomic_exchange(&words[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            words[4] = r0;
            words[5] = r1;
            __hip_atomic_exchange(&words[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Whole-tensor (min, max) as order-preserving uints: {max ~enc(x), max enc(x)}, so
// one zero memset initialises both words (exact, order-independent).
__global__ void __launch_bounds__(kThreads)
range_enc_kernel(const float* __restrict__ x, int64_t n, uint32_t* __restrict__ enc) {
    __shared__ float smn[kThreads / kWave], smx[kThreads / kWave];
    float a = INFINITY, b = -INFINITY;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = x[i];
        a = fminf(a, v);
        b = fmaxf(b, v);
    }
    a = wave_min(a);
    b = wave_max(b);
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
    if (lane == 0) {
        smn[w] = a;
        smx[w] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kThreads / kWave; ++k) {
            a = fminf(a, smn[k]);
            b = fmaxf(b, smx[k]);
        }
        atomicMax(&enc[0], ~enc_ord(a));
        atomicMax(&enc[1], enc_ord(b));
    }
}

// ---------------------------------------------------------------------------
// quantize()'s data range with num_chunks (utils/quantize.py:26-37):
// y = x.view(rows, -1); min = y.min(-1)[0].mean(-1), max likewise (fp32).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads)
chunk_row_range_kernel(const float* __restrict__ x, int64_t rows, int64_t row_len, float* __restrict__ mins,
                       float* __restrict__ maxs) {
    __shared__ float smn[kThreads / kWave], smx[kThreads / kWave];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
        const float* row = x + r * row_len;
        float a = INFINITY, b = -INFINITY;
        for (int64_t i = threadIdx.x; i < row_len; i += kThreads) {
            const float v = row[i];
            a = fminf(a, v);
            b = fmaxf(b, v);
        }
        a = wave_min(a);
        b = wave_max(b);
        if (lane == 0) {
            smn[w] = a;
            smx[w] = b;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < kThreads / kWave; ++k) {
                a = fminf(a, smn[k]);
                b = fmaxf(b, smx[k]);
            }
            mins[r] = a;
            maxs[r] = b;
        }
        __syncthreads();
    }
}

// One wave: torch.mean over the rows' mins / maxs in ATen's order (sum, then / n).
__global__ void chunk_mean_kernel(const float* __restrict__ mins, const float* __restrict__ maxs, int64_t rows,
                                  float* __restrict__ out2) {
    const int lane = threadIdx.x;
    const float smn = wave_inner_sum([&](int64_t i) { return mins[i]; }, rows, lane);
    const float smx = wave_inner_sum([&](int64_t i) { return maxs[i]; }, rows, lane);
    if (lane == 0) {
        out2[0] = smn / (float)rows;
        out2[1] = smx / (float)rows;
    }
}

// ---------------------------------------------------------------------------
// QuantMeasure.forward's statistics (utils/quantize.py:94-126) in two launches
// instead of ~8 torch ops: the rows' (min, max) of x.view(rows, -1) by a 2-D grid
// (each block a slice of one row, ordered-uint atomics into a per-observer word
// pair), then one wave takes the rows' means in ATen's order and applies the
// observer's updates.  The word pairs are re-armed by that wave (self-cleaning:
// the host arms them once when it allocates them).
// ---------------------------------------------------------------------------
//
// NaN: torch's min / max propagate it, so a slice holding one stores the words of
// -NaN (min) and +NaN (max) -- the largest values of both ordered encodings, so
// the atomics keep them -- and the rows' means, the momentum update and the
// fake-quant range come out NaN as in the reference.
__global__ void __launch_bounds__(kThreads)
observe_rows_kernel(const float* __restrict__ x, int64_t rows, int64_t row_len, int64_t slices,
                    uint32_t* __restrict__ words) {
    __shared__ float smn[kThreads / kWave], smx[kThreads / kWave];
    __shared__ int snan[kThreads / kWave];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
    const int64_t per = ceil_div(row_len, slices);
    for (int64_t b = blockIdx.x; b < rows * slices; b += gridDim.x) {
        const int64_t r = b / slices, k = b % slices;
        const int64_t e0 = k * per, e1 = min(row_len, e0 + per);
        const float* row = x + r * row_len;
        float a = INFINITY, c = -INFINITY;
        bool nan = false;
        const bool v4 = (row_len % 4 == 0) && (per % 4 == 0) && (reinterpret_cast<uintptr_t>(x) % 16 == 0);
        if (v4) {
            const float4* q = reinterpret_cast<const float4*>(row + e0);
            for (int64_t i = threadIdx.x; i < (e1 - e0) / 4; i += kThreads) {
                const float4 v = q[i];
                a = fminf(a, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
                c = fmaxf(c, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
                nan |= (v.x != v.x) | (v.y != v.y) | (v.z != v.z) | (v.w != v.w);
            }
        } else {
            for (int64_t i = e0 + threadIdx.x; i < e1; i += kThreads) {
                const float v = row[i];
                a = fminf(a, v);
                c = fmaxf(c, v);
                nan |= (v != v);
            }
        }
        a = wave_min(a);
        c = wave_max(c);
        const bool wnan = __ballot(nan) != 0;
        if (lane == 0) {
            smn[w] = a;
            smx[w] = c;
            snan[w] = wnan ? 1 : 0;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int anynan = snan[0];
            for (int q = 1; q < kThreads / kWave; ++q) {
                a = fminf(a, smn[q]);
                c = fmaxf(c, smx[q]);
                anynan |= snan[q];
            }
            if (anynan) {
                a = __uint_as_float(0xFFC00000u);   // -NaN: enc_ord's smallest, so ~enc wins atomicMax
                c = __uint_as_float(0x7FC00000u);   // +NaN: enc_ord's largest
            }
            atomicMax(&words[2 * r], ~enc_ord(a));
            atomicMax(&words[2 * r + 1], enc_ord(c));
        }
        __syncthreads();
    }
}

// One wave.  mn / mx = the means of the rows' mins / maxs (fp32, ATen's sum order,
// as flat.min(-1)[0].mean()).  update_stat: running_max = mx if mx > running_max
// (Python max on tensors), running_min likewise; training: running_* =
// running_* * (1 - m) + (mn|mx) * m, each op rounded to fp32 as the in-place torch
// ops do.  out2 = the range the fake quant uses: (mn, mx) in training, the running
// values otherwise.
__global__ void observe_finish_kernel(uint32_t* __restrict__ words, int64_t rows, float* __restrict__ running_min,
                                      float* __restrict__ running_max, int32_t update_stat, int32_t training,
                                      float one_minus_m, float m, float* __restrict__ out2) {
    const int lane = threadIdx.x;
    const float smn = wave_inner_sum([&](int64_t i) { return dec_ord(~words[2 * i]); }, rows, lane);
    const float smx = wave_inner_sum([&](int64_t i) { return dec_ord(words[2 * i + 1]); }, rows, lane);
    __syncthreads();   // every lane has read the words
    for (int64_t i = lane; i < 2 * rows; i += kWave) words[i] = 0u;   // re-armed for the next call
    if (lane == 0) {
        const float mn = smn / (float)rows, mx = smx / (float)rows;
        float rmn = *running_min, rmx = *running_max;
        if (update_stat) {
            rmx = (mx > rmx) ? mx : rmx;
            rmn = (mn < rmn) ? mn : rmn;
        }
        if (training) {
            const float t0 = rmn * one_minus_m, t1 = mn * m;
            rmn = t0 + t1;
            const float t2 = rmx * one_minus_m, t3 = mx * m;
            rmx = t2 + t3;
        }
        *running_min = rmn;
        *running_max = rmx;
        out2[0] = training ? mn : rmn;
        out2[1] = training ? mx : rmx;
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

// Up to kClampBatch weights per launch, the batch in the kernel arguments
// (blockIdx.y picks the tensor; each is 16-B aligned, float4 body + scalar tail).
constexpr int kClampBatch = 64;
struct ClampBatch {
    float* w[kClampBatch];
    int64_t n[kClampBatch];
};

__global__ void __launch_bounds__(kThreads) clamp_batch_kernel(ClampBatch b, float lo, float hi) {
    float* __restrict__ w = b.w[blockIdx.y];
    const int64_t n = b.n[blockIdx.y];
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

extern "C" int dfq_clamp_batch(float* const* w, const int64_t* n, int32_t count, float lo, float hi, void* stream) {
    if (count < 0 || (count > 0 && (!w || !n))) return DFQ_ERR_INVALID;
    for (int32_t k = 0; k < count; ++k)
        if (!w[k] || n[k] < 0 || reinterpret_cast<uintptr_t>(w[k]) % 16) return DFQ_ERR_INVALID;
    for (int32_t k0 = 0; k0 < count; k0 += kClampBatch) {
        ClampBatch b{};
        int cnt = 0;
        int64_t most = 0;
        for (int32_t k = k0; k < std::min(count, k0 + kClampBatch); ++k) {
            if (n[k] == 0) continue;
            b.w[cnt] = w[k];
            b.n[cnt] = n[k];
            most = std::max(most, n[k]);
            ++cnt;
        }
        if (cnt == 0) continue;
        hipLaunchKernelGGL(clamp_batch_kernel, dim3(blocks_for(most, 16), cnt), dim3(kThreads), 0,
                           static_cast<hipStream_t>(stream), b, lo, hi);
        DFQ_LAUNCH_CHECK();
    }
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

// ---- batched absorption ---------------------------------------------------
namespace dfq {
struct AbsRel {
    const float* w2;
    const float* bn_w;
    float* bn_b;
    int64_t o2, i2, khw2, o2g;
    int64_t wc;    // float offset of this relation's W2sum @ c in the scratch
};
struct AbsRows {   // GEMV task: rows [o0, o1) of relation r, one wave per row
    int32_t r;
    int32_t pad;
    int64_t o0, o1;
};
struct AbsVec {    // a bias vector and its update list
    float* b;
    int64_t n;
    int32_t op0, nops;
};
struct AbsOp {     // kind 0: b += wc[r]; kind 1: b -= c[r] and beta[r] -= c[r]
    int32_t kind;
    int32_t r;
};
struct AbsElems {  // bias walk task: elements [e0, e1) of vector v
    int32_t v;
    int32_t pad;
    int64_t e0, e1;
};

__global__ void absorb_batch_gemv_kernel(const AbsRel* __restrict__ rels, const AbsRows* __restrict__ tasks,
                                         int64_t ntasks, float* __restrict__ wc, float n_sigma) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t t = wave; t < ntasks; t += nwaves) {
        const AbsRows tk = tasks[t];
        const AbsRel R = rels[tk.r];
        for (int64_t o = tk.o0; o < tk.o1; ++o) {
            const int64_t g = o / R.o2g;
            const float* row = R.w2 + o * R.i2 * R.khw2;
            float acc = 0.f;
            for (int64_t i = lane; i < R.i2; i += 64) {
                float ssum = 0.f;
                for (int64_t k = 0; k < R.khw2; ++k) ssum += row[i * R.khw2 + k];
                const int64_t ch = g * R.i2 + i;
                acc += ssum * absorb_c(R.bn_b[ch], R.bn_w[ch], n_sigma);
            }
            acc = wave_sum_f(acc);
            if (lane == 0) wc[R.wc + o] = acc;
        }
    }
}

__global__ void absorb_batch_bias_kernel(const AbsRel* __restrict__ rels, const AbsVec* __restrict__ vecs,
                                         const AbsOp* __restrict__ ops, const AbsElems* __restrict__ tasks,
                                         int64_t ntasks, const float* __restrict__ wc, float n_sigma) {
    for (int64_t t = blockIdx.x; t < ntasks; t += gridDim.x) {
        const AbsElems tk = tasks[t];
        const AbsVec V = vecs[tk.v];
        for (int64_t e = tk.e0 + threadIdx.x; e < tk.e1; e += blockDim.x) {
            float b = V.b[e];
            for (int32_t q = 0; q < V.nops; ++q) {
                const AbsOp op = ops[V.op0 + q];
                const AbsRel& R = rels[op.r];
                if (op.kind == 0) {
                    b = b + wc[R.wc + e];
                } else {
                    const float cc = absorb_c(R.bn_b[e], R.bn_w[e], n_sigma);
                    b = b + (-cc);
                    R.bn_b[e] = R.bn_b[e] + (-cc);
                }
            }
            V.b[e] = b;
        }
    }
}

struct AbsTables {
    std::vector<AbsRel> rels;
    std::vector<AbsRows> rows;
    std::vector<AbsVec> vecs;
    std::vector<AbsOp> ops;
    std::vector<AbsElems> elems;
    int64_t wc_floats = 0;
};

static int absorb_tables(const dfq_absorb_desc* d, int32_t n, AbsTables& T, int32_t* failed) {
    // per bias vector, its updates in relation order
    std::vector<std::pair<float*, int64_t>> vlist;
    std::vector<std::vector<AbsOp>> vops;
    auto vec_of = [&](float* b, int64_t len) {
        for (size_t k = 0; k < vlist.size(); ++k)
            if (vlist[k].first == b) return (int32_t)k;
        vlist.push_back({b, len});
        vops.emplace_back();
        return (int32_t)vlist.size() - 1;
    };
    for (int32_t r = 0; r < n; ++r) {
        const dfq_absorb_desc& x = d[r];
        if (failed) *failed = r;
        if (!x.w2 || !x.b1 || !x.b2 || !x.bn_w || !x.bn_b || x.c1 <= 0 || x.o2 <= 0 || x.i2 <= 0 || x.khw2 <= 0)
            return DFQ_ERR_INVALID;
        const int64_t groups = x.c1 / x.i2;   // bias_absorption.py:159
        if (groups <= 0 || x.o2 % groups != 0 || groups * x.i2 > x.c1) return DFQ_ERR_SHAPE;
        if (x.b1 == x.b2) return DFQ_ERR_SHAPE;
        for (int32_t q = 0; q < r; ++q)   // a BN shared by two relations: the per-relation call keeps its order
            if (d[q].bn_b == x.bn_b) return DFQ_ERR_UNSUPPORTED;
        AbsRel R{x.w2, x.bn_w, x.bn_b, x.o2, x.i2, x.khw2, x.o2 / groups, T.wc_floats};
        T.wc_floats += ceil_div(x.o2, (int64_t)64) * 64;
        T.rels.push_back(R);
        for (int64_t o = 0; o < x.o2; o += 4) T.rows.push_back(AbsRows{r, 0, o, std::min<int64_t>(o + 4, x.o2)});
        // reference order inside a relation: b1 -= c (and beta), then b2 += wc
        const int32_t v1 = vec_of(x.b1, x.c1);
        if (vlist[v1].second != x.c1) return DFQ_ERR_SHAPE;
        vops[v1].push_back(AbsOp{1, r});
        const int32_t v2 = vec_of(x.b2, x.o2);
        if (vlist[v2].second != x.o2) return DFQ_ERR_SHAPE;
        vops[v2].push_back(AbsOp{0, r});
    }
    if (failed) *failed = -1;
    for (size_t k = 0; k < vlist.size(); ++k) {
        T.vecs.push_back(AbsVec{vlist[k].first, vlist[k].second, (int32_t)T.ops.size(), (int32_t)vops[k].size()});
        T.ops.insert(T.ops.end(), vops[k].begin(), vops[k].end());
        for (int64_t e = 0; e < vlist[k].second; e += 1024)
            T.elems.push_back(AbsElems{(int32_t)k, 0, e, std::min<int64_t>(e + 1024, vlist[k].second)});
    }
    return DFQ_OK;
}

struct AbsLayout {
    int64_t o_rels, o_rows, o_vecs, o_ops, o_elems, host, o_wc, total;
};
static AbsLayout absorb_layout(const AbsTables& T) {
    AbsLayout L{};
    int64_t o = 0;
    auto add = [&](int64_t bytes) {
        const int64_t at = o;
        o += ceil_div(std::max<int64_t>(bytes, 1), (int64_t)256) * 256;
        return at;
    };
    L.o_rels = add(sizeof(AbsRel) * T.rels.size());
    L.o_rows = add(sizeof(AbsRows) * T.rows.size());
    L.o_vecs = add(sizeof(AbsVec) * T.vecs.size());
    L.o_ops = add(sizeof(AbsOp) * T.ops.size());
    L.o_elems = add(sizeof(AbsElems) * T.elems.size());
    L.host = o;
    L.o_wc = add(sizeof(float) * T.wc_floats);
    L.total = o;
    return L;
}
}  // namespace dfq

extern "C" int64_t dfq_bias_absorb_ws_bytes(const dfq_absorb_desc* d, int32_t n) {
    if (n < 0 || (n > 0 && !d)) return -1;
    AbsTables T;
    if (absorb_tables(d, n, T, nullptr) != DFQ_OK) return -1;
    return absorb_layout(T).total;
}

extern "C" int dfq_bias_absorb_batch(const dfq_absorb_desc* d, int32_t n, float n_sigma, void* ws, int64_t ws_bytes,
                                     int32_t* failed, void* stream) {
    if (failed) *failed = -1;
    if (n < 0 || (n > 0 && !d)) return DFQ_ERR_INVALID;
    if (n == 0) return DFQ_OK;
    AbsTables T;
    const int rc = absorb_tables(d, n, T, failed);
    if (rc != DFQ_OK) return rc;
    const AbsLayout L = absorb_layout(T);
    if (!ws || ws_bytes < L.total || reinterpret_cast<uintptr_t>(ws) % 256 != 0) return DFQ_ERR_WORKSPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    char* base = static_cast<char*>(ws);
    std::vector<char> blob(L.host, 0);
    auto put = [&](int64_t off, const auto& v) {
        if (!v.empty()) std::memcpy(blob.data() + off, v.data(), sizeof(v[0]) * v.size());
    };
    put(L.o_rels, T.rels); put(L.o_rows, T.rows); put(L.o_vecs, T.vecs); put(L.o_ops, T.ops); put(L.o_elems, T.elems);
    DFQ_HIP_CHECK(stage_h2d(base, blob.data(), L.host, s));
    const AbsRel* dr = reinterpret_cast<const AbsRel*>(base + L.o_rels);
    float* wc = reinterpret_cast<float*>(base + L.o_wc);
    const int64_t nrow = (int64_t)T.rows.size(), nel = (int64_t)T.elems.size();
    hipLaunchKernelGGL(absorb_batch_gemv_kernel, dim3((int)std::min<int64_t>(ceil_div(nrow, kThreads / 64), 4096)),
                       dim3(kThreads), 0, s, dr, reinterpret_cast<const AbsRows*>(base + L.o_rows), nrow, wc, n_sigma);
    DFQ_LAUNCH_CHECK();
    hipLaunchKernelGGL(absorb_batch_bias_kernel, dim3((int)std::min<int64_t>(nel, 4096)), dim3(kThreads), 0, s, dr,
                       reinterpret_cast<const AbsVec*>(base + L.o_vecs), reinterpret_cast<const AbsOp*>(base + L.o_ops),
                       reinterpret_cast<const AbsElems*>(base + L.o_elems), nel, wc, n_sigma);
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
    hipLaunchKernelGGL(bc_apply_kernel, dim3((int)std::min<int64_t>(ceil_div(o, (int64_t)4), 2048)), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), E,
                       o, i2, expect, f, bcols, bias, bias_vec);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_bc_propagate(const float* bias_vec, int64_t numel, float* fake_b, int64_t f, int32_t ref_threads,
                                void* stream) {
    if (!bias_vec || !fake_b || numel <= 0 || f <= 0 || ref_threads < 1) return DFQ_ERR_INVALID;
    if (numel % f != 0) return DFQ_ERR_SHAPE;   // .view(-1, F) fails
    hipLaunchKernelGGL(bc_propagate_kernel, dim3((int)std::min<int64_t>(ceil_div(f, (int64_t)4), 2048)), dim3(kThreads),
                       0, static_cast<hipStream_t>(stream),
                       bias_vec, numel / f, f, (int)ref_threads, fake_b);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

// Up to kCopyBatch consecutive DFQ_BC_OP_COPY ops of a chain in one launch: the
// batch rides in the kernel arguments, blockIdx.y picks the copy.
constexpr int kCopyBatch = 64;   // 1.5 KB of kernel arguments
struct CopyBatch {
    const float* src[kCopyBatch];
    float*       dst[kCopyBatch];
    int64_t      n[kCopyBatch];
};

__global__ void __launch_bounds__(256) copy_batch_kernel(CopyBatch b) {
    const int k = blockIdx.y;
    const float* __restrict__ src = b.src[k];
    float* __restrict__ dst = b.dst[k];
    const int64_t n = b.n[k];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

namespace dfq {
namespace {
struct Span {
    uintptr_t lo, hi;
};
Span span(const void* p, int64_t floats) {
    const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
    return Span{lo, lo + 4 * (uintptr_t)std::max<int64_t>(floats, 0)};
}
bool overlap(const Span& x, const Span& y) { return x.lo < x.hi && y.lo < y.hi && x.lo < y.hi && y.lo < x.hi; }
}  // namespace

// ops[k..] as one layer group for bc_layer_kernel: EXPECT (plain) [+ EXPECT
// (accumulate) ...] into one slot, the APPLY reading that slot, and optionally
// the PROPAGATE of that APPLY's bias_vec right after it.  Returns the ops used,
// or 0 (the ops then run one launch each).  Fused only when no op of the group
// writes what another one reads (the launch has no order inside it).
int32_t bc_layer_group(const dfq_bc_op* ops, int32_t n_ops, int32_t k, BcLayerJob& J) {
    const dfq_bc_op& e0 = ops[k];
    if (e0.kind != DFQ_BC_OP_EXPECT || (e0.flag & 2) || e0.n <= 0 || e0.n > kBcMaxExpect) return 0;
    int32_t m = k;
    J.nterms = 0;
    while (m < n_ops && ops[m].kind == DFQ_BC_OP_EXPECT && ops[m].out == e0.out && ops[m].n == e0.n &&
           (m == k || (ops[m].flag & 2))) {
        if (J.nterms == kBcMaxTerms) return 0;
        J.ew[J.nterms] = ops[m].a;
        J.eb[J.nterms] = ops[m].b;
        J.relu[J.nterms] = ops[m].flag & 1;
        ++J.nterms;
        ++m;
    }
    if (m >= n_ops) return 0;
    const dfq_bc_op& ap = ops[m];
    if (ap.kind != DFQ_BC_OP_APPLY || ap.b != e0.out || ap.f != e0.n) return 0;
    if (!(ap.i2 == ap.f || ap.f == 1 || ap.i2 == 1)) return 0;   // the launches report the shape error
    J.f = e0.n;
    J.expect_out = e0.out;
    J.E = ap.a;
    J.o = ap.n;
    J.i2 = ap.i2;
    J.bcols = (ap.i2 == ap.f || ap.f == 1) ? ap.i2 : ap.f;
    // the kernel stages a row / column in LDS and indexes bias_vec in 32 bits;
    // larger ones take the per-op launches
    if (J.bcols > kBcStage || J.o * J.bcols >= (int64_t(1) << 31)) return 0;
    J.bias = ap.out;
    J.vec = ap.out2;
    J.apply_blocks = std::min<int64_t>(ceil_div(J.o, (int64_t)4), 2048);
    int32_t used = m - k + 1;
    const dfq_bc_op* pr = (m + 1 < n_ops) ? &ops[m + 1] : nullptr;
    if (pr && pr->kind == DFQ_BC_OP_PROPAGATE && ap.out2 && pr->a == ap.out2 && pr->n == J.o * J.bcols &&
        pr->f > 0 && pr->n % pr->f == 0 && pr->flag >= 1 && pr->n / pr->f <= kBcStage) {
        J.fake_b = pr->out;
        J.F = pr->f;
        J.nrows = pr->n / pr->f;
        J.threads = pr->flag;
        ++used;
    }
    // hazards: what the group writes (slot, bias, bias_vec, fake_b) vs what it reads
    // (BN stats, E) -- and the writes among themselves
    // (fixed-size span lists: this runs once per layer on the host, between launches)
    Span rd[2 * kBcMaxTerms + 3], wr[4];
    int nr = 0, nw = 0;
    for (int t = 0; t < J.nterms; ++t) {
        rd[nr++] = span(J.ew[t], J.f);
        rd[nr++] = span(J.eb[t], J.f);
    }
    rd[nr++] = span(J.E, J.o * (J.i2 > 1 ? J.i2 : 1));
    rd[nr++] = span(J.bias, J.o);   // bias[r] = bias[r] + ...
    wr[nw++] = span(J.expect_out, J.f);
    wr[nw++] = span(J.bias, J.o);
    if (J.vec) wr[nw++] = span(J.vec, J.o * J.bcols);
    if (J.fake_b) {
        wr[nw++] = span(J.fake_b, J.F);
        rd[nr++] = span(J.fake_b, J.F);
    }
    for (int a = 0; a < nw; ++a) {
        for (int b = 0; b < nr; ++b) {
            const bool same = (a == 1 && b == nr - (J.fake_b ? 2 : 1)) ||        // bias vs bias
                              (J.fake_b && a == nw - 1 && b == nr - 1);   // fake_b vs fake_b
            if (!same && overlap(wr[a], rd[b])) return 0;
        }
        for (int b = a + 1; b < nw; ++b)
            if (overlap(wr[a], wr[b])) return 0;
    }
    return used;
}
}  // namespace dfq

extern "C" int dfq_bc_chain(const dfq_bc_op* ops, int32_t n_ops, int32_t* failed_op, void* stream) {
    if (failed_op) *failed_op = -1;
    if (n_ops < 0 || (n_ops > 0 && !ops)) return DFQ_ERR_INVALID;
    auto fail = [&](int32_t k, int rc) {
        if (failed_op) *failed_op = k;
        return rc;
    };
    // validate everything first: a rejected op enqueues nothing
    for (int32_t k = 0; k < n_ops; ++k) {
        const dfq_bc_op& op = ops[k];
        switch (op.kind) {
            case DFQ_BC_OP_EXPECT:
                if (!op.a || !op.b || !op.out || op.n < 0) return fail(k, DFQ_ERR_INVALID);
                break;
            case DFQ_BC_OP_APPLY: {
                if (!op.a || !op.b || !op.out || op.n <= 0 || op.i2 <= 0 || op.f <= 0) return fail(k, DFQ_ERR_INVALID);
                const bool bcast = op.i2 == op.f || op.f == 1 || op.i2 == 1;
                const int64_t bcols = (op.i2 == op.f || op.f == 1) ? op.i2 : op.f;
                if (!bcast || op.n * bcols <= op.n) return fail(k, DFQ_ERR_SHAPE);
                break;
            }
            case DFQ_BC_OP_PROPAGATE:
                if (!op.a || !op.out || op.n <= 0 || op.f <= 0 || op.flag < 1) return fail(k, DFQ_ERR_INVALID);
                if (op.n % op.f != 0) return fail(k, DFQ_ERR_SHAPE);
                break;
            case DFQ_BC_OP_COPY:
                if (!op.a || !op.out || op.n < 0) return fail(k, DFQ_ERR_INVALID);
                break;
            default:
                return fail(k, DFQ_ERR_INVALID);
        }
    }
    if (n_ops == 0) return DFQ_OK;
    for (int32_t k = 0; k < n_ops; ++k) {
        const dfq_bc_op& op = ops[k];
        int rc = DFQ_OK;
        if (op.kind == DFQ_BC_OP_EXPECT) {   // a layer's EXPECT+ -> APPLY (-> PROPAGATE) group: one launch
            dfq::BcLayerJob J{};
            const int32_t used = dfq::bc_layer_group(ops, n_ops, k, J);
            if (used > 0) {
                const int64_t pb = J.fake_b ? std::min<int64_t>(ceil_div(J.F, (int64_t)4), 2048) : 0;
                hipLaunchKernelGGL(dfq::bc_layer_kernel, dim3((int)(J.apply_blocks + pb)), dim3(kThreads), 0,
                                   static_cast<hipStream_t>(stream), J);
                const hipError_t e = hipGetLastError();
                if (e != hipSuccess) {
                    dfq::set_last_hip_error(e);
                    return fail(k, DFQ_ERR_HIP);
                }
                k += used - 1;
                continue;
            }
        }
        if (op.kind == DFQ_BC_OP_COPY) {   // this copy and the ones right after it: one launch
            CopyBatch b{};
            int cnt = 0;
            int64_t most = 0;
            int32_t j = k;
            for (; j < n_ops && ops[j].kind == DFQ_BC_OP_COPY && cnt < kCopyBatch; ++j) {
                if (ops[j].n == 0) continue;
                b.src[cnt] = ops[j].a;
                b.dst[cnt] = ops[j].out;
                b.n[cnt] = ops[j].n;
                most = std::max(most, ops[j].n);
                ++cnt;
            }
            if (cnt > 0) {
                hipLaunchKernelGGL(copy_batch_kernel, dim3(blocks_for(most), cnt), dim3(256), 0,
                                   static_cast<hipStream_t>(stream), b);
                const hipError_t e = hipGetLastError();
                if (e != hipSuccess) {
                    dfq::set_last_hip_error(e);
                    return fail(k, DFQ_ERR_HIP);
                }
            }
            k = j - 1;
            continue;
        }
        if (op.kind == DFQ_BC_OP_EXPECT)
            rc = dfq_bc_expect(op.a, op.b, op.n, op.flag & 1, (op.flag >> 1) & 1, op.out, stream);
        else if (op.kind == DFQ_BC_OP_APPLY)
            rc = dfq_bc_apply(op.a, op.n, op.i2, op.b, op.f, op.out, op.out2, nullptr, stream);
        else
            rc = dfq_bc_propagate(op.a, op.n, op.out, op.f, op.flag, stream);
        if (rc != DFQ_OK) return fail(k, rc);
    }
    return DFQ_OK;
}

extern "C" int dfq_act_moments(const float* w, const float* b, int64_t n, int32_t kind, int32_t sqrt_w, float eps,
                               int32_t accumulate, float* mean, float* var, void* stream) {
    if (!w || !b || !mean || !var || n < 0 || kind < 0 || kind > 2) return DFQ_ERR_INVALID;
    if (n == 0) return DFQ_OK;
    hipLaunchKernelGGL(act_moments_kernel, dim3(blocks_for(n)), dim3(kThreads), 0, static_cast<hipStream_t>(stream), w,
                       b, n, (int)kind, (int)sqrt_w, eps, (int)accumulate, mean, var);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_act_minmax(const float* a, const float* w, int64_t n, int32_t w_is_var, float eps, float nsig,
                              float* out2, void* stream) {
    if (!a || !w || !out2 || n <= 0) return DFQ_ERR_INVALID;
    hipLaunchKernelGGL(act_minmax_kernel, dim3(1), dim3(kThreads), 0, static_cast<hipStream_t>(stream), a, w, n,
                       (int)w_is_var, eps, nsig, out2);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_act_affine(const float* x, const float* w, const float* bias, int64_t o, int64_t i2, int64_t khw,
                              int64_t groups, float* out, void* stream) {
    if (!x || !w || !out || o <= 0 || i2 <= 0 || khw <= 0 || groups <= 0 || o % groups) return DFQ_ERR_INVALID;
    hipLaunchKernelGGL(act_affine_kernel, dim3((int)std::min<int64_t>(ceil_div(o, (int64_t)4), 2048)), dim3(kThreads),
                       0, static_cast<hipStream_t>(stream), x, w, bias, o, i2, khw, o / groups, out);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

// Tables of one batched fold: the jobs, and 8192-element weight chunks.
// Elements per chunk (one block's work): 8192, or more for batches past 2^27
// elements so the chunk table stays small (<= ~16K chunks of 24 B).
static int64_t bn_fold_span(const dfq_bn_fold_desc* d, int32_t n) {
    int64_t total = 0;
    for (int32_t j = 0; j < n; ++j) total += d[j].rows * d[j].row_len;
    return std::min<int64_t>(std::max<int64_t>(8192, ceil_div(total, (int64_t)16384 * 8192) * 8192), 1 << 20);
}

static int bn_fold_tables(const dfq_bn_fold_desc* d, int32_t n, std::vector<BnFoldJob>& jobs,
                          std::vector<BnFoldChunk>& chunks) {
    const int64_t span = bn_fold_span(d, n);
    {   // each weight folded once per call (sequential semantics otherwise)
        std::vector<const float*> ws(n);
        for (int32_t j = 0; j < n; ++j) ws[j] = d[j].w;
        std::sort(ws.begin(), ws.end());
        if (std::adjacent_find(ws.begin(), ws.end()) != ws.end()) return DFQ_ERR_INVALID;
    }
    jobs.resize(n);
    for (int32_t j = 0; j < n; ++j) {
        const dfq_bn_fold_desc& x = d[j];
        if (!x.w || !x.bias || !x.bn_w || !x.bn_b || !x.bn_mean || !x.bn_var || x.rows < 0 || x.row_len < 0)
            return DFQ_ERR_INVALID;
        if (x.row_len > (int64_t(1) << 22)) return DFQ_ERR_UNSUPPORTED;   // fold_one's fp32 row map
        jobs[j] = BnFoldJob{x.w, x.bias, x.bn_w, x.bn_b, x.bn_mean, x.bn_var, x.fake_w, x.fake_b, x.eps, x.flags, x.rows,
                            x.row_len, x.range_enc};
        const int64_t ne = x.rows * x.row_len;
        for (int64_t e = 0; e < ne; e += span) chunks.push_back(BnFoldChunk{j, 0, e, std::min<int64_t>(e + span, ne)});
    }
    return DFQ_OK;
}

static int64_t round256(int64_t b) { return ceil_div(b, (int64_t)256) * 256; }

extern "C" int64_t dfq_bn_fold_ws_bytes(const dfq_bn_fold_desc* d, int32_t n) {
    if (n < 0 || (n > 0 && !d)) return -1;
    int64_t nchunks = 0;
    for (int32_t j = 0; j < n; ++j)
        if (d[j].rows < 0 || d[j].row_len < 0) return -1;
    const int64_t span = bn_fold_span(d, n);
    for (int32_t j = 0; j < n; ++j) nchunks += ceil_div(d[j].rows * d[j].row_len, span);
    return round256((int64_t)sizeof(BnFoldJob) * n) + round256((int64_t)sizeof(BnFoldChunk) * nchunks);
}

extern "C" int dfq_bn_fold_batch(const dfq_bn_fold_desc* d, int32_t n, void* ws, int64_t ws_bytes, void* stream) {
    if (n < 0 || (n > 0 && !d)) return DFQ_ERR_INVALID;
    if (n == 0) return DFQ_OK;
    std::vector<BnFoldJob> jobs;
    std::vector<BnFoldChunk> chunks;
    const int rc = bn_fold_tables(d, n, jobs, chunks);
    if (rc != DFQ_OK) return rc;
    const int64_t jb = round256((int64_t)sizeof(BnFoldJob) * n);
    const int64_t need = jb + round256((int64_t)sizeof(BnFoldChunk) * (int64_t)chunks.size());
    if (ws && (ws_bytes < need || reinterpret_cast<uintptr_t>(ws) % 256 != 0)) return DFQ_ERR_INVALID;
    hipStream_t s = static_cast<hipStream_t>(stream);
    void* own = nullptr;
    if (!ws) {   // no caller workspace: a private one, freed after a stream sync
        DFQ_HIP_CHECK(hipMalloc(&own, need));
        ws = own;
    }
    char* base = static_cast<char*>(ws);
    BnFoldJob* dj = reinterpret_cast<BnFoldJob*>(base);
    BnFoldChunk* dc = reinterpret_cast<BnFoldChunk*>(base + jb);
    // one staging blob, one copy
    std::vector<char> blob(need, 0);
    std::memcpy(blob.data(), jobs.data(), sizeof(BnFoldJob) * n);
    if (!chunks.empty()) std::memcpy(blob.data() + jb, chunks.data(), sizeof(BnFoldChunk) * chunks.size());
    hipError_t e = own ? hipMemcpyAsync(base, blob.data(), need, hipMemcpyHostToDevice, s)
                       : stage_h2d(base, blob.data(), need, s);
    // zero the range outputs: one memset per run of adjacent 2-word records
    std::vector<uint32_t*> rp;
    for (int32_t j = 0; j < n; ++j)
        if (d[j].range_enc) rp.push_back(d[j].range_enc);
    std::sort(rp.begin(), rp.end());
    for (size_t k = 0; k < rp.size() && e == hipSuccess;) {
        size_t m = k + 1;
        while (m < rp.size() && rp[m] == rp[m - 1] + 2) ++m;
        e = hipMemsetAsync(rp[k], 0, sizeof(uint32_t) * 2 * (m - k), s);
        k = m;
    }
    if (e == hipSuccess && !chunks.empty()) {
        hipLaunchKernelGGL(bn_fold_weight_batch_kernel, dim3((int)std::min<size_t>(chunks.size(), 4096)),
                           dim3(kThreads), 0, s, dj, dc, (int64_t)chunks.size());
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(bn_fold_channel_batch_kernel, dim3(std::min(n, 2048)), dim3(kThreads), 0, s, dj, n);
        e = hipGetLastError();
    }
    // Caller workspace: stream-ordered (pinned staging).  Private tables die with
    // this call: wait for the stream then.
    if (e == hipSuccess && own) e = hipStreamSynchronize(s);
    if (own) (void)hipFree(own);
    if (e != hipSuccess) {
        set_last_hip_error(e);
        return DFQ_ERR_HIP;
    }
    return DFQ_OK;
}

extern "C" int dfq_chunk_range(const float* x, int64_t rows, int64_t row_len, float* rowbuf, float* out2,
                               void* stream) {
    if (!x || !rowbuf || !out2 || rows < 1) return DFQ_ERR_INVALID;
    if (row_len < 1) return DFQ_ERR_SHAPE;   // torch: min over an empty dim raises
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int grid = (int)std::min<int64_t>(rows, 4096);
    hipLaunchKernelGGL(chunk_row_range_kernel, dim3(grid), dim3(kThreads), 0, s, x, rows, row_len, rowbuf,
                       rowbuf + rows);
    DFQ_LAUNCH_CHECK();
    hipLaunchKernelGGL(chunk_mean_kernel, dim3(1), dim3(kWave), 0, s, rowbuf, rowbuf + rows, rows, out2);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_act_observe(const float* x, int64_t rows, int64_t row_len, uint32_t* words, float* running_min,
                               float* running_max, int32_t update_stat, int32_t training, double momentum,
                               float* out2, void* stream) {
    if (!x || !words || !running_min || !running_max || !out2 || rows < 1) return DFQ_ERR_INVALID;
    if (row_len < 1) return DFQ_ERR_SHAPE;   // torch: min over an empty dim raises
    hipStream_t s = static_cast<hipStream_t>(stream);
    // slices of >= 16K elements per block, >= 1024 blocks when the tensor allows
    const int64_t slices = std::max<int64_t>(1, std::min<int64_t>(ceil_div(row_len, (int64_t)16384),
                                                                  ceil_div((int64_t)1024, rows)));
    const int grid = (int)std::min<int64_t>(rows * slices, 8192);
    hipLaunchKernelGGL(observe_rows_kernel, dim3(grid), dim3(kThreads), 0, s, x, rows, row_len, slices, words);
    DFQ_LAUNCH_CHECK();
    hipLaunchKernelGGL(observe_finish_kernel, dim3(1), dim3(kWave), 0, s, words, rows, running_min, running_max,
                       update_stat, training, (float)(1.0 - momentum), (float)momentum, out2);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_range(const float* x, int64_t n, uint32_t* range_enc, void* stream) {
    if (n < 1 || !x || !range_enc) return DFQ_ERR_INVALID;
    hipStream_t s = static_cast<hipStream_t>(stream);
    DFQ_HIP_CHECK(hipMemsetAsync(range_enc, 0, 2 * sizeof(uint32_t), s));
    const int grid = (int)std::min<int64_t>(ceil_div(n, (int64_t)kThreads * 8), 2048);
    hipLaunchKernelGGL(range_enc_kernel, dim3(std::max(grid, 1)), dim3(kThreads), 0, s, x, n, range_enc);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_fake_quant_tensor(const float* x, float* y, int64_t n, int32_t bits, int32_t symmetric,
                                     int32_t flags, uint32_t* words, void* stream) {
    if (n < 1 || !x || !y || bits < 2 || bits > 16) return DFQ_ERR_INVALID;
    if (flags & ~(DFQ_SCALE_F32)) return DFQ_ERR_INVALID;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (n <= kFqSmall) {
        hipLaunchKernelGGL(fq_tensor_small_kernel, dim3(1), dim3(kThreads), 0, s, x, y, n, bits, symmetric, flags);
        DFQ_LAUNCH_CHECK();
        return DFQ_OK;
    }
    if (!words) return DFQ_ERR_INVALID;
    const int grid = (int)std::min<int64_t>(ceil_div(n, (int64_t)kThreads * 8), 2048);
    hipLaunchKernelGGL(fq_tensor_range_kernel, dim3(std::max(grid, 1)), dim3(kThreads), 0, s, x, n, words);
    DFQ_LAUNCH_CHECK();
    const int vec4 = (n % 4 == 0) && (reinterpret_cast<uintptr_t>(x) % 16 == 0) &&
                     (reinterpret_cast<uintptr_t>(y) % 16 == 0);
    const int64_t work = vec4 ? n / 4 : n;
    const int g2 = (int)std::min<int64_t>(ceil_div(work, (int64_t)kThreads * 4), 16384);
    hipLaunchKernelGGL(fq_given_kernel, dim3(std::max(g2, 1)), dim3(kThreads), 0, s, x, y, n, bits, symmetric, flags,
                       nullptr, nullptr, static_cast<const uint32_t*>(words + 4), 0.0, 0.0, vec4);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

extern "C" int dfq_fake_quant_given(const float* x, float* y, int64_t n, int32_t bits, int32_t symmetric,
                                    int32_t flags, const float* min_dev, const float* max_dev,
                                    const uint32_t* range_enc, double given_min, double given_max, void* stream) {
    if (n < 0 || (n > 0 && (!x || !y)) || bits < 2 || bits > 16) return DFQ_ERR_INVALID;
    if (flags & ~(DFQ_SCALE_F32)) return DFQ_ERR_INVALID;
    if (n == 0) return DFQ_OK;
    const int vec4 = (n % 4 == 0) && (reinterpret_cast<uintptr_t>(x) % 16 == 0) &&
                     (reinterpret_cast<uintptr_t>(y) % 16 == 0);
    const int64_t work = vec4 ? n / 4 : n;
    const int grid = (int)std::min<int64_t>(ceil_div(work, (int64_t)kThreads * 4), 16384);
    hipLaunchKernelGGL(fq_given_kernel, dim3(std::max(grid, 1)), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                       x, y, n, bits, symmetric, flags, min_dev, max_dev, range_enc, given_min, given_max, vec4);
    DFQ_LAUNCH_CHECK();
    return DFQ_OK;
}

namespace dfq {
hipError_t preload_transform() {   // see dfq_preload
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(bn_fold_weight_batch_kernel));
    if (e == hipSuccess) e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(absorb_batch_gemv_kernel));
    return e;
}
}  // namespace dfq
