// Cross-layer equalization, one relation at a time (Cross_layer_equal.py:11-59):
// dfq_cle_relation (range kernels + rescale) and the dfq_diff_plan_* metric of
// the host-driven loop (Cross_layer_equal.py:83,107-108).  The device-resident
// loop (dfq_cle_plan_*) is in dfq_cle.hip.
#include "dfq_cle_common.h"

#include <algorithm>
#include <new>
#include <vector>

namespace dfq {

static int blocks_for(int64_t n, int per_thread = 1) {
    const int64_t b = ceil_div(std::max<int64_t>(n, 1), (int64_t)kThreads * per_thread);
    return (int)std::min<int64_t>(b, 256 * 8);
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
        cle_wave_minmax(vmin, vmax);
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
        cle_wave_minmax(vmin, vmax);
        if (lane == 0) {
            mins[c] = enc_ord(vmin);
            maxs[c] = enc_ord(vmax);
        }
    }
}

// i2 > 1: each block takes a tile of W2 rows; a thread owns column i and reduces it
// over the tile's rows, then one ordered-uint atomic per (block, column).
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

}  // namespace dfq

using namespace dfq;

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

