// Device helpers shared by the per-relation CLE kernels (dfq_cle_relation.hip)
// and the device-resident loop (dfq_cle.hip): Cross_layer_equal.py:11-59.
#pragma once
#include "dfq_common.h"

namespace dfq {

constexpr int kThreads = 256;
constexpr int kColTileRows = 16;   // W2 rows per column tile (range and rescale tiles)

__device__ __forceinline__ void cle_wave_minmax(float& lo, float& hi) {
    lo = fminf(lo, dpp_f(lo, 0xB1));
    hi = fmaxf(hi, dpp_f(hi, 0xB1));
    lo = fminf(lo, dpp_f(lo, 0x4E));
    hi = fmaxf(hi, dpp_f(hi, 0x4E));
    lo = fminf(lo, dpp_f(lo, 0x141));
    hi = fmaxf(hi, dpp_f(hi, 0x141));
    lo = fminf(lo, dpp_f(lo, 0x140));
    hi = fmaxf(hi, dpp_f(hi, 0x140));
    lo = fminf(fminf(rl_f(lo, 0), rl_f(lo, 16)), fminf(rl_f(lo, 32), rl_f(lo, 48)));
    hi = fmaxf(fmaxf(rl_f(hi, 0), rl_f(hi, 16)), fmaxf(rl_f(hi, 32), rl_f(hi, 48)));
}

struct CleScale {
    float s;    // stored in S and multiplied into W1 rows, B1, bn_w, bn_b
    float inv;  // multiplied into W2 columns
};

// s = (1 / (r1 + eps)) * sqrt(r1 * r2 + eps); s = max(smin, min(smax, s))  (Python builtins)
__device__ __forceinline__ CleScale cle_scale_from(float mn1, float mx1, float mn2, float mx2, int is_signed, float eps,
                                                   double smin, double smax) {
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

__device__ __forceinline__ CleScale cle_scale(const uint32_t* mins, const uint32_t* maxs, int64_t c1, int64_t c,
                                              int is_signed, float eps, double smin, double smax) {
    return cle_scale_from(dec_ord(mins[c]), dec_ord(maxs[c]), dec_ord(mins[c1 + c]), dec_ord(maxs[c1 + c]), is_signed,
                          eps, smin, smax);
}

}  // namespace dfq
