"""TEST INFRASTRUCTURE ONLY: numpy front-end of the C oracle (oracle/dfq_oracle.c).

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker.  Never imported by the product package.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "libdfq_oracle.so"

TENSOR_ASYM, TENSOR_SYM, CHANNEL_ASYM, CHANNEL_SYM = 0, 1, 2, 3
F_CLIP, F_GIVEN, F_F32 = 1, 2, 4

_lib = None


def build(force: bool = False) -> Path:
    src = HERE / "dfq_oracle.c"
    if force or not LIB.exists() or LIB.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE), "-B" if force else "_build/libdfq_oracle.so"], check=True,
                       stdout=subprocess.DEVNULL)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(LIB))
        P, I64, I32, F32, F64 = C.c_void_p, C.c_int64, C.c_int, C.c_float, C.c_double
        L.oracle_quantize.argtypes = [P, I64, I64, I32, I32, I32, I32, F32, F32, F64, F64, P, P, P, P, P]
        L.oracle_bn_fold.argtypes = [P, P, P, P, P, P, P, P, F32, I64, I64]
        L.oracle_chunk_range.argtypes = [P, I64, I64, P]
        L.oracle_cle_relation.argtypes = [P, P, P, P, P, I64, I64, I64, I64, I64, F64, F64, I32, F32, P]
        L.oracle_bias_absorb.argtypes = [P, P, P, P, P, I64, I64, I64, I64, F32]
        L.oracle_bc_expect.argtypes = [P, P, I64, I32, I32, P]
        L.oracle_bc_apply.argtypes = [P, I64, I64, P, I64, P, P, C.POINTER(I64)]
        L.oracle_bc_propagate.argtypes = [P, I64, P, I64, I32]
        L.oracle_mean_abs_diff.argtypes = [P, P, I64, I32]
        L.oracle_mean_abs_diff.restype = C.c_float
        L.oracle_np_sum.argtypes = [P, I64]
        L.oracle_np_sum.restype = C.c_double
        L.oracle_act_moments.argtypes = [P, P, I64, I32, I32, F32, I32, P, P]
        L.oracle_act_minmax.argtypes = [P, P, I64, I32, F32, F32, P]
        L.oracle_act_affine.argtypes = [P, P, P, I64, I64, I64, I64, P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def quantize(x, bits=8, mode=TENSOR_ASYM, rows=None, khw=1, flags=0, clip=(0.0, 0.0), given=(0.0, 0.0),
             want_esum=False):
    """Returns dict(dq, codes, scale, zero[, esum]) for x viewed as [rows, numel/rows]."""
    x = _f32(x)
    n = x.size
    if rows is None:
        rows = x.shape[0] if x.ndim > 0 else 1
    row_len = n // rows if rows else 0
    sym = mode in (TENSOR_SYM, CHANNEL_SYM)
    cdt = (np.int8 if sym else np.uint8) if bits <= 8 else (np.int16 if sym else np.uint16)
    dq = np.empty_like(x)
    codes = np.empty(x.shape, dtype=cdt)
    npar = rows if mode >= CHANNEL_ASYM else 1
    scale = np.empty(npar, np.float32)
    zero = np.empty(npar, np.float32)
    esum = np.empty(n // khw, np.float32) if want_esum else None
    rc = lib().oracle_quantize(_p(x), rows, row_len, khw, bits, mode, flags, clip[0], clip[1], given[0], given[1],
                               _p(dq), _p(codes), _p(scale), _p(zero), _p(esum))
    if rc:
        raise RuntimeError(f"oracle_quantize rc={rc}")
    out = dict(dq=dq, codes=codes, scale=scale, zero=zero)
    if want_esum:
        out["esum"] = esum
    return out


def chunk_range(x, rows):
    """quantize()'s range for min/max None (utils/quantize.py:26-37): mean over the
    rows of x.view(rows, -1) of each row's min / max, as fp32."""
    x = _f32(x)
    out = np.empty(2, np.float32)
    rc = lib().oracle_chunk_range(_p(x), rows, x.size // rows, _p(out))
    if rc:
        raise RuntimeError(f"oracle_chunk_range rc={rc}")
    return out[0], out[1]


def bn_fold(w, bias, g, b, m, v, eps):
    """Returns (w, bias, g, b, m, v, fake_w, fake_b) after merge_batchnorm's arithmetic."""
    w, bias, g, b, m, v = (_f32(a).copy() for a in (w, bias, g, b, m, v))
    fw, fb = np.empty_like(g), np.empty_like(b)
    lib().oracle_bn_fold(_p(w), _p(bias), _p(g), _p(b), _p(m), _p(v), _p(fw), _p(fb), eps, g.size,
                         w.size // max(g.size, 1))
    return w, bias, g, b, m, v, fw, fb


def cle_relation(w1, w2, b1, bn_w, bn_b, s_min=1e-8, s_max=1e8, signed=False, eps=0.0):
    """In-place-free version of _layer_equalization: returns (w1, w2, b1, bn_w, bn_b, S)."""
    w1, w2 = _f32(w1).copy(), _f32(w2).copy()
    b1 = None if b1 is None else _f32(b1).copy()
    bn_w = None if bn_w is None else _f32(bn_w).copy()
    bn_b = None if bn_b is None else _f32(bn_b).copy()
    c1 = w1.shape[0]
    o2, i2 = w2.shape[0], w2.shape[1]
    S = np.empty(c1, np.float32)
    rc = lib().oracle_cle_relation(_p(w1), _p(w2), _p(b1), _p(bn_w), _p(bn_b), c1, w1.size // c1, o2, i2,
                                   w2.size // (o2 * i2), s_min, s_max, int(signed), eps, _p(S))
    if rc:
        raise RuntimeError(f"oracle_cle_relation rc={rc}")
    return w1, w2, b1, bn_w, bn_b, S


def bias_absorb(w2, b1, b2, bn_w, bn_b, c1, n_sigma=3.0):
    w2 = _f32(w2)
    b1, b2, bn_w, bn_b = (_f32(a).copy() for a in (b1, b2, bn_w, bn_b))
    o2, i2 = w2.shape[0], w2.shape[1]
    rc = lib().oracle_bias_absorb(_p(w2), _p(b1), _p(b2), _p(bn_w), _p(bn_b), c1, o2, i2, w2.size // (o2 * i2),
                                  n_sigma)
    if rc:
        raise RuntimeError(f"oracle_bias_absorb rc={rc}")
    return b1, b2, bn_w, bn_b


def bc_expect(w, b, relu, out=None):
    w, b = _f32(w), _f32(b)
    acc = out is not None
    out = np.empty_like(w) if out is None else _f32(out).copy()
    lib().oracle_bc_expect(_p(w), _p(b), w.size, int(relu), int(acc), _p(out))
    return out


def bc_apply(E, expect, bias):
    E, expect = _f32(E), _f32(expect)
    bias = _f32(bias).copy()
    o, i2 = E.shape[0], E.size // E.shape[0]
    bcols = C.c_int64(0)
    f = expect.size
    bc_guess = i2 if (i2 == f or f == 1) else f
    vec = np.empty(o * bc_guess, np.float32)
    rc = lib().oracle_bc_apply(_p(E), o, i2, _p(expect), f, _p(bias), _p(vec), C.byref(bcols))
    if rc:
        raise ValueError(f"oracle_bc_apply rc={rc}")
    return bias, vec[: o * bcols.value]


def bc_propagate(vec, fake_b, threads=8):
    vec = _f32(vec)
    fake_b = _f32(fake_b).copy()
    rc = lib().oracle_bc_propagate(_p(vec), vec.size, _p(fake_b), fake_b.size, threads)
    if rc:
        raise RuntimeError(f"oracle_bc_propagate rc={rc}")
    return fake_b


def mean_abs_diff(a, b, threads=8):
    """float(torch.mean(torch.abs(a - b))) in ATen's CPU order (Cross_layer_equal.py:107)."""
    a, b = _f32(a), _f32(b)
    return float(lib().oracle_mean_abs_diff(_p(a), _p(b), a.size, threads))


def np_sum(values):
    """np.sum(list_of_floats) (numpy pairwise summation), restated."""
    v = np.ascontiguousarray(values, dtype=np.float64)
    return float(lib().oracle_np_sum(_p(v), v.size))


def act_moments(w, b, kind, sqrt_w=False, eps=1e-6, into=None):
    """set_quant_minmax's (mean, var) of one BN branch (utils/layer_transform.py:396-410)."""
    w, b = _f32(w), _f32(b)
    if into is None:
        mean, var, acc = np.empty_like(b), np.empty_like(b), 0
    else:
        mean, var = into
        acc = 1
    lib().oracle_act_moments(_p(w), _p(b), b.size, kind, int(sqrt_w), eps, acc, _p(mean), _p(var))
    return mean, var


def act_minmax(a, w, nsig, w_is_var=False, eps=1e-6):
    a, w = _f32(a), _f32(w)
    out = np.empty(2, np.float32)
    lib().oracle_act_minmax(_p(a), _p(w), a.size, int(w_is_var), eps, float(nsig), _p(out))
    return float(out[0]), float(out[1])


def act_affine(x, w, bias, groups=1):
    """Case (d.) of set_quant_minmax: x pushed through W (summed over KH*KW) + bias."""
    x, w = _f32(x), _f32(w)
    b = None if bias is None else _f32(bias)
    o, i2 = w.shape[0], w.shape[1]
    khw = w.size // (o * i2)
    out = np.empty(o, np.float32)
    lib().oracle_act_affine(_p(x), _p(w), _p(b), o, i2, khw, groups, _p(out))
    return out
