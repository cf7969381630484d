"""ctypes binding of libdfq_hip.so (include/dfq_hip.h).

This is the only door from the Python host layer into the HIP kernels.  There is
no CPU fallback: if the library is missing, or a tensor is not on a ROCm device,
the call raises.  (The CPU restatement under oracle/ is test infrastructure and
is never imported here.)
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path
from typing import Optional

import torch

PKG = Path(__file__).resolve().parent
LIB_PATH = PKG / "libdfq_hip.so"

DFQ_TENSOR_ASYM, DFQ_TENSOR_SYM, DFQ_CHANNEL_ASYM, DFQ_CHANNEL_SYM = 0, 1, 2, 3
DFQ_CLIP, DFQ_GIVEN_RANGE, DFQ_SCALE_F32, DFQ_PACK_INT4, DFQ_DEVICE_RANGE = 0x1, 0x2, 0x4, 0x8, 0x10
DFQ_OK, DFQ_ERR_INVALID, DFQ_ERR_HIP, DFQ_ERR_UNSUPPORTED = 0, -1, -2, -3
DFQ_ERR_NOMEM, DFQ_ERR_SHAPE, DFQ_ERR_WORKSPACE = -4, -5, -6

EXPORTS = [
    "dfq_abi_version", "dfq_preload", "dfq_error_string", "dfq_last_hip_error",
    "dfq_quantize_ws_bytes", "dfq_quantize_tensor", "dfq_chunk_range", "dfq_range", "dfq_fake_quant_given",
    "dfq_fake_quant_tensor",
    "dfq_act_observe",
    "dfq_sweep_plan_create", "dfq_sweep_plan_ws_bytes", "dfq_sweep_plan_create_ws", "dfq_sweep_plan_execute",
    "dfq_sweep_plan_stats", "dfq_sweep_plan_destroy",
    "dfq_bn_fold", "dfq_bn_fold_ws_bytes", "dfq_bn_fold_batch", "dfq_clamp", "dfq_clamp_batch",
    "dfq_cle_ws_bytes", "dfq_cle_relation",
    "dfq_diff_plan_create", "dfq_diff_plan_snapshot", "dfq_diff_plan_execute", "dfq_diff_plan_destroy",
    "dfq_cle_plan_ws_bytes", "dfq_cle_plan_create", "dfq_cle_plan_run", "dfq_cle_plan_launch", "dfq_cle_plan_join",
    "dfq_cle_plan_info", "dfq_cle_plan_set_timing", "dfq_cle_plan_stats", "dfq_cle_plan_destroy",
    "dfq_bias_absorb", "dfq_bias_absorb_ws_bytes", "dfq_bias_absorb_batch", "dfq_bc_expect", "dfq_bc_apply", "dfq_bc_propagate", "dfq_bc_chain",
    "dfq_act_moments", "dfq_act_minmax", "dfq_act_affine",
]
#: entry points only the diagnostics library exports (include/dfq_diag.h)
DIAG_EXPORTS = ["dfq_probe_stream", "dfq_probe_lds", "dfq_debug_timeline", "dfq_debug_ablate",
                "dfq_diag_cle_check_structure"]
DIAG_LIB_PATH = PKG / "libdfq_diag.so"


class TensorDesc(C.Structure):
    _fields_ = [
        ("src", C.c_void_p), ("dst", C.c_void_p), ("codes", C.c_void_p), ("scale", C.c_void_p),
        ("zero", C.c_void_p), ("esum", C.c_void_p), ("rows", C.c_int64), ("row_len", C.c_int64),
        ("khw", C.c_int32), ("bits", C.c_int32), ("mode", C.c_int32), ("flags", C.c_int32),
        ("clip_lo", C.c_float), ("clip_hi", C.c_float), ("given_min", C.c_double), ("given_max", C.c_double),
        ("range_enc", C.c_void_p),
    ]


class SweepStats(C.Structure):
    _fields_ = [
        ("n_tensors", C.c_int64), ("n_elems", C.c_int64), ("n_tasks_reduce", C.c_int64),
        ("n_tasks_main", C.c_int64), ("algo_bytes", C.c_int64), ("launches", C.c_int32),
        ("grid_blocks", C.c_int32), ("variant", C.c_int32), ("reserved", C.c_int32),
    ]


class BnFoldDesc(C.Structure):
    _fields_ = [
        ("w", C.c_void_p), ("bias", C.c_void_p), ("bn_w", C.c_void_p), ("bn_b", C.c_void_p),
        ("bn_mean", C.c_void_p), ("bn_var", C.c_void_p), ("fake_w", C.c_void_p), ("fake_b", C.c_void_p),
        ("eps", C.c_float), ("flags", C.c_int32), ("rows", C.c_int64), ("row_len", C.c_int64),
        ("range_enc", C.c_void_p),
    ]


class CleRel(C.Structure):
    _fields_ = [
        ("w1", C.c_void_p), ("w2", C.c_void_p), ("b1", C.c_void_p), ("bn_w", C.c_void_p), ("bn_b", C.c_void_p),
        ("s_acc", C.c_void_p), ("c1", C.c_int64), ("len1", C.c_int64), ("o2", C.c_int64), ("i2", C.c_int64),
        ("khw2", C.c_int64), ("s_acc_init", C.c_int32), ("reserved", C.c_int32),
    ]


class AbsorbDesc(C.Structure):
    _fields_ = [
        ("w2", C.c_void_p), ("b1", C.c_void_p), ("b2", C.c_void_p), ("bn_w", C.c_void_p), ("bn_b", C.c_void_p),
        ("c1", C.c_int64), ("o2", C.c_int64), ("i2", C.c_int64), ("khw2", C.c_int64),
    ]


class BcOp(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("flag", C.c_int32), ("a", C.c_void_p), ("b", C.c_void_p), ("out", C.c_void_p),
        ("out2", C.c_void_p), ("n", C.c_int64), ("i2", C.c_int64), ("f", C.c_int64),
    ]


DFQ_BC_OP_EXPECT, DFQ_BC_OP_APPLY, DFQ_BC_OP_PROPAGATE, DFQ_BC_OP_COPY = 0, 1, 2, 3
DFQ_BC_APPLY_VEC_SCRATCH = 1
DFQ_BN_FOLD_ZERO_BIAS = 1

_LIB: Optional[C.CDLL] = None


class DFQLibraryError(RuntimeError):
    pass


def load(path: Optional[os.PathLike] = None) -> C.CDLL:
    """Load (once) and type the library.  Raises if it is not built.
    ``DFQ_LIB=diag`` makes the diagnostics build (libdfq_diag.so: the same entry
    points plus A/B variants, environment switches and probes) the library of this
    process -- for scripts/ A/B runs only."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    by_env = path is None and os.environ.get("DFQ_LIB") == "diag"
    if by_env:
        path = DIAG_LIB_PATH
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise DFQLibraryError(
            f"{p} is missing: build it with `python -m data_free_quantization_amd.build` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    L = C.CDLL(str(p))
    P, I32, I64, F32, F64, SZ = C.c_void_p, C.c_int32, C.c_int64, C.c_float, C.c_double, C.c_size_t
    sig = {
        "dfq_abi_version": ([], C.c_int),
        "dfq_preload": ([], C.c_int),
        "dfq_error_string": ([C.c_int], C.c_char_p),
        "dfq_last_hip_error": ([], C.c_char_p),
        "dfq_quantize_ws_bytes": ([C.POINTER(TensorDesc), C.POINTER(SZ)], C.c_int),
        "dfq_quantize_tensor": ([C.POINTER(TensorDesc), P, SZ, P], C.c_int),
        "dfq_chunk_range": ([P, I64, I64, P, P, P], C.c_int),
        "dfq_range": ([P, I64, P, P], C.c_int),
        "dfq_act_observe": ([P, I64, I64, P, P, P, I32, I32, F64, P, P], C.c_int),
        "dfq_fake_quant_given": ([P, P, I64, I32, I32, I32, P, P, P, F64, F64, P], C.c_int),
        "dfq_fake_quant_tensor": ([P, P, I64, I32, I32, I32, P, P], C.c_int),
        "dfq_sweep_plan_create": ([C.POINTER(TensorDesc), I32, C.POINTER(P)], C.c_int),
        "dfq_sweep_plan_ws_bytes": ([C.POINTER(TensorDesc), I32], C.c_int64),
        "dfq_sweep_plan_create_ws": ([C.POINTER(TensorDesc), I32, P, I64, P, C.POINTER(P)], C.c_int),
        "dfq_sweep_plan_execute": ([P, P], C.c_int),
        "dfq_sweep_plan_stats": ([P, C.POINTER(SweepStats)], C.c_int),
        "dfq_sweep_plan_destroy": ([P], C.c_int),
        "dfq_bn_fold": ([P, P, P, P, P, P, P, P, F32, I64, I64, P], C.c_int),
        "dfq_clamp": ([P, I64, F32, F32, P], C.c_int),
        "dfq_clamp_batch": ([C.POINTER(P), C.POINTER(I64), I32, F32, F32, P], C.c_int),
        "dfq_bn_fold_ws_bytes": ([C.POINTER(BnFoldDesc), I32], C.c_int64),
        "dfq_bn_fold_batch": ([C.POINTER(BnFoldDesc), I32, P, I64, P], C.c_int),
        "dfq_cle_ws_bytes": ([I64], SZ),
        "dfq_cle_relation": ([P, P, P, P, P, I64, I64, I64, I64, I64, F64, F64, I32, F32, P, P, I32, P, SZ, P],
                             C.c_int),
        "dfq_diff_plan_create": ([C.POINTER(P), C.POINTER(P), C.POINTER(I64), I32, C.POINTER(P)], C.c_int),
        "dfq_diff_plan_snapshot": ([P, P], C.c_int),
        "dfq_diff_plan_execute": ([P, C.POINTER(F64), P], C.c_int),
        "dfq_diff_plan_destroy": ([P], C.c_int),
        "dfq_cle_plan_ws_bytes": ([C.POINTER(I64), I32], C.c_int64),
        "dfq_cle_plan_create": ([C.POINTER(CleRel), I32, C.POINTER(P), C.POINTER(I64), I32, F64, F64, I32, F32, I32,
                                 P, I64, C.POINTER(P)], C.c_int),
        "dfq_cle_plan_run": ([P, F64, I32, I32, C.POINTER(I32), C.POINTER(F64), P], C.c_int),
        "dfq_cle_plan_launch": ([P, F64, I32, I32, P], C.c_int),
        "dfq_cle_plan_join": ([P, C.POINTER(I32), C.POINTER(F64)], C.c_int),
        "dfq_cle_plan_info": ([P, C.POINTER(I32), C.POINTER(I32), C.POINTER(I32)], C.c_int),
        "dfq_cle_plan_destroy": ([P], C.c_int),
        "dfq_cle_plan_set_timing": ([P, I32], C.c_int),
        "dfq_cle_plan_stats": ([P, C.POINTER(I64), C.POINTER(F64), C.POINTER(I32)], C.c_int),
        "dfq_bias_absorb": ([P, P, P, P, P, I64, I64, I64, I64, F32, P], C.c_int),
        "dfq_bias_absorb_ws_bytes": ([C.POINTER(AbsorbDesc), I32], C.c_int64),
        "dfq_bias_absorb_batch": ([C.POINTER(AbsorbDesc), I32, F32, P, I64, C.POINTER(I32), P], C.c_int),
        "dfq_bc_expect": ([P, P, I64, I32, I32, P, P], C.c_int),
        "dfq_bc_apply": ([P, I64, I64, P, I64, P, P, C.POINTER(I64), P], C.c_int),
        "dfq_bc_propagate": ([P, I64, P, I64, I32, P], C.c_int),
        "dfq_bc_chain": ([C.POINTER(BcOp), I32, C.POINTER(I32), P], C.c_int),
        "dfq_act_moments": ([P, P, I64, I32, I32, F32, I32, P, P, P], C.c_int),
        "dfq_act_minmax": ([P, P, I64, I32, F32, F32, P, P], C.c_int),
        "dfq_act_affine": ([P, P, P, I64, I64, I64, I64, P, P], C.c_int),
    }
    diag = {
        "dfq_probe_stream": ([P, P, P, P, I64, I32, P], C.c_int),
        "dfq_debug_timeline": ([P, I64], C.c_int),
        "dfq_debug_ablate": ([C.c_uint32], C.c_int),
        "dfq_probe_lds": ([P, P, P, P, I64, I32, I32, P], C.c_int),
        "dfq_diag_cle_check_structure": ([C.POINTER(CleRel), I32, C.POINTER(P), C.POINTER(I64), I32, I32,
                                          C.POINTER(I64), C.c_char_p, I32], C.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    for name, (args, res) in diag.items():
        if hasattr(L, name):
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
    if L.dfq_abi_version() != 1:
        raise DFQLibraryError("libdfq_hip.so ABI version mismatch")
    if path is None or by_env:   # the process's library (the diagnostics one under DFQ_LIB=diag):
        _LIB = L                 # cached -- loaded and typed per call it cost ~0.1 ms a call
    return L


_PRELOADED = False


def preload() -> C.CDLL:
    """Load the library, every kernel's code object on the current device and the
    buffers a first run would allocate (dfq_preload: CLE pools, history, signal
    word and worker, pinned staging slots) so the first DFQ stage does not pay for
    them.  Needs a GPU."""
    global _PRELOADED
    L = load()
    if not _PRELOADED:
        check(L.dfq_preload(), "dfq_preload")
        _PRELOADED = True
    return L


_DIAG: Optional[C.CDLL] = None


def load_diag() -> C.CDLL:
    """The diagnostics library (include/dfq_diag.h): bench.py's ceiling probes."""
    global _DIAG
    if _DIAG is None:
        _DIAG = load(DIAG_LIB_PATH)
    return _DIAG


def check(rc: int, what: str, shape_error=RuntimeError):
    """Map a DFQ_ERR_* code to the exception the reference would raise."""
    if rc == DFQ_OK:
        return
    L = load()
    msg = f"{what}: {L.dfq_error_string(rc).decode()}"
    if rc == DFQ_ERR_HIP:
        msg += f" ({L.dfq_last_hip_error().decode()})"
    if rc == DFQ_ERR_SHAPE:
        raise shape_error(msg)
    if rc == DFQ_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise DFQLibraryError(msg)


_F32 = torch.float32


def require_device(*tensors: Optional[torch.Tensor]):
    for t in tensors:
        if t is None or (t.is_cuda and t.dtype is _F32 and t.is_contiguous()):
            continue
        if not t.is_cuda:
            raise RuntimeError(
                "data_free_quantization_amd runs the DFQ weight path on a ROCm GPU only; "
                f"got a tensor on {t.device} (move the model with .cuda() first)")
        if t.dtype != torch.float32:
            raise TypeError(f"expected float32 tensors, got {t.dtype}")
        raise ValueError("expected contiguous tensors")


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


#: Generation of the model weights as the DFQ transforms see them: every transform
#: that rewrites weights or biases in place through the library (which bypasses
#: torch's version counters) advances it, so caches of derived weights
#: (utils.quantize's per-layer fake-quant cache) know they are stale.
WEIGHT_GENERATION = 0


def weights_changed() -> None:
    global WEIGHT_GENERATION
    WEIGHT_GENERATION += 1


#: intra-op thread count of the reference run the BC reductions reproduce
#: (torch.get_num_threads() when tests/golden was generated)
REF_THREADS = int(os.environ.get("DFQ_REF_THREADS", "8"))


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def raw_stream(device: torch.device) -> C.c_void_p:
    """The device's current stream handle, without building a torch Stream object
    (torch.cuda.current_stream measured tens of us per call on the GPU boxes)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if _RAW_STREAM is not None:
        return C.c_void_p(_RAW_STREAM(idx))
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def stream_of(t: torch.Tensor):
    return raw_stream(t.device)
