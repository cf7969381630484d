"""Grouped weight sweep: many tensors, one (or two) kernel launches.

Host wrapper of ``dfq_sweep_plan_*`` (include/dfq_hip.h).  A ``SweepPlan`` keeps
every tensor it references alive; ``execute()`` is asynchronous on the current
stream and replays with no host work beyond one C call.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib


@dataclass
class SweepItem:
    """One fp32 tensor viewed as [rows, row_len] and what to write for it.  The
    outputs (codes, scale, zero, esum) may also be raw device addresses (int) into
    memory the caller keeps alive until the plan has run."""
    src: torch.Tensor
    bits: int = 8
    per_channel: bool = True
    symmetric: bool = True
    dst: Optional[torch.Tensor] = None       # dequantized output (may be src)
    codes: Optional[torch.Tensor] = None
    scale: Optional[torch.Tensor] = None
    zero: Optional[torch.Tensor] = None
    esum: Optional[torch.Tensor] = None
    khw: int = 1
    clip: Optional[Sequence[float]] = None
    rows: Optional[int] = None
    pack_int4: bool = False                  # codes as packed nibbles (bits <= 4; n/2 bytes)
    # per-tensor modes: the (min, max) already on the device in dfq_range's encoding
    # (2 int32 words, e.g. merge_batchnorm(ranges=...)'s by-product): one HBM pass
    range_enc: Optional[torch.Tensor] = None

    def mode(self) -> int:
        if self.per_channel:
            return _lib.DFQ_CHANNEL_SYM if self.symmetric else _lib.DFQ_CHANNEL_ASYM
        return _lib.DFQ_TENSOR_SYM if self.symmetric else _lib.DFQ_TENSOR_ASYM


def code_dtype(bits: int, symmetric: bool) -> torch.dtype:
    if bits <= 8:
        return torch.int8 if symmetric else torch.uint8
    return torch.int16


def allocate(src: torch.Tensor, bits=8, per_channel=True, symmetric=True, khw=1, in_place=False,
             want_codes=True, want_esum=False, clip=None, pack_int4=False) -> SweepItem:
    """A SweepItem with freshly allocated outputs on src's device.  ``pack_int4``:
    codes as nibbles, two per byte (element 2k low, 2k+1 high; DFQ_PACK_INT4)."""
    rows = src.shape[0] if (per_channel and src.dim() > 0) else 1
    npar = rows if per_channel else 1
    dev = src.device
    if pack_int4 and bits > 4:
        raise ValueError("packed codes need bits <= 4")
    if pack_int4:
        codes = torch.empty((src.numel() + 1) // 2, dtype=torch.uint8, device=dev) if want_codes else None
    else:
        codes = torch.empty(src.shape, dtype=code_dtype(bits, symmetric), device=dev) if want_codes else None
    return SweepItem(
        src=src, bits=bits, per_channel=per_channel, symmetric=symmetric,
        dst=src if in_place else torch.empty_like(src),
        codes=codes, pack_int4=pack_int4,
        scale=torch.empty(npar, dtype=torch.float32, device=dev),
        zero=torch.empty(npar, dtype=torch.float32, device=dev),
        esum=torch.empty(src.numel() // khw, dtype=torch.float32, device=dev) if want_esum else None,
        khw=khw, clip=clip, rows=rows)


_DESC = np.dtype([("src", "<u8"), ("dst", "<u8"), ("codes", "<u8"), ("scale", "<u8"), ("zero", "<u8"),
                  ("esum", "<u8"), ("rows", "<i8"), ("row_len", "<i8"), ("khw", "<i4"), ("bits", "<i4"),
                  ("mode", "<i4"), ("flags", "<i4"), ("clip_lo", "<f4"), ("clip_hi", "<f4"),
                  ("given_min", "<f8"), ("given_max", "<f8"), ("range_enc", "<u8")])
assert _DESC.itemsize == C.sizeof(_lib.TensorDesc)
assert all(_DESC.fields[f][1] == getattr(_lib.TensorDesc, f).offset for f, _ in _lib.TensorDesc._fields_)


class SweepPlan:
    def __init__(self, items: List[SweepItem]):
        self.items = list(items)
        L = _lib.load()
        rows_ = []
        for it in self.items:
            _lib.require_device(it.src, it.dst, *(t for t in (it.scale, it.zero, it.esum) if not isinstance(t, int)))
            if it.codes is not None and not isinstance(it.codes, int) and not it.codes.is_cuda:
                raise RuntimeError("codes must live on the GPU")
            rows = it.rows if it.rows is not None else (it.src.shape[0] if (it.per_channel and it.src.dim()) else 1)
            flags = (_lib.DFQ_CLIP if it.clip is not None else 0) | (_lib.DFQ_PACK_INT4 if it.pack_int4 else 0)
            rng = 0
            if it.range_enc is not None and not it.per_channel:
                r = it.range_enc
                if not (r.is_cuda and r.dtype == torch.int32 and r.numel() >= 2 and r.is_contiguous()):
                    raise TypeError("range_enc: 2 contiguous int32 words on the GPU")
                flags |= _lib.DFQ_DEVICE_RANGE
                rng = r.data_ptr()
            clo, chi = (float(it.clip[0]), float(it.clip[1])) if it.clip is not None else (0.0, 0.0)
            ptr = lambda t: t if isinstance(t, int) else (t.data_ptr() if t is not None else 0)   # noqa: E731
            rows_.append((it.src.data_ptr(), ptr(it.dst), ptr(it.codes), ptr(it.scale), ptr(it.zero), ptr(it.esum),
                          rows, it.src.numel() // rows if rows else 0, it.khw, it.bits, it.mode(), flags, clo, chi,
                          0.0, 0.0, rng))
        # the descriptor table as a numpy record array (layout of _lib.TensorDesc),
        # filled row-wise from plain tuples instead of ctypes field by field
        tab = np.array(rows_ if rows_ else [(0,) * 6 + (0, 0, 1, 8, 0, 0, 0.0, 0.0, 0.0, 0.0, 0)], dtype=_DESC)
        self._tab = tab
        descs = tab.ctypes.data_as(C.POINTER(_lib.TensorDesc))
        self._plan = C.c_void_p()
        self._device = self.items[0].src.device if self.items else None
        self._ws = None
        if self.items:
            # task tables in torch's caching allocator (stream-ordered): no hipMalloc /
            # hipFree per plan, and destroy() needs no device sync
            nb = int(L.dfq_sweep_plan_ws_bytes(descs, len(self.items)))
            if nb < 0:
                _lib.check(L.dfq_sweep_plan_create(descs, len(self.items), C.byref(self._plan)),
                           "dfq_sweep_plan_create", ValueError)   # raises with the planner's error
            self._stream = torch.cuda.current_stream(self._device)
            self._ws = torch.empty(max(nb, 256), dtype=torch.uint8, device=self._device)
            _lib.check(L.dfq_sweep_plan_create_ws(descs, len(self.items), self._ws.data_ptr(), self._ws.numel(),
                                                  C.c_void_p(self._stream.cuda_stream), C.byref(self._plan)),
                       "dfq_sweep_plan_create_ws", ValueError)
        else:
            _lib.check(L.dfq_sweep_plan_create(descs, 0, C.byref(self._plan)), "dfq_sweep_plan_create", ValueError)
        st = _lib.SweepStats()
        _lib.check(L.dfq_sweep_plan_stats(self._plan, C.byref(st)), "dfq_sweep_plan_stats")
        self.stats = {f: getattr(st, f) for f, _ in _lib.SweepStats._fields_}

    def execute(self, stream: Optional[torch.cuda.Stream] = None):
        if self._plan is None:
            raise RuntimeError("plan destroyed")
        if not self.items:
            return
        s = stream if stream is not None else torch.cuda.current_stream(self._device)
        if s != self._stream:   # the tables must outlive work queued on another stream
            self._ws.record_stream(s)
        _lib.check(_lib.load().dfq_sweep_plan_execute(self._plan, C.c_void_p(s.cuda_stream)),
                   "dfq_sweep_plan_execute")

    def destroy(self):
        if self._plan is not None and self._plan.value:
            # workspace-backed: the C plan holds no device memory, and the tables are
            # released to torch's allocator in stream order (no sync needed)
            _lib.load().dfq_sweep_plan_destroy(self._plan)
        self._plan = None
        self._ws = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def khw_of(weight: torch.Tensor) -> int:
    """Spatial size KH*KW of a KCRS conv weight (1 for Linear)."""
    s = weight.shape   # from the shape: no view per call
    return math.prod(s[2:]) if len(s) >= 3 else 1
