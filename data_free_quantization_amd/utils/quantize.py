"""Drop-in for the reference's ``utils/quantize.py`` (utils/quantize.py:1-379).

Same names, signatures and semantics; the fake-quant arithmetic runs in the HIP
kernel ``dfq_quantize_tensor`` (libdfq_hip.so), bit-exact with the reference's
CPU path.  Extensions are additive keyword arguments or
new functions (``quantize_per_channel``, ``fake_quant``).

Tensors must live on a ROCm device; there is no CPU fallback.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import struct
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.autograd.function import InplaceFunction

from .. import _lib


@dataclass
class QuantResult:
    """Outputs of one fake-quant call (extension API)."""
    dq: torch.Tensor                 # dequantized fp32, same shape as the input
    codes: Optional[torch.Tensor]    # integer grid indices (uint8/int8/int16)
    scale: torch.Tensor              # [rows] or [1]
    zero: torch.Tensor               # [rows] or [1] (the range min for asym, 0 for sym)
    esum: Optional[torch.Tensor] = None


def _code_dtype(bits: int, symmetric: bool):
    if bits <= 8:
        return torch.int8 if symmetric else torch.uint8
    return torch.int16


def _is_tensor_value(v) -> bool:
    return isinstance(v, torch.Tensor)


def fake_quant(x: torch.Tensor, num_bits: int = 8, *, per_channel: bool = False, symmetric: bool = False,
               min_value=None, max_value=None, out: Optional[torch.Tensor] = None, want_codes: bool = True,
               khw: int = 1, want_esum: bool = False, clip=None, scale_f32: bool = False) -> QuantResult:
    """Quantize-dequantize ``x`` (viewed as [x.shape[0], -1] in per-channel mode)
    on the GPU.  ``min_value``/``max_value`` (Python floats) fix the per-tensor
    range like quantize(x, b, min, max); otherwise the data range is used."""
    _lib.require_device(x, out)
    L = _lib.load()
    rows = x.shape[0] if (per_channel and x.dim() > 0) else 1
    n = x.numel()
    row_len = n // rows if rows else 0
    d = _lib.TensorDesc()
    d.src = x.data_ptr()
    dq = torch.empty_like(x) if out is None else out
    d.dst = dq.data_ptr()
    codes = torch.empty(x.shape, dtype=_code_dtype(num_bits, symmetric), device=x.device) if want_codes else None
    d.codes = codes.data_ptr() if codes is not None else None
    npar = rows if per_channel else 1
    scale = torch.empty(npar, dtype=torch.float32, device=x.device)
    zero = torch.empty(npar, dtype=torch.float32, device=x.device)
    d.scale, d.zero = scale.data_ptr(), zero.data_ptr()
    esum = None
    if want_esum:
        esum = torch.empty(n // khw, dtype=torch.float32, device=x.device)
        d.esum = esum.data_ptr()
    d.rows, d.row_len, d.khw, d.bits = rows, row_len, khw, num_bits
    d.mode = (_lib.DFQ_CHANNEL_SYM if symmetric else _lib.DFQ_CHANNEL_ASYM) if per_channel else \
        (_lib.DFQ_TENSOR_SYM if symmetric else _lib.DFQ_TENSOR_ASYM)
    flags = 0
    if clip is not None:
        flags |= _lib.DFQ_CLIP
        d.clip_lo, d.clip_hi = float(clip[0]), float(clip[1])
    if min_value is not None or max_value is not None:
        if per_channel:
            raise ValueError("a fixed range is per-tensor only")
        flags |= _lib.DFQ_GIVEN_RANGE
        d.given_min, d.given_max = float(min_value), float(max_value)
    if scale_f32:
        flags |= _lib.DFQ_SCALE_F32
    d.flags = flags
    if n == 0:
        return QuantResult(dq, codes, scale, zero, esum)
    ws_bytes = C.c_size_t(0)
    _lib.check(L.dfq_quantize_ws_bytes(C.byref(d), C.byref(ws_bytes)), "dfq_quantize_ws_bytes", ValueError)
    ws = torch.empty(max(ws_bytes.value, 1), dtype=torch.uint8, device=x.device)
    _lib.check(L.dfq_quantize_tensor(C.byref(d), C.c_void_p(ws.data_ptr()), ws_bytes, _lib.stream_of(x)),
               "dfq_quantize_tensor", ValueError)
    return QuantResult(dq, codes, scale, zero, esum)


def _chunk_range(x: torch.Tensor, rows: int):
    """(min, max) as quantize() builds them when a bound is None
    (utils/quantize.py:26-37): mean over x.view(rows, -1)'s rows of each row's
    min / max, fp32 (0-d tensors in the reference)."""
    if rows == 1:
        return _data_range(x)
    xc = x.detach().contiguous()
    rowbuf = torch.empty(2 * rows, dtype=torch.float32, device=x.device)
    out2 = torch.empty(2, dtype=torch.float32, device=x.device)
    _lib.check(_lib.load().dfq_chunk_range(_lib.ptr(xc), rows, xc.numel() // rows, _lib.ptr(rowbuf), _lib.ptr(out2),
                                           _lib.stream_of(xc)), "dfq_chunk_range", RuntimeError)
    mn, mx = out2.tolist()
    return mn, mx


def _resolve_range(input, min_value, max_value, num_chunks, symmetric):
    """The (min, max) quantize() ends up using and whether its scale is built in
    fp32 (0-d tensor arithmetic) or in double (Python floats), as
    utils/quantize.py:26-68 does.  None: both bounds from the whole tensor, taken
    inside the kernel."""
    B = input.shape[0]   # the reference indexes shape[0] too (IndexError for 0-d)
    if min_value is None or max_value is None:
        nc = B if num_chunks is None else num_chunks
        rows = B // nc
        n = input.numel()
        if rows == 0 or n % rows != 0:
            raise RuntimeError(f"shape '[{rows}, -1]' is invalid for input of size {n}")
        if n == 0:
            raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0")
        if min_value is None and max_value is None and rows == 1:
            return None
        mn, mx = _chunk_range(input, rows)
        t_min, v_min = (True, mn) if min_value is None else (_is_tensor_value(min_value), float(min_value))
        t_max, v_max = (True, mx) if max_value is None else (_is_tensor_value(max_value), float(max_value))
    else:
        t_min, v_min = _is_tensor_value(min_value), float(min_value)
        t_max, v_max = _is_tensor_value(max_value), float(max_value)
    if not symmetric:
        return v_min, v_max, t_min or t_max
    # max_value = abs(max); min_value = abs(min); if max < min: max = min;
    # scale = max / qmax -- a tensor winner divides in fp32, a float one in double.
    # A tensor-vs-float comparison runs in fp32 (the float is cast to the tensor's dtype).
    a_max, a_min = abs(v_max), abs(v_min)
    if t_min or t_max:
        less = bool(torch.tensor(a_max, dtype=torch.float32) < torch.tensor(a_min, dtype=torch.float32))
    else:
        less = a_max < a_min
    w, t = (a_min, t_min) if less else (a_max, t_max)
    return w, w, t


class UniformQuantize(InplaceFunction):
    """Uniform quantize -> dequantize with a straight-through backward
    (utils/quantize.py:16-85)."""

    @staticmethod
    def forward(ctx, input, num_bits=8, min_value=None, max_value=None, inplace=False, symmetric=False,
                num_chunks=None):
        rng = _resolve_range(input, min_value, max_value, num_chunks, symmetric)
        ctx.inplace = inplace
        ctx.num_bits = num_bits
        ctx.min_value = min_value
        ctx.max_value = max_value
        if inplace:
            ctx.mark_dirty(input)
            out = input
        else:
            out = torch.empty_like(input)
        # async: one elementwise launch (plus the range reduction), no task table,
        # no host synchronisation
        x = input.detach()
        if rng is None:   # 0-d fp32 range of the whole tensor, reduced on the device
            fake_quant_given(x, num_bits, symmetric, range_enc=device_range(x), scale_f32=True, out=out)
        else:
            fake_quant_given(x, num_bits, symmetric, min_value=rng[0], max_value=rng[1], scale_f32=rng[2], out=out)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, None, None, None, None, None, None


def _dec_ord(e: int) -> float:
    """Inverse of the library's order-preserving float encoding (dfq_common.h enc_ord)."""
    u = (e & 0x7FFFFFFF) if (e & 0x80000000) else (~e & 0xFFFFFFFF)
    return struct.unpack("<f", struct.pack("<I", u))[0]


def _data_range(x: torch.Tensor):
    """fp32 (min, max) of x: one dfq_range launch and one 8-byte read back."""
    a, b = (v & 0xFFFFFFFF for v in device_range(x).tolist())
    return _dec_ord(~a & 0xFFFFFFFF), _dec_ord(b)


def _no_autograd(*tensors) -> bool:
    """True when no STE backward is needed (inference): the async paths apply."""
    return not (torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors))


def device_range(x: torch.Tensor) -> torch.Tensor:
    """dfq_range: the whole tensor's (min, max) on the device, async, as the
    library's 2-word order-preserving encoding (input of fake_quant_given)."""
    _lib.require_device(x)
    xc = x.detach().contiguous()
    enc = torch.empty(2, dtype=torch.int32, device=x.device)
    _lib.check(_lib.load().dfq_range(_lib.ptr(xc), xc.numel(), _lib.ptr(enc), _lib.stream_of(xc)), "dfq_range",
               RuntimeError)
    return enc


def fake_quant_given(x: torch.Tensor, num_bits: int = 8, symmetric: bool = False, *, min_dev=None, max_dev=None,
                     range_enc=None, min_value=None, max_value=None, scale_f32: bool = False,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """quantize(x, num_bits, min, max, symmetric=...) with a given range as ONE
    async elementwise launch (dfq_fake_quant_given): no workspace, no host sync.
    The range comes from ``range_enc`` (device_range), or device scalars
    ``min_dev`` / ``max_dev`` (read as float() would), or Python floats.
    ``scale_f32``: the bounds were 0-d tensors in the reference call (fp32 scale)."""
    _lib.require_device(x, out)
    xc = x.detach().contiguous()
    y = torch.empty_like(xc) if out is None else out
    rc = _lib.load().dfq_fake_quant_given(
        _lib.ptr(xc), _lib.ptr(y), xc.numel(), int(num_bits), int(bool(symmetric)),
        _lib.DFQ_SCALE_F32 if scale_f32 else 0, _lib.ptr(min_dev), _lib.ptr(max_dev), _lib.ptr(range_enc),
        float(min_value) if min_value is not None else 0.0, float(max_value) if max_value is not None else 0.0,
        _lib.stream_of(xc))
    _lib.check(rc, "dfq_fake_quant_given", ValueError)
    return y


def fake_quant_tensor(x: torch.Tensor, num_bits: int = 8, symmetric: bool = False, *, scale_f32: bool = False,
                      words: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """quantize(x, num_bits, float(x.min()), float(x.max()), symmetric=...) -- the
    Quant* layers' weight fake quant (utils/quantize.py:225-238; ``scale_f32`` for
    the bias's 0-d bounds) -- as ONE library call (dfq_fake_quant_tensor): the range
    and the fake quant without a fill or a host read.  ``words``: 8 int32 of device
    scratch, zeroed once and reused by the caller's later calls on the same stream
    (needed above 16,384 elements)."""
    _lib.require_device(x, out)
    xc = x.detach().contiguous()
    y = torch.empty_like(xc) if out is None else out
    if words is None and xc.numel() > 16384:
        words = torch.zeros(8, dtype=torch.int32, device=xc.device)
    rc = _lib.load().dfq_fake_quant_tensor(_lib.ptr(xc), _lib.ptr(y), xc.numel(), int(num_bits), int(bool(symmetric)),
                                           _lib.DFQ_SCALE_F32 if scale_f32 else 0, _lib.ptr(words),
                                           _lib.stream_of(xc))
    _lib.check(rc, "dfq_fake_quant_tensor", ValueError)
    return y


def quantize(x, num_bits=8, min_value=None, max_value=None, inplace=False, symmetric=False, num_chunks=None):
    """utils/quantize.py:88-89."""
    return UniformQuantize.apply(x, num_bits, min_value, max_value, inplace, symmetric, num_chunks)


def quantize_per_channel(x, num_bits=8, symmetric=False, inplace=False):
    """Extension: the reference ``quantize()`` applied to every output-channel
    slice ``x[o]`` with that slice's own float(min)/float(max) -- one kernel."""
    out = x if inplace else torch.empty_like(x)
    fake_quant(x.detach(), num_bits, per_channel=True, symmetric=symmetric, out=out, want_codes=False)
    return out


class QuantMeasure(nn.Module):
    """Activation range observer + fake quant (utils/quantize.py:94-126)."""

    def __init__(self, update_stat=False, num_bits=8, momentum=0.1):
        super().__init__()
        self.register_buffer("running_min", torch.zeros(1))
        self.register_buffer("running_max", torch.zeros(1))
        self.momentum = momentum
        self.num_bits = num_bits
        self.update_stat = update_stat

    def forward(self, input):
        if (self.update_stat or self.training) and input.is_cuda and input.dtype is torch.float32 \
                and input.numel() > 0 and input.dim() > 0:
            return self._forward_fused(input)
        flat = input.detach().view(input.size(0), -1)
        if self.update_stat:
            # Python max(a, b) / min(a, b) on tensors: b if b > a (b < a) else a --
            # as a device select instead of a host round trip
            mx_new, mn_new = flat.max(-1)[0].mean(), flat.min(-1)[0].mean()
            self.running_max = torch.where(mx_new > self.running_max, mx_new, self.running_max)
            self.running_min = torch.where(mn_new < self.running_min, mn_new, self.running_min)
        if self.training:
            mn = flat.min(-1)[0].mean()
            mx = flat.max(-1)[0].mean()
            self.running_min.mul_(1 - self.momentum).add_(mn * self.momentum)
            self.running_max.mul_(1 - self.momentum).add_(mx * self.momentum)
        else:
            mn, mx = self.running_min, self.running_max
        if _no_autograd(input):
            # no STE backward: float(mn) / float(mx) are read on the device by one
            # async launch (the reference's main_dfq runs its observers in training
            # mode at inference -- set_layer_bits makes new ones -- so both branches)
            input.shape[0]   # the reference's quantize() indexes shape[0]
            return fake_quant_given(input, self.num_bits, min_dev=mn, max_dev=mx)
        return quantize(input, self.num_bits, min_value=float(mn), max_value=float(mx), num_chunks=16)

    def _forward_fused(self, input):
        """Live statistics: the observer update in ONE dfq_act_observe call (rows'
        min / max, their means in ATen's CPU sum order -- the order of every other
        reduction this library reproduces, and of the reference's CPU fixtures --
        the update_stat select and the training momentum, two launches) and, at
        inference, the fake quant in one more: instead of eight torch ops and
        their allocations per call.  The running buffers are updated in place (the
        reference rebinds them to new tensors of the same values)."""
        x = input.detach()
        if not x.is_contiguous():
            x = x.contiguous()
        rows = x.size(0)
        # the call's scratch: the self-re-arming row words (zeroed once, reset by
        # the kernel) and the 2-float range the fake quant reads asynchronously --
        # one pair per (device, stream), so calls on two streams never share them
        stream = _lib.stream_of(x)
        bufs = self.__dict__.setdefault("_obs_bufs", {})
        key = (x.device, stream.value)
        words, out2 = bufs.get(key, (None, None))
        if words is None or words.numel() != 2 * rows:
            words = torch.zeros(2 * rows, dtype=torch.int32, device=x.device)   # armed once
            out2 = torch.empty(2, dtype=torch.float32, device=x.device)
            bufs[key] = (words, out2)
        rmin, rmax = self._buffers["running_min"], self._buffers["running_max"]
        _lib.require_device(rmin, rmax)
        _lib.check(_lib.load().dfq_act_observe(_lib.ptr(x), rows, x.numel() // rows, _lib.ptr(words), _lib.ptr(rmin),
                                               _lib.ptr(rmax), int(bool(self.update_stat)), int(bool(self.training)),
                                               float(self.momentum), _lib.ptr(out2), stream),
                   "dfq_act_observe", RuntimeError)
        if _no_autograd(input):
            return fake_quant_given(input, self.num_bits, min_dev=out2[0], max_dev=out2[1])
        mn, mx = out2.tolist()   # the STE path: the reference's float(mn) / float(mx)
        return quantize(input, self.num_bits, min_value=mn, max_value=mx, num_chunks=16)

    def set_update_stat(self, update_stat):
        self.update_stat = update_stat


def invalidate_weight_cache() -> None:
    """Drop every Quant* layer's cached weight / bias fake-quant (inside a
    ``frozen_weights()`` scope, after rewriting weights through ``.data``)."""
    _lib.weights_changed()


_FROZEN = 0   # depth of open frozen_weights() scopes


@contextlib.contextmanager
def frozen_weights():
    """Inference over fixed weights: inside this scope the Quant* layers keep their
    weight / bias fake-quant between forwards instead of re-quantizing on every call
    as the reference does (/root/reference/utils/quantize.py:225-238).  The caller
    promises that weights change only through the library's transforms or torch's
    own in-place ops (both seen by the cache key); a write through ``.data`` inside
    the scope needs ``invalidate_weight_cache()``.  Outside any scope -- the default
    -- every forward re-quantizes, so the reference's ``weight.data.copy_`` idiom
    (utils/layer_transform.py:300,303, clip_weight.py:29, bias_absorption.py:78-80)
    is always seen.  main_dfq's evaluation runs inside one."""
    global _FROZEN
    _lib.weights_changed()   # nothing cached before the scope is trusted in it
    _FROZEN += 1
    try:
        yield
    finally:
        _FROZEN -= 1
        _lib.weights_changed()


class _QuantWeightMixin:
    """Forward of the Quant* layers: activation fake-quant, per-tensor weight
    fake-quant with float(min)/float(max), bias fake-quant with the data range."""

    def _qparams(self, weight, bias):
        if _no_autograd(weight, bias):
            # inference: float(weight.min()) / float(weight.max()) and the bias's own
            # 0-d fp32 range stay on the device (dfq_range), one async launch each.
            # Inside frozen_weights() the result is kept while the key holds: the
            # module's OWN parameters (a temporary -- QConv2d's scaled weight -- is
            # never cached: its id and address are reused), their torch version
            # counters, and the DFQ transforms' generation (_lib.WEIGHT_GENERATION:
            # they write through the library, past the version counters).
            cacheable = _FROZEN > 0 and weight is self.weight and bias is self.bias
            if cacheable:
                key = (weight.data_ptr(), weight._version, self.num_bits, _lib.WEIGHT_GENERATION,
                       None if bias is None else (bias.data_ptr(), bias._version), self.num_bits_bias)
                hit = self.__dict__.get("_qw_cache")
                if hit is not None and hit[0] == key:
                    return hit[1], hit[2]
            # the tensor's range and its fake quant in one library call each (the
            # range words: this module's scratch per stream, re-armed by every call)
            stream = _lib.stream_of(weight)
            bufs = self.__dict__.setdefault("_fq_words", {})
            words = bufs.get((weight.device, stream.value))
            if words is None:
                words = bufs[(weight.device, stream.value)] = torch.zeros(16, dtype=torch.int32, device=weight.device)
            qweight = fake_quant_tensor(weight, self.num_bits, words=words[:8])
            qbias = None
            if bias is not None:
                qbias = fake_quant_tensor(bias, self.num_bits_bias, scale_f32=True, words=words[8:])
            if cacheable:
                self.__dict__["_qw_cache"] = (key, qweight, qbias)
            else:
                self.__dict__.pop("_qw_cache", None)
            return qweight, qbias
        qweight = quantize(weight, num_bits=self.num_bits, min_value=float(weight.min()),
                           max_value=float(weight.max()))
        qbias = quantize(bias, num_bits=self.num_bits_bias) if bias is not None else None
        return qweight, qbias


class QuantConv2d(_QuantWeightMixin, nn.Conv2d):
    """utils/quantize.py:213-238."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 bias=True, num_bits=8, num_bits_act=8, num_bits_bias=16, momentum=0.1):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)
        self.num_bits = num_bits
        self.num_bits_bias = num_bits_bias
        self.quant = QuantMeasure(num_bits=num_bits_act, momentum=momentum)

    def forward(self, input):
        input = self.quant(input)
        qweight, qbias = self._qparams(self.weight, self.bias)
        return F.conv2d(input, qweight, qbias, self.stride, self.padding, self.dilation, self.groups)


class QuantNConv2d(nn.Conv2d):
    """Conv2d with activation fake-quant only (utils/quantize.py:240-256)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 bias=True, num_bits=8, num_bits_act=8, momentum=0.1):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)
        self.quant = QuantMeasure(num_bits=num_bits_act, momentum=momentum)

    def forward(self, input):
        return F.conv2d(self.quant(input), self.weight, self.bias, self.stride, self.padding, self.dilation,
                        self.groups)


class QuantLinear(_QuantWeightMixin, nn.Linear):
    """utils/quantize.py:326-348."""

    def __init__(self, in_features, out_features, bias=True, num_bits=8, num_bits_act=8, num_bits_bias=16,
                 momentum=0.1):
        super().__init__(in_features, out_features, bias)
        self.num_bits = num_bits
        self.num_bits_bias = num_bits_bias
        self.quant = QuantMeasure(num_bits=num_bits_act, momentum=momentum)

    def forward(self, input):
        input = self.quant(input)
        qweight, qbias = self._qparams(self.weight, self.bias)
        return F.linear(input, qweight, qbias)


class QuantNLinear(nn.Linear):
    """utils/quantize.py:350-363."""

    def __init__(self, in_features, out_features, bias=True, num_bits=8, num_bits_act=8, momentum=0.1):
        super().__init__(in_features, out_features, bias)
        self.quant = QuantMeasure(num_bits=num_bits_act, momentum=momentum)

    def forward(self, input):
        return F.linear(self.quant(input), self.weight, self.bias)


class QConv2d(QuantConv2d):
    """QConv2d with the (unused by main_dfq) scale/scale_prev hooks
    (utils/quantize.py:129-210)."""

    def set_scale(self, scale=None, scale_prev=None):
        if scale is not None:
            self.register_parameter("scale", nn.Parameter(scale.view(-1, 1, 1, 1)))
        if scale_prev is not None:
            self.scale_prev = scale_prev

    def _scaled(self):
        w, b = self.weight, self.bias
        sp = getattr(self, "scale_prev", None)
        if sp is not None:
            step, step_s = w.shape[0] // self.groups, w.shape[1]
            sp = sp[:, 0, 0, 0].view(1, -1, 1, 1)
            w = torch.cat([w[g * step:(g + 1) * step] / sp[:, g * step_s:(g + 1) * step_s]
                           for g in range(self.groups)])
        sc = getattr(self, "scale", None)
        if sc is not None:
            w = w * sc
            b = b * sc.view(-1) if b is not None else None
        return w, b

    def merge_scale_to_weight(self):
        with torch.no_grad():
            w, b = self._scaled()
            self.weight.data.copy_(w)
            if b is not None:
                self.bias.data.copy_(b)
        self.scale_prev = None
        self.scale = None
        invalidate_weight_cache()   # written through .data

    def forward(self, input):
        input = self.quant(input)
        w, b = self._scaled()
        qweight, qbias = self._qparams(w, b)
        return F.conv2d(input, qweight, qbias, self.stride, self.padding, self.dilation, self.groups)


class QLinear(QuantLinear):
    """utils/quantize.py:260-324."""

    def set_scale(self, scale=None, scale_prev=None):
        if scale is not None:
            self.register_parameter("scale", nn.Parameter(scale.view(-1, 1)))
        if scale_prev is not None:
            self.scale_prev = scale_prev

    def _scaled(self):
        w, b = self.weight, self.bias
        sp = getattr(self, "scale_prev", None)
        if sp is not None:
            w = w * sp.view(1, -1)
        sc = getattr(self, "scale", None)
        if sc is not None:
            w = w * sc
            b = b * sc.view(-1) if b is not None else None
        return w, b

    def merge_scale_to_weight(self):
        with torch.no_grad():
            w, b = self._scaled()
            self.weight.data.copy_(w)
            if b is not None:
                self.bias.data.copy_(b)
        self.scale_prev = None
        self.scale = None
        invalidate_weight_cache()   # written through .data

    def forward(self, input):
        input = self.quant(input)
        w, b = self._scaled()
        qweight, qbias = self._qparams(w, b)
        return F.linear(input, qweight, qbias)


def set_layer_bits(graph, bits_weight=8, bits_activation=8, bits_bias=16, targ_type=None):
    """utils/quantize.py:366-379, including its quirk: ``QuantMeasure(bits_activation)``
    passes the bit width positionally into ``update_stat`` so activations stay
    8-bit."""
    print("Setting num_bits for targ layers...")
    assert targ_type is not None, "targ_type cannot be None"
    # the new observers' running_min / running_max: views of ONE device buffer of
    # zeros per device (one H2D copy instead of two per layer)
    need = [graph[idx] for idx in graph if type(graph[idx]) in targ_type and hasattr(graph[idx], "quant")]
    by_dev = {}
    for m in need:
        by_dev.setdefault(next(m.parameters()).device, []).append(m)
    for dev, mods in by_dev.items():
        zeros = torch.zeros(2 * len(mods)).to(dev)
        for k, m in enumerate(mods):
            q = QuantMeasure(bits_activation)
            q._buffers["running_min"] = zeros[2 * k:2 * k + 1]
            q._buffers["running_max"] = zeros[2 * k + 1:2 * k + 2]
            m.quant = q
    for idx in graph:
        if type(graph[idx]) in targ_type:
            if hasattr(graph[idx], "num_bits"):
                graph[idx].num_bits = bits_weight
            if hasattr(graph[idx], "num_bits_bias"):
                graph[idx].num_bits_bias = bits_bias
