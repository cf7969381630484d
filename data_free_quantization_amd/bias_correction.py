"""Drop-in for the reference's ``bias_correction.py`` (bias_correction.py:1-258).

The host walk is the reference's, quirks included:
it iterates ``enumerate(graph.values())`` and looks the *index* up in
``bottoms`` (:185-190), so with opaque graph keys every layer is skipped (the
reference's effective no-op), and with positional keys the coded arithmetic runs.
The arithmetic is HIP:
  * E[o,i] = sum_k (Q(W) - W)[o,i,k]   -- the quantize sweep's error sums
    (``_quantize_error`` + spatial sum, :128-131,231)
  * expect from BN fake stats            -- ``dfq_bc_expect`` (:33-53,170-172)
  * bias += mean_j (E + expect)[o, j]     -- ``dfq_bc_apply`` (:61-106)
  * next BN fake_bias += mean over rows   -- ``dfq_bc_propagate`` (:206-213)
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
from collections.abc import Mapping
import logging

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .utils.layer_transform import find_prev_bn
from .utils.quantize import fake_quant

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger(__name__)


def _buf(m, name):
    """A module's registered buffer without Module.__getattr__ (else getattr)."""
    b = getattr(m, "_buffers", None)
    if b is not None and name in b:
        return b[name]
    return getattr(m, name)


def _param(m, name):
    """A module's registered parameter (None if registered as None) without
    Module.__getattr__ (else getattr, None if absent)."""
    p = getattr(m, "_parameters", None)
    if p is not None and name in p:
        return p[name]
    return getattr(m, name, None)


def _bc_expect(bn_weight, bn_bias, relu, out=None):
    """calculate_mean (γφ(-β/γ) + β(1-Φ(-β/γ)), clamped at 0) when a ReLU follows the
    BN, else β; ``out`` given: accumulate into it (the 'add' branch sum)."""
    _lib.require_device(bn_weight, bn_bias, out)
    acc = out is not None
    if out is None:
        out = torch.empty_like(bn_bias)
    rc = _lib.load().dfq_bc_expect(_lib.ptr(bn_weight), _lib.ptr(bn_bias), bn_bias.numel(), int(bool(relu)),
                                   int(acc), _lib.ptr(out), _lib.stream_of(bn_bias))
    _lib.check(rc, "dfq_bc_expect")
    return out


def _calculate_bias_correction_for_branches(bn_branch, calculate_mean=None):
    """bias_correction.py:15-58 (``calculate_mean`` is the HIP expectation)."""
    res = {}
    for key, branch in bn_branch.items():
        cum = None
        connect_type = None
        for layer, relu_attached, connect_type in branch:
            if connect_type == "cat":
                e = _bc_expect(layer.fake_weight, layer.fake_bias, relu_attached)
                cum = e if cum is None else torch.cat([cum, e])
            elif cum is None:
                cum = _bc_expect(layer.fake_weight, layer.fake_bias, relu_attached)
            else:
                _bc_expect(layer.fake_weight, layer.fake_bias, relu_attached, out=cum)
        res[key] = (connect_type, cum)
    return res


def _broadcast_cols(i2: int, f: int) -> int:
    if i2 == f or f == 1:
        return i2
    if i2 == 1:
        return f
    raise RuntimeError(f"The size of tensor a ({i2}) must match the size of tensor b ({f}) at non-singleton "
                       "dimension 1")


def _apply_bias_correction_E(layer, E, o, i2, connect_type, expect):
    """_compute_final_bias_correction + _apply_bias_correction (:61-106) on the
    device; returns the [o*bcols] bias_vec (kept for the next BN)."""
    if connect_type == "cat":
        # torch.cat([eps (2-D), expect (1-D)]) raises in the reference (:74-75)
        raise RuntimeError("Tensors must have same number of dimensions: got 2 and 1")
    if layer.bias is None:   # :89-90 references an undefined `nn`
        raise NameError("name 'nn' is not defined")
    f = expect.numel()
    bcols = _broadcast_cols(i2, f)
    if o * bcols <= o:
        logger.error("Error in applying bias correction: Bias correction shape mismatch that cannot be handled "
                     "automatically.")
        raise ValueError("Bias correction shape mismatch that cannot be handled automatically.")
    vec = torch.empty(o * bcols, dtype=torch.float32, device=E.device)
    out_cols = C.c_int64(0)
    rc = _lib.load().dfq_bc_apply(_lib.ptr(E), o, i2, _lib.ptr(expect), f, _lib.ptr(layer.bias.data),
                                  _lib.ptr(vec), C.byref(out_cols), _lib.stream_of(E))
    _lib.check(rc, "dfq_bc_apply", ValueError)
    return vec


def _compute_final_bias_correction(eps, bn_values):
    """bias_correction.py:61-80: eps (+) expect, or torch.cat for a 'cat' branch
    (which raises for a 2-D eps, as in the reference)."""
    connect_type, expect = bn_values
    if connect_type == "cat":
        return torch.cat([eps, expect])
    return eps + expect


def _apply_bias_correction(layer, bias):
    """bias_correction.py:82-106: add ``bias`` to ``layer.bias`` -- directly when the
    shapes match, else its per-output-channel mean (``bias.view(O, -1).mean(1)`` in
    ATen's order, ``dfq_bc_apply`` with a zero expectation)."""
    if layer.bias is None:   # :89-90 references an undefined `nn`
        raise NameError("name 'nn' is not defined")
    if bias.size() == layer.bias.size():
        layer.bias.data.add_(bias)
        return
    if bias.numel() <= layer.bias.data.numel():
        raise ValueError("Bias correction shape mismatch that cannot be handled automatically.")
    o = layer.bias.size(0)
    if bias.numel() % o:
        raise RuntimeError(f"shape '[{o}, -1]' is invalid for input of size {bias.numel()}")
    E = bias.detach().contiguous().view(-1)
    _lib.require_device(E, layer.bias.data)
    zero = torch.zeros(1, dtype=torch.float32, device=E.device)
    vec = torch.empty_like(E)
    out_cols = C.c_int64(0)
    rc = _lib.load().dfq_bc_apply(_lib.ptr(E), o, E.numel() // o, _lib.ptr(zero), 1, _lib.ptr(layer.bias.data),
                                  _lib.ptr(vec), C.byref(out_cols), _lib.stream_of(E))
    _lib.check(rc, "dfq_bc_apply", ValueError)


def _quantize_error(param, num_bits=8, reduction="none", signed=False):
    """bias_correction.py:111-144: Q(param) - param (per-tensor range), reduced."""
    x = param.detach().contiguous()
    r = fake_quant(x, num_bits, symmetric=signed, want_codes=False, khw=1, want_esum=True)
    err = r.esum.view_as(x)
    if reduction == "sum":
        return torch.sum(torch.abs(err))
    if reduction == "mean":
        return torch.mean(torch.abs(err))
    if reduction == "channel":
        return torch.sum(torch.abs(err.view(err.size(0), -1)), dim=-1)
    if reduction == "spatial":
        return torch.sum(torch.abs(err.view(err.size(0), err.size(1), -1)), dim=-1)
    if reduction == "none" or reduction is None:
        return err
    raise ValueError(f"Unknown reduction method: {reduction}")


def _error_sums(weight, bits, signed, precomputed=None):
    """E [O, I] = sum over KH*KW of the per-tensor quantization error, as a chain
    ref (tensor, float offset).  ``precomputed``: E as a tensor, or as a
    (buffer, float offset, numel) ref (layer_transform.esum_source: no view)."""
    sh = weight.shape
    o, i2 = sh[0], sh[1]
    if precomputed is not None:
        if isinstance(precomputed, torch.Tensor):
            return (precomputed.view(o * i2), 0), o, i2   # the reference's .view errors on a wrong size
        t, off, n = precomputed
        if n != o * i2:
            raise RuntimeError(f"shape '[{o}, {i2}]' is invalid for input of size {n}")
        return (t, off), o, i2
    khw = weight.numel() // (o * i2)
    r = fake_quant(weight.detach().contiguous(), bits, symmetric=signed, want_codes=False, khw=khw,
                   want_esum=True)
    return (r.esum, 0), o, i2


class _Snapshot(Mapping):
    """{name: clone} whose values are views of ONE buffer, made on first access
    (the walk itself never reads them)."""

    def __init__(self, flat, spans):
        self._flat, self._spans, self._views = flat, spans, {}

    def __getitem__(self, name):
        v = self._views.get(name)
        if v is None:
            off, shape, n = self._spans[name]
            v = self._views[name] = self._flat[off:off + n].view(shape)
        return v

    def __iter__(self):
        return iter(self._spans)

    def __len__(self):
        return len(self._spans)


def _snapshot(chain, tensors, which=0, keys=None):
    """{name: t.clone()} (bias_correction.py:196,255 clone each bias) in one
    buffer, filled by COPY ops recorded in the chain, so the copies run in walk
    order with the rest of the chain's work.  (``which`` / ``keys``: the
    snapshot's symbolic names for a recorded walk.)"""
    if not tensors:
        return {}
    vals = list(tensors.values())
    _lib.require_device(*vals)
    flat = torch.empty(sum(t.numel() for t in vals), dtype=torch.float32, device=vals[0].device)
    spans, off = {}, 0
    for i, (name, t) in enumerate(tensors.items()):
        n = t.numel()
        chain.copy(t, flat, off, (_S_BIAS, keys[i], 0) if keys else _NULL, (_S_SNAP, which, 0))
        spans[name] = (off, t.shape, n)
        off += n
    return _Snapshot(flat, spans)


# symbolic address spaces of a recorded walk (_WalkTemplate): (space, key, float offset)
_S_NONE, _S_BN_W, _S_BN_B, _S_BIAS, _S_E, _S_SCRATCH, _S_SNAP = range(7)
_NULL = (_S_NONE, 0, 0)

_BC_OP = np.dtype([("kind", "<i4"), ("flag", "<i4"), ("a", "<u8"), ("b", "<u8"), ("out", "<u8"), ("out2", "<u8"),
                   ("n", "<i8"), ("i2", "<i8"), ("f", "<i8")])
assert _BC_OP.itemsize == C.sizeof(_lib.BcOp)


#: scratch floats per chunk of the chain's expectation / bias-vector slots
_SCRATCH_CHUNK = 1 << 22
#: recorded ops that trigger a flush between target layers: the device works
#: through the walk's first layers while Python walks the rest
_FLUSH_OPS = 32


class _BcChain:
    """The walk's device work recorded in graph order and enqueued by
    ``dfq_bc_chain`` calls (instead of a Python call per expect / apply /
    propagate).  Expectations and bias vectors live in scratch chunks allocated
    as the walk goes, so every ref ``(tensor, float offset)`` is a device address
    at once and the recorded ops can be flushed at any point: the walk flushes
    once ``_FLUSH_OPS`` ops are recorded, at a BN node right after its
    propagate (so a layer's expect / apply / propagate group reaches the library
    in one call, which runs it as one launch), and before it raises, so the ops
    before an error take effect, as in the reference.  Ops are recorded as rows
    of plain integers (device addresses computed once, at record time)."""

    def __init__(self, dev, record=False):
        self.dev = dev
        self.ops = []
        self.keep = []          # tensors the recorded ops point into
        self._chunk = None      # current scratch chunk
        self._base = 0          # its device address
        self._fill = 0          # floats used in it
        self._chunks = []       # chunks the unflushed ops point into
        # record=True: every op also as a symbolic row (_WalkTemplate) -- its
        # addresses as (space, key, float offset) -- and the flush points
        self.sym = [] if record else None
        self.flushes = []
        self._nchunk = -1       # ordinal of the current scratch chunk
        self.chunk_fill = []    # floats used per scratch chunk

    def alloc(self, n):
        """A 256-B aligned scratch slot of n floats: (chunk, offset, address)."""
        need = -(-n // 64) * 64
        if self._chunk is None or self._fill + need > self._chunk.numel():
            self._chunk = torch.empty(max(need, _SCRATCH_CHUNK), dtype=torch.float32, device=self.dev)
            self._base = self._chunk.data_ptr()
            self._chunks.append(self._chunk)
            self._fill = 0
            self._nchunk += 1
            self.chunk_fill.append(0)
        off = self._fill
        self._fill += need
        self.chunk_fill[self._nchunk] = self._fill
        return (self._chunk, off, self._base + 4 * off, (_S_SCRATCH, self._nchunk, off))

    def extend_last(self, ref, size, n):
        """Grow the most recent slot ``ref`` ([size] floats) by n (torch.cat):
        in place when its chunk has room, else into a fresh slot that a COPY op
        fills with the size floats already written.  Returns the slot's ref."""
        t, off, addr, _ = ref
        assert t is self._chunk and self._fill == off + -(-size // 64) * 64, "cat target is not the last slot"
        need = -(-(size + n) // 64) * 64
        if off + need <= t.numel():
            self._fill = off + need
            self.chunk_fill[self._nchunk] = self._fill
            return ref
        new = self.alloc(size + n)
        self._op((_lib.DFQ_BC_OP_COPY, 0, addr, 0, new[2], 0, size, 0, 0), (ref[3], _NULL, new[3], _NULL))
        return new

    def _op(self, row, syms):
        self.ops.append(row)
        if self.sym is not None:
            self.sym.append((row, syms))

    def expect(self, bn, relu, dst, accumulate, bn_key=None):
        w, b = _buf(bn, "fake_weight"), _buf(bn, "fake_bias")
        _lib.require_device(w, b)
        self.keep += [w, b]
        self._op((_lib.DFQ_BC_OP_EXPECT, int(bool(relu)) | (int(accumulate) << 1), w.data_ptr(),
                  b.data_ptr(), dst[2], 0, b.numel(), 0, 0),
                 ((_S_BN_W, bn_key, 0), (_S_BN_B, bn_key, 0), dst[3], _NULL))

    def apply(self, E, o, i2, expect, f, bias, vec, key=None):
        # E: a ref (tensor, float offset); vec: a scratch slot only this chain's propagate reads
        e, eoff = E
        self.keep += [e, bias]
        self._op((_lib.DFQ_BC_OP_APPLY, _lib.DFQ_BC_APPLY_VEC_SCRATCH, e.data_ptr() + 4 * eoff, expect[2],
                  bias.data_ptr(), vec[2], o, i2, f),
                 ((_S_E, key, 0), expect[3], (_S_BIAS, key, 0), vec[3]))

    def propagate(self, vec, numel, fake_b, f, bn_key=None):
        _lib.require_device(fake_b)
        self.keep.append(fake_b)
        self._op((_lib.DFQ_BC_OP_PROPAGATE, _lib.REF_THREADS, vec[2], 0, fake_b.data_ptr(), 0, numel, 0, f),
                 (vec[3], _NULL, (_S_BN_B, bn_key, 0), _NULL))

    def copy(self, src, dst, off, src_sym=_NULL, dst_sym=_NULL):   # src / dst validated by the caller
        self.keep += [src, dst]
        self._op((_lib.DFQ_BC_OP_COPY, 0, src.data_ptr(), 0, dst.data_ptr() + 4 * off, 0, src.numel(), 0, 0),
                 (src_sym, _NULL, (dst_sym[0], dst_sym[1], off), _NULL))

    def flush(self, stream):
        if not self.ops:
            return
        if self.sym is not None:
            self.flushes.append(len(self.sym))
        # the op table as a numpy record array (layout of _lib.BcOp) from the rows of integers
        arr = np.array(self.ops, dtype=_BC_OP)
        failed = C.c_int32(-1)
        rc = _lib.load().dfq_bc_chain(arr.ctypes.data_as(C.POINTER(_lib.BcOp)), len(self.ops), C.byref(failed),
                                      stream)
        _lib.check(rc, f"dfq_bc_chain (op {failed.value})", RuntimeError)
        # the ops run asynchronously: the scratch chunks stay with the current stream
        cur = torch.cuda.current_stream(self.dev)
        for t in self._chunks:
            t.record_stream(cur)
        self._chunks = [self._chunk] if self._chunk is not None else []
        self.ops, self.keep = [], []


def _record_branches(chain, bn_branch):
    """_calculate_bias_correction_for_branches (bias_correction.py:15-58) as chain
    ops: {key: (connect_type, expect ref, numel)}."""
    res = {}
    for key, branch in bn_branch.items():
        ref, size, connect_type = None, 0, None
        for layer, relu_attached, connect_type, bn_key in branch:
            n = _buf(layer, "fake_bias").numel()
            if ref is None:
                ref, size = chain.alloc(n), n
                chain.expect(layer, relu_attached, ref, False, bn_key)
            elif connect_type == "cat":   # torch.cat([cum, e]): e lands right after cum
                ref = chain.extend_last(ref, size, n)
                sym = ref[3]
                chain.expect(layer, relu_attached, (ref[0], ref[1] + size, ref[2] + 4 * size,
                                                    (sym[0], sym[1], sym[2] + size)), False, bn_key)
                size += n
            else:                          # cum += e (in place)
                if n != size:
                    raise RuntimeError(f"output with shape [{size}] doesn't match the broadcast shape [{n}]"
                                       if n != 1 else "a one-channel BN expectation broadcast is not supported")
                chain.expect(layer, relu_attached, ref, True, bn_key)
        res[key] = (connect_type, ref, size)
    return res


def _record_apply(chain, layer, E, o, i2, connect_type, expect, f, key=None):
    """_apply_bias_correction_E's checks, then one chain op; returns the bias_vec
    ref and its numel (kept for the next BN)."""
    if connect_type == "cat":
        raise RuntimeError("Tensors must have same number of dimensions: got 2 and 1")
    bias = _param(layer, "bias")
    if bias is None:   # :89-90 references an undefined `nn`
        raise NameError("name 'nn' is not defined")
    bcols = _broadcast_cols(i2, f)
    if o * bcols <= o:
        logger.error("Error in applying bias correction: Bias correction shape mismatch that cannot be handled "
                     "automatically.")
        raise ValueError("Bias correction shape mismatch that cannot be handled automatically.")
    _lib.require_device(E[0], bias)
    vec = chain.alloc(o * bcols)
    chain.apply(E, o, i2, expect, f, bias, vec, key)
    return vec, o * bcols


#: compiled walks (_WalkTemplate) by the graph's structure, most recent last
_TEMPLATES = OrderedDict()
_TEMPLATE_CAP = 8


#: node kind per (module type, targ_type, bn_type): 1 BN, 2 target layer, 0 other
_KINDS = {}


def _structure(graph, bottoms, targ_type, bn_type, signed, bits_weight, error_sums):
    """Everything the walk's control flow and op fields depend on (the graph's
    keys, node types, bottoms, the shapes of targets / biases / BN statistics /
    error sums), as a hashable signature of flat tuples (cheap to hash and to
    compare); plus what a replay takes addresses from: per node index two device
    addresses (BN: fake_weight, fake_bias; target layer: bias, E) and the tensors
    behind them.  The walk never reads a tensor value."""
    shp = []
    kinds = _KINDS
    keys = tuple(graph.keys())
    vals = list(graph.values())
    types = tuple(map(type, vals))
    ptrs = [(0, 0)] * len(vals)
    tensors = []
    for i, v in enumerate(vals):
        t = types[i]
        k = kinds.get((t, targ_type, bn_type))
        if k is None:
            k = kinds[(t, targ_type, bn_type)] = (1 if issubclass(t, bn_type) else
                                                  2 if issubclass(t, targ_type) and t is not str else 0)
        if k == 1:
            bufs = getattr(v, "_buffers", {})
            fw, fb = bufs.get("fake_weight"), bufs.get("fake_bias")
            if fw is None or fb is None:   # a BN merge_batchnorm never folded: the walk must not use it
                shp += (i, -7)             # (the live walk raises, as the reference does, if it does)
                continue
            ptrs[i] = (fw.data_ptr(), fb.data_ptr())
            tensors += (fw, fb)
            shp += (i, -1, *fw.shape, -2, *fb.shape)
        elif k == 2:
            w, b = _param(v, "weight"), _param(v, "bias")
            pre = error_sums.get(keys[i])
            if pre is None:
                e = 0
            elif isinstance(pre, torch.Tensor):   # E itself, or a (buffer, float offset, numel) ref
                e = pre.data_ptr()
                tensors.append(pre)
            else:
                e = pre[0].data_ptr() + 4 * pre[1]
                tensors.append(pre[0])
            if b is not None:
                tensors.append(b)
            ptrs[i] = (0 if b is None else b.data_ptr(), e)
            shp += (i, -3, *w.shape, -4, *(() if b is None else b.shape), -5 if b is None else -6,
                    -1 if pre is None else (pre.numel() if isinstance(pre, torch.Tensor) else pre[2]))
    sig = (keys, types, tuple(bottoms.keys()),
           tuple(None if v is None else tuple(v) for v in bottoms.values()), targ_type, bn_type, bool(signed),
           int(bits_weight), _lib.REF_THREADS, tuple(shp))
    return sig, (np.array(ptrs, dtype=np.int64), tensors)


class _WalkTemplate:
    """A recorded walk (record=True chain): its ops with symbolic addresses, the
    warnings it logged and the before / after snapshot layouts.  ``replay`` binds
    the addresses of another graph of the same structure and enqueues every op in
    one dfq_bc_chain call."""

    def __init__(self, chain, warnings_, before, after):
        # the recording as it is; the tables are built at the first replay, so a
        # walk that is never replayed costs only its recording
        self.warnings = list(warnings_)
        self.before = (dict(before._spans), before._flat.numel()) if before else None
        self.after = (dict(after._spans), after._flat.numel()) if after else None
        self._raw = (chain.sym, list(chain.chunk_fill))
        self.static = None

    def _build(self):
        sym, chunk_fill = self._raw
        self.static = np.array([(row[0], row[1], row[6], row[7], row[8]) for row, _ in sym], dtype=np.int64)
        # scratch chunks -> one buffer; symbolic slots -> indices into an address vector
        cbase, tot = [], 0
        for fill in chunk_fill:
            cbase.append(tot)
            tot += fill
        self.scratch = -(-tot // 64) * 64
        snap = [0 if x is None else -(-x[1] // 64) * 64 for x in (self.before, self.after)]
        # one device allocation per replay: [scratch | before snapshot | after snapshot]
        self.snap_off = (self.scratch, self.scratch + snap[0])
        self.alloc = max(self.scratch + snap[0] + snap[1], 1)
        slots = {}          # (space, key) -> index; 0 = null
        keys = [(_S_NONE, 0)]
        idx = np.zeros((len(sym), 4), dtype=np.int64)
        off = np.zeros((len(sym), 4), dtype=np.int64)
        for k, (_, syms) in enumerate(sym):
            for j, (space, key, o) in enumerate(syms):
                if space == _S_NONE:
                    continue
                if space == _S_SCRATCH:
                    key, o = 0, cbase[key] + o
                sk = (space, key)
                if sk not in slots:
                    slots[sk] = len(keys)
                    keys.append(sk)
                idx[k, j], off[k, j] = slots[sk], o
        self.idx, self.off = idx, off
        # per slot: the node index and the field of _structure's address table
        # (BN weight / bias; bias / E), or a float offset into the replay's allocation
        self.slot_node = np.array([key if sp in (_S_BN_W, _S_BN_B, _S_BIAS, _S_E) else 0 for sp, key in keys],
                                  dtype=np.int64)
        self.slot_field = np.array([1 if sp in (_S_BN_B, _S_E) else 0 for sp, _ in keys], dtype=np.int64)
        self.slot_tab = np.array([sp in (_S_BN_W, _S_BN_B, _S_BIAS, _S_E) for sp, _ in keys])
        self.slot_local = np.array([0 if sp == _S_SCRATCH else self.snap_off[key] if sp == _S_SNAP else -1
                                    for sp, key in keys], dtype=np.int64)
        self._raw = None

    def replay(self, where, dev, stream):
        if self.static is None:
            self._build()
        for m in self.warnings:
            logger.warning(m)
        ptrs, tensors = where
        _lib.require_device(*tensors)
        buf = torch.empty(self.alloc, dtype=torch.float32, device=dev)
        base = np.zeros(len(self.slot_node), dtype=np.int64)
        base[self.slot_tab] = ptrs[self.slot_node[self.slot_tab], self.slot_field[self.slot_tab]]
        if not base[self.slot_tab].all():   # a tensor the recorded walk used is missing here
            raise RuntimeError("bias_correction: an error sum the compiled walk reads is missing")
        loc = self.slot_local >= 0
        base[loc] = buf.data_ptr() + 4 * self.slot_local[loc]
        a = base[self.idx] + 4 * self.off
        a[self.idx == 0] = 0
        arr = np.empty(len(self.static), dtype=_BC_OP)
        arr["kind"], arr["flag"] = self.static[:, 0], self.static[:, 1]
        arr["n"], arr["i2"], arr["f"] = self.static[:, 2], self.static[:, 3], self.static[:, 4]
        for j, name in enumerate(("a", "b", "out", "out2")):
            arr[name] = a[:, j].astype(np.uint64)
        if len(arr):
            failed = C.c_int32(-1)
            rc = _lib.load().dfq_bc_chain(arr.ctypes.data_as(C.POINTER(_lib.BcOp)), len(arr), C.byref(failed), stream)
            _lib.check(rc, f"dfq_bc_chain (op {failed.value})", RuntimeError)
            buf.record_stream(torch.cuda.current_stream(dev))
        before = _Snapshot(buf[self.snap_off[0]:self.snap_off[0] + self.before[1]], self.before[0]) if self.before else {}
        after = _Snapshot(buf[self.snap_off[1]:self.snap_off[1] + self.after[1]], self.after[0]) if self.after else {}
        return before, after


def bias_correction(graph, bottoms, targ_type, bits_weight=8, bn_type=torch.nn.BatchNorm2d, signed=False, *,
                    error_sums=None):
    """Returns (bias_before_correction, bias_after_correction) keyed "layer_<idx>"
    (read-only mappings whose tensors are views made on first access; the
    reference returns dicts of clones).

    ``error_sums`` (extension, ``--bc_mode fused``): {graph key: E} from the fused
    quantize sweep, used instead of re-quantizing the (already quantized) weight."""
    assert isinstance(graph, dict), "Expected 'graph' to be a dictionary."
    assert isinstance(bottoms, dict), "Expected 'bottoms' to be a dictionary."
    assert isinstance(targ_type, (type, tuple)), "Expected 'targ_type' to be a type or tuple of types."
    logger.info("Starting bias correction...")
    _lib.weights_changed()
    # A graph of a structure walked before replays the compiled walk: the walk's
    # control flow and every op's fields depend on the structure only (keys, node
    # types, bottoms, shapes), never on a tensor value; the addresses are bound
    # afresh.  Only fused-mode walks (error sums given) are compiled: the other
    # mode quantizes each weight inside the walk.
    sig = where = None
    if error_sums is not None:
        sig, where = _structure(graph, bottoms, targ_type, bn_type, signed, bits_weight, error_sums)
        tpl = _TEMPLATES.get(sig)
        if tpl is not None:
            _TEMPLATES.move_to_end(sig)
            dev = where[1][0].device if where[1] else torch.device("cuda", torch.cuda.current_device())
            with torch.no_grad():
                res = tpl.replay(where, dev, _lib.raw_stream(dev))
            logger.info("Bias correction completed.")
            return res
    warned = []
    bn_module, relu_attached, bn_key = {}, {}, {}
    bias_prev = None        # device bias_vec of the last corrected layer (negated when used)
    bias = None             # persists across layers like the reference's local
    before, after = {}, {}
    keys = list(graph.keys())
    after_src = {}
    with torch.no_grad():
        # The walk only writes the bias of the layer it is on, after recording it, so
        # every "before" value is the bias at entry: one batched copy instead of a
        # clone per layer (and likewise for "after", at the end).
        biases = {}
        for i, l in enumerate(graph.values()):
            if i in bottoms and isinstance(l, targ_type):
                b = _param(l, "bias")
                if b is not None:
                    biases[f"layer_{i}"] = b   # read through data_ptr only (no .data view)
        chain = _BcChain(next(iter(biases.values())).device if biases else torch.device("cuda"),
                         record=sig is not None)
        before = _snapshot(chain, biases, 0, [int(k[6:]) for k in biases])
        stream = None
        try:
            for idx_layer, layer in enumerate(graph.values()):
                layer_name = f"layer_{idx_layer}"
                if idx_layer not in bottoms:
                    warned.append(f"Layer index {idx_layer} not found in bottoms")
                    logger.warning(warned[-1])
                    continue
                bot = bottoms[idx_layer]
                if bot is None or bot[0] == "Data":
                    continue
                node = graph[idx_layer]
                if isinstance(node, bn_type):
                    bn_module[idx_layer] = node
                    bn_key[id(node)] = idx_layer
                    relu_attached[idx_layer] = False
                    if bias_prev is not None:
                        vec, numel = bias_prev
                        fake_b = _buf(node, "fake_bias")
                        f = fake_b.size(0)
                        if numel == f:
                            # fake_bias.add_(bias_prev) with a 2-D bias_prev cannot broadcast in place
                            raise RuntimeError("output with shape [{}] doesn't match the broadcast shape".format(f))
                        if numel % f:
                            raise RuntimeError(f"shape '[-1, {f}]' is invalid for input of size {numel}")
                        chain.propagate(vec, numel, fake_b, f, idx_layer)
                        bias_prev = None
                        if len(chain.ops) >= _FLUSH_OPS:   # the device starts on what is recorded so far
                            chain.flush(stream)
                    continue
                if isinstance(node, torch.nn.ReLU) and bot[0] in bn_module:
                    relu_attached[bot[0]] = True
                if isinstance(node, targ_type):
                    bn_list, relu_list, type_list, no_bn = find_prev_bn(bn_module, relu_attached, graph, bottoms,
                                                                        bot[:])
                    if no_bn:   # find_prev_bn printed a warning: not a walk to replay silently
                        sig = None
                    pre = None if error_sums is None else error_sums.get(keys[idx_layer])
                    if pre is None:   # E computed inside the walk (a fake quant outside the chain): not replayable
                        sig = None
                    E, o, i2 = _error_sums(_param(node, "weight"), bits_weight, signed, pre)
                    if stream is None:
                        stream = _lib.stream_of(E[0])
                        chain.dev = E[0].device
                    branches = {}
                    for j, (bn_layer, bid) in enumerate(bn_list):
                        branches.setdefault(bid[0], []).append((bn_layer, relu_list[j], type_list[j],
                                                                bn_key.get(id(bn_layer))))
                    for connect_type, expect, f in _record_branches(chain, branches).values():
                        try:
                            bias = _record_apply(chain, node, E, o, i2, connect_type, expect, f, idx_layer)
                        except ValueError as e:
                            logger.error(f"Error in applying bias correction: {e}")
                            raise
                    if bias is None:
                        raise UnboundLocalError("local variable 'bias' referenced before assignment")
                    bias_prev = bias
                    b = _param(layer, "bias")
                    if b is not None:
                        after_src[layer_name] = b
            after = _snapshot(chain, after_src, 1, [int(k[6:]) for k in after_src])
        finally:   # the ops recorded before an error still take effect, as in the reference
            if chain.ops:
                chain.flush(stream if stream is not None else _lib.stream_of(next(iter(biases.values()))))
    if sig is not None and all(isinstance(k, int) for k in bn_key.values()):
        _TEMPLATES[sig] = _WalkTemplate(chain, warned, before, after)
        if len(_TEMPLATES) > _TEMPLATE_CAP:
            _TEMPLATES.popitem(last=False)
    logger.info("Bias correction completed.")
    return before, after
