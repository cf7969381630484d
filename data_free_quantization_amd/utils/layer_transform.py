"""Drop-in for the DFQ-path functions of the reference's ``utils/layer_transform.py``:

* ``merge_batchnorm``     (utils/layer_transform.py:240-285) -> HIP ``dfq_bn_fold``
* ``quantize_targ_layer`` (utils/layer_transform.py:288-305) -> one grouped HIP sweep
* ``find_prev_bn``        (utils/layer_transform.py:308-353) host graph walk
* ``switch_layers``       (utils/layer_transform.py:161-197) with this package's tracer
* ``set_quant_minmax``    (utils/layer_transform.py:356-618) -> HIP ``dfq_act_*``
* ``replace_op`` / ``restore_op`` (utils/layer_transform.py:128-158): tensor-op
  input quantization during inference

Graph/bottoms follow SURVEY.md 8b.  Target tensors must be on a ROCm device.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import time
from collections.abc import Mapping
import types
from typing import Dict, Optional

import numpy as np

import torch
import torch.nn as nn

from .. import _lib
from ..sweep import SweepItem, SweepPlan, khw_of
from .quantize import (QConv2d, QLinear, QuantConv2d, QuantLinear, QuantMeasure, QuantNConv2d,
                       QuantNLinear)
from .tracer import TorchTransformer

_CONV_TYPES = (nn.Conv2d, QConv2d, QuantConv2d, QuantNConv2d)
_LINEAR_TYPES = (nn.Linear, QLinear, QuantLinear, QuantNLinear)


def merge_batchnorm(model, graph, bottoms, targ_type=[QConv2d], *, ranges: Optional[Dict] = None):
    """Fold each BatchNorm2d into the target layer feeding it, keep |gamma| and beta
    as ``fake_weight``/``fake_bias`` buffers, and turn the BN into an identity
    (utils/layer_transform.py:240-285).  Every fold of the model runs in one
    ``dfq_bn_fold_batch`` call (two launches).

    ``ranges`` (extension): a dict that receives {layer: 2 int32 device words},
    each folded weight's (min, max) as a by-product of the fold's read, for
    ``quantize_targ_layer(weight_ranges=...)`` right after (main_dfq.py:211-214:
    the second fold, whose factors are exactly 1, then only reads the weights)."""
    pairs = []
    targ = tuple(targ_type)
    for layer_idx, bn in graph.items():   # BN nodes first: most nodes are not (the same pairs, in graph order)
        if type(bn) is not nn.BatchNorm2d:
            continue
        bots = bottoms[layer_idx]
        if bots is None:
            continue
        for bot_idx in bots:
            layer = graph[bot_idx]
            if type(layer) in targ:
                pairs.append((bn, layer))
                break
    if not pairs:
        return model
    # a layer feeding two BNs is folded twice in sequence by the reference: one
    # batch call per fold then, in graph order
    if len({id(layer._parameters["weight"]) for _, layer in pairs}) < len(pairs):
        for pair in pairs:
            _fold_batch([pair], ranges)
    else:
        _fold_batch(pairs, ranges)
    return model


# dfq_bn_fold_desc as a numpy record (same layout as _lib.BnFoldDesc): the table
# of a model's folds is filled column-wise instead of field by field
_BN_DESC = np.dtype([("ptr", "<u8", (8,)), ("eps", "<f4"), ("flags", "<i4"), ("rows", "<i8"),
                     ("row_len", "<i8"), ("range_enc", "<u8")])
assert _BN_DESC.itemsize == C.sizeof(_lib.BnFoldDesc)


_BN_TIMING = bool(os.environ.get("DFQ_BN_TIMING"))   # host-side split of the fold (stderr)


def _fold_batch(pairs, ranges=None):
    tb = [time.perf_counter()] if _BN_TIMING else None
    _lib.weights_changed()
    with torch.no_grad():
        # module state straight from the parameter / buffer dicts: Module.__getattr__
        # on every access was most of this function's host time
        lps = [layer._parameters for _, layer in pairs]
        bps = [bn._parameters for bn, _ in pairs]
        bbs = [bn._buffers for bn, _ in pairs]
        W = [lp["weight"] for lp in lps]
        Bi = [lp.get("bias") for lp in lps]
        G = [bp["weight"] for bp in bps]
        Be = [bp["bias"] for bp in bps]
        Mu = [bb["running_mean"] for bb in bbs]
        Va = [bb["running_var"] for bb in bbs]
        if tb:
            tb.append(time.perf_counter())
        _lib.require_device(*W, *G, *Be, *Mu, *Va, *[b for b in Bi if b is not None])
        if tb:
            tb.append(time.perf_counter())
        dev = W[0].device
        n = len(pairs)
        rows_n = np.array([w.shape[0] for w in W], dtype=np.int64)
        chans = np.array([g.numel() for g in G], dtype=np.int64)
        tab = np.zeros(n, dtype=_BN_DESC)
        ptr = tab["ptr"]
        # :262-263 give a bias-less layer torch.zeros; here the fold reads such a
        # bias as 0 (DFQ_BN_FOLD_ZERO_BIAS) and writes every element of it.  The new
        # biases and the fake weight / bias buffers are views of ONE allocation
        # whose addresses come from the offsets (no data_ptr call per view).
        need = [j for j, b in enumerate(Bi) if b is None]
        nb_f = int(rows_n[need].sum()) if need else 0
        nch = int(chans.sum())
        flat = torch.empty(max(nb_f + 2 * nch, 1), dtype=torch.float32, device=dev)
        base = np.uint64(flat.data_ptr())
        if tb:
            tb.append(time.perf_counter())
        views = torch.split(flat[:nb_f + 2 * nch], [int(rows_n[j]) for j in need] + chans.tolist() * 2)
        if tb:
            tb.append(time.perf_counter())
        for j, z in zip(need, views[:len(need)]):
            layer = pairs[j][1]
            b = torch.Tensor._make_subclass(nn.Parameter, z, False)   # nn.Parameter(z, requires_grad=False)
            if "bias" in layer._parameters:   # registered as None: what Module.__setattr__ would do
                layer._parameters["bias"] = b
            else:
                layer.bias = b
        if tb:
            tb.append(time.perf_counter())
        if need:
            boff = np.zeros(n, dtype=np.uint64)
            boff[need] = np.concatenate([[0], np.cumsum(rows_n[need])[:-1]]).astype(np.uint64)
        coff = np.concatenate([[0], np.cumsum(chans)[:-1]]).astype(np.uint64) + np.uint64(nb_f)
        fw_v, fb_v = views[len(need):len(need) + n], views[len(need) + n:]
        for (bn, _), fw, fb in zip(pairs, fw_v, fb_v):
            buf = bn._buffers   # register_buffer("fake_weight" / "fake_bias") without the per-call checks
            buf["fake_weight"], buf["fake_bias"] = fw, fb
        ptr[:, 0] = [t.data_ptr() for t in W]
        ptr[:, 1] = [0 if t is None else t.data_ptr() for t in Bi]
        if need:
            ptr[need, 1] = base + np.uint64(4) * boff[need]
        ptr[:, 2] = [t.data_ptr() for t in G]
        ptr[:, 3] = [t.data_ptr() for t in Be]
        ptr[:, 4] = [t.data_ptr() for t in Mu]
        ptr[:, 5] = [t.data_ptr() for t in Va]
        ptr[:, 6] = base + np.uint64(4) * coff
        ptr[:, 7] = base + np.uint64(4) * (coff + np.uint64(nch))
        if tb:
            tb.append(time.perf_counter())
        tab["eps"] = [bn.eps for bn, _ in pairs]
        if need:
            tab["flags"][need] = _lib.DFQ_BN_FOLD_ZERO_BIAS
        if ranges is not None:   # 8 bytes per fold, in one allocation (zeroed by the call)
            rbuf = torch.empty(2 * n, dtype=torch.int32, device=dev)
            tab["range_enc"] = rbuf.data_ptr() + 8 * np.arange(n, dtype=np.uint64)
            for j, (_, layer) in enumerate(pairs):
                ranges[layer] = rbuf[2 * j:2 * j + 2]
        tab["rows"] = rows_n
        tab["row_len"] = [w.numel() for w in W] // rows_n
        descs = tab.ctypes.data_as(C.POINTER(_lib.BnFoldDesc))
        L = _lib.load()
        nb = int(L.dfq_bn_fold_ws_bytes(descs, n))
        if nb < 0:
            raise RuntimeError("dfq_bn_fold_ws_bytes: invalid layer shapes")
        ws = torch.empty(max(nb, 256), dtype=torch.uint8, device=dev)   # stream-ordered (caching allocator)
        if tb:
            tb.append(time.perf_counter())
        rc = L.dfq_bn_fold_batch(descs, n, ws.data_ptr(), ws.numel(), _lib.stream_of(W[0]))
        _lib.check(rc, "dfq_bn_fold_batch")
        if tb:
            tb.append(time.perf_counter())
        for bn, _ in pairs:
            bn.__dict__["eps"] = 0   # plain attributes: what Module.__setattr__ ends in
            _identity_forward(bn)
        if tb:
            tb.append(time.perf_counter())
            print("DFQ_BN_TIMING fold x%d: module dicts %.1f us, device checks %.1f us, shapes + allocation %.1f us, "
                  "split %.1f us, bias Parameters %.1f us, fakes + rows %.1f us, tables + workspace "
                  "%.1f us, call %.1f us, identity BNs %.1f us" % ((len(pairs),) + tuple(
                      (b - a) * 1e6 for a, b in zip(tb, tb[1:]))), file=sys.stderr)


_TINY = float(torch.finfo(torch.float32).tiny)


def _folded_bn_forward(self, input):
    """The folded BN (weight 1, bias 0, mean 0, var 1, eps 0 -- the reference's
    state) is an identity, but torch >= 2 rejects eps == 0 in F.batch_norm: run
    the forward with the smallest normal fp32 eps (1 + eps == 1 in fp32, so the
    result is unchanged) and put eps = 0 back afterwards."""
    if self.eps != 0:
        return nn.BatchNorm2d.forward(self, input)
    self.eps = _TINY
    try:
        return nn.BatchNorm2d.forward(self, input)
    finally:
        self.eps = 0


def _identity_forward(bn):
    if "forward" not in bn.__dict__:   # one instance attribute (no per-BN hook objects)
        bn.__dict__["forward"] = types.MethodType(_folded_bn_forward, bn)


def quantize_targ_layer(graph, bit_weight=8, bits_bias=16, targ_type=None, *, granularity="tensor",
                        symmetric=False, clip=None, state: Optional[Dict] = None, shard: bool = False,
                        group=None, weight_ranges: Optional[Dict] = None):
    """Fake-quantize every target layer's weight (and bias when bits_bias < 32) in
    place, all layers in one grouped launch.

    Reference semantics by default (per-tensor asymmetric with float(min)/float(max),
    utils/layer_transform.py:298-303).  Extensions: ``granularity="channel"``,
    ``symmetric=True``, ``clip=(lo, hi)`` fused (the clip_weight clamp), and
    ``state`` -- a dict filled with per-layer codes/scale/zero and the BC error
    sums E[o,i] of this quantization.

    ``weight_ranges`` (per-tensor modes): {layer: device range} from
    ``merge_batchnorm(ranges=...)`` run just before, with no write to the weights in
    between (main_dfq's order): those weights are quantized in one HBM pass
    (DFQ_DEVICE_RANGE) instead of a reduce pass and a quantize pass.

    ``shard=True`` with torch.distributed initialised (main_dfq --world_size N,
    every rank holding the model): each rank sweeps its LPT share of the tensors
    into its slab of an output arena, one in-place all-gather (RCCL) gives every
    rank every result, and each rank writes them back into its parameters
    (distributed.ShardedSweep).  Results are identical to the unsharded call."""
    _lib.weights_changed()
    if shard and torch.distributed.is_initialized():
        return _quantize_targ_layer_sharded(graph, bit_weight, bits_bias, targ_type, granularity=granularity,
                                            symmetric=symmetric, clip=clip, state=state, group=group)
    print("Quantizing Layer parameters")
    if bits_bias == 32:
        print("Skipping bias quantization (32 bits)")
    assert targ_type is not None, "targ_type cannot be None!"
    per_channel = granularity == "channel"
    if granularity not in ("tensor", "channel"):
        raise ValueError("granularity must be 'tensor' or 'channel'")
    items = []
    keys = []
    tt = tuple(targ_type)
    for layer_idx, layer in graph.items():
        if type(layer) not in tt:
            continue
        lp = layer._parameters   # no Module.__getattr__ per access
        w = lp["weight"]   # written in place by the kernel: no .data view needed
        rows = w.size(0) if per_channel else 1
        npar = rows
        khw = khw_of(w)
        it = SweepItem(src=w, dst=w, bits=bit_weight, per_channel=per_channel, symmetric=symmetric, clip=clip,
                       khw=khw, rows=rows,
                       range_enc=weight_ranges.get(layer) if (weight_ranges and not per_channel) else None)
        items.append(it)
        keys.append(layer_idx)
        if lp.get("bias") is not None and bits_bias < 32:
            b = lp["bias"]
            items.append(SweepItem(src=b, dst=b, bits=bits_bias, per_channel=False, symmetric=False, rows=1))
            keys.append(None)
    if not items:
        return graph
    if state is not None:   # codes / scale / zero / E of every layer in two allocations
        wl = [it for it, k in zip(items, keys) if k is not None]
        dev = wl[0].src.device
        cdt = (torch.int8 if symmetric else torch.uint8) if bit_weight <= 8 else torch.int16
        up = lambda k: -(-k // 16) * 16   # noqa: E731  -- 16-element aligned pieces (vector paths)
        spans, co, fo = [], 0, 0
        for it in wl:
            n, r, ne = it.src.numel(), it.rows, it.src.numel() // it.khw
            spans.append((co, fo, n, r, ne))
            co += up(n)
            fo += 2 * up(r) + up(ne)
        codes = torch.empty(max(co, 1), dtype=cdt, device=dev)
        f32 = torch.empty(max(fo, 1), dtype=torch.float32, device=dev)
        cb, fb, cs = codes.data_ptr(), f32.data_ptr(), codes.element_size()
        for it, (c0, f0, n, r, ne) in zip(wl, spans):   # raw addresses: no per-layer views here
            it.codes = cb + cs * c0
            it.scale, it.zero, it.esum = fb + 4 * f0, fb + 4 * (f0 + up(r)), fb + 4 * (f0 + 2 * up(r))
    plan = SweepPlan(items)
    plan.execute()
    plan.destroy()   # stream-ordered: the task tables return to torch's allocator
    if state is not None:
        wk = [k for k in keys if k is not None]
        for k, it, sp in zip(wk, wl, spans):
            state[k] = _StateEntry(codes, f32, sp, tuple(it.src.shape), it.khw, up)
    return graph


class _StateEntry(Mapping):
    """quantize_targ_layer's per-layer outputs {codes, scale, zero, esum, khw}:
    views of the two shared allocations, made on first access."""

    __slots__ = ("_codes", "_f32", "_span", "_shape", "_khw", "_up", "_views")

    def __init__(self, codes, f32, span, shape, khw, up):
        self._codes, self._f32, self._span, self._shape, self._khw, self._up = codes, f32, span, shape, khw, up
        self._views = {}

    def __getitem__(self, key):
        v = self._views.get(key)
        if v is not None:
            return v
        c0, f0, n, r, ne = self._span
        if key == "codes":
            v = self._codes[c0:c0 + n].view(self._shape)
        elif key == "scale":
            v = self._f32[f0:f0 + r]
        elif key == "zero":
            v = self._f32[f0 + self._up(r):f0 + self._up(r) + r]
        elif key == "esum":
            v = self._f32[f0 + 2 * self._up(r):f0 + 2 * self._up(r) + ne]
        elif key == "khw":
            return self._khw
        else:
            raise KeyError(key)
        self._views[key] = v
        return v

    def __iter__(self):
        return iter(("codes", "scale", "zero", "esum", "khw"))

    def __len__(self):
        return 5

    def esum_ref(self):
        """The E sums as (shared buffer, float offset, numel): no view made."""
        _, f0, _, r, ne = self._span
        return (self._f32, f0 + 2 * self._up(r), ne)


def esum_source(entry):
    """What bias_correction(error_sums=...) takes for one quantize state entry:
    a (buffer, float offset, numel) ref when the entry has one, else its E tensor."""
    ref = getattr(entry, "esum_ref", None)
    return ref() if ref is not None else entry["esum"]


def _quantize_targ_layer_sharded(graph, bit_weight, bits_bias, targ_type, *, granularity, symmetric, clip, state,
                                 group):
    """quantize_targ_layer's layer list sharded over the process group (see above)."""
    from .. import distributed as D
    print("Quantizing Layer parameters")
    if bits_bias == 32:
        print("Skipping bias quantization (32 bits)")
    assert targ_type is not None, "targ_type cannot be None!"
    if granularity not in ("tensor", "channel"):
        raise ValueError("granularity must be 'tensor' or 'channel'")
    per_channel = granularity == "channel"
    want = state is not None
    specs, srcs, keys = [], [], []
    for layer_idx in graph:
        layer = graph[layer_idx]
        if type(layer) not in targ_type:
            continue
        lp = layer._parameters
        w = lp["weight"].data
        _lib.require_device(w)
        specs.append(D.LayerSpec(shape=tuple(w.shape), bits=bit_weight, per_channel=per_channel,
                                 symmetric=symmetric, want_codes=want, want_esum=want,
                                 clip=tuple(clip) if clip is not None else None))
        srcs.append(w)
        keys.append(layer_idx)
        if lp.get("bias") is not None and bits_bias < 32:
            b = lp["bias"].data
            specs.append(D.LayerSpec(shape=tuple(b.shape), bits=bits_bias, per_channel=False, symmetric=False,
                                     want_codes=False))
            srcs.append(b)
            keys.append(None)
    if not specs:
        return graph
    sw = D.ShardedSweep(specs, sources=srcs, replicate=True, group=group)
    sw.run()
    sw.gather("all")
    outs = [sw.outputs(i) for i in range(len(specs))]
    torch._foreach_copy_(srcs, [o.dq for o in outs])        # back into the parameters, in place
    sw.destroy()
    if state is not None:
        for k, sp, o in zip(keys, specs, outs):
            if k is not None:
                state[k] = dict(codes=o.codes, scale=o.scale, zero=o.zero, esum=o.esum, khw=sp.khw)
    return graph


def find_prev_bn(bn_module, relu_attached, graph, bottoms, bot):
    """Walk upward from ``bot`` to the BatchNorms feeding a layer; tag each branch
    'one' / 'add' / 'add_<relu>' / 'cat'.  Returns (bn_list, relu_attach_list,
    connect_type_list, targ_without_bn) exactly as utils/layer_transform.py:308-353
    (branch ids are strings whose first character names the input branch)."""
    frontier = [(b, str(i)) for i, b in enumerate(bot)]
    branch_type = {str(i): "one" for i in range(len(bot))}
    targ_without_bn = {}
    bn_list, relu_attach_list, connect_type_list = [], [], []
    merged = False   # an add/cat node was crossed
    while frontier:
        key, bid = frontier.pop(0)
        node = graph[key]
        if type(node) == str:
            if "add" in key:
                branch_type[bid] = "add_{}".format(relu_attached[key]) if key in relu_attached else "add"
                merged = True
            elif "cat" in key:
                branch_type[bid] = "cat"
                merged = True
        elif not merged and type(node) in _CONV_TYPES + _LINEAR_TYPES:
            print("Warning: {} layer before first batch norm layer detected. "
                  "The calculated value range might be off.".format(type(node)))
            if bid[0] in targ_without_bn:
                assert False, "Multiple conv/linear layer without batch_norm is not supported."
            targ_without_bn[bid[0]] = ("conv" if type(node) in _CONV_TYPES else "linear", node)
        if key in bn_module:
            bn_list.append((bn_module[key], bid))
            relu_attach_list.append(relu_attached[key])
            connect_type_list.append(branch_type[bid])
        else:
            child = bid + bid[0]
            frontier.extend((b, child) for b in bottoms[key])
            branch_type[child] = branch_type[bid]
    return bn_list, relu_attach_list, connect_type_list, targ_without_bn


#: the tensor-op quantizers installed by switch_layers(quant_op=True) (the
#: reference keeps the same module-level global, utils/layer_transform.py:186)
module_tensor_op = None

# tensor ops whose inputs get QuantMeasures (utils/layer_transform.py:8-13), as
# this package's tracer names their graph nodes
_QUANT_OPS = ("add", "cat", "mean", "interpolate", "softmax")
_QUANT_OP_PREFIXES = ("add_", "torch.cat_", "torch.mean_", "F.interpolate_", "F.softmax_")


class CustomTensorOP(nn.Module):
    """QuantMeasures for the inputs of the graph's tensor-op nodes (add / cat /
    mean / interpolate / softmax), one per tensor input, in graph order
    (utils/layer_transform.py:199-236).  The reference finds a call's quantizers
    by cycling an index over the ops PyTransformer recorded; here they are keyed by
    the graph's op node, and ``replace_op`` matches calls to nodes in execution
    order."""

    def __init__(self, graph, bottoms, ignore_op=("pad",)):
        super().__init__()
        self.quants = nn.ModuleList()
        self.offsets: Dict[str, tuple] = {}
        self.names = []
        for key, node in graph.items():
            if type(node) != str or bottoms.get(key) is None:
                continue
            if any(ig in key for ig in ignore_op) or not key.startswith(_QUANT_OP_PREFIXES):
                continue
            n = len(bottoms[key])
            self.offsets[key] = (len(self.quants), n)
            self.names.append(key)
            for _ in range(n):
                self.quants.append(QuantMeasure(num_bits=8, momentum=0.1))
        self.idx_name_tensor_op = 0

    def get(self, key):
        o, n = self.offsets[key]
        return [self.quants[o + i] for i in range(n)]

    def next_name(self):
        """The op node the next intercepted call belongs to (execution order)."""
        key = self.names[self.idx_name_tensor_op]
        self.idx_name_tensor_op = (self.idx_name_tensor_op + 1) % len(self.names)
        return key


def switch_layers(model, transformer, data, module_dict, ignore_layer=[], ignore_op=["pad"], quant_op=True):
    """Swap layer types (module_dict {1: [(Conv2d, QuantConv2d), ...], 0: [(ReLU6, ReLU)]}),
    build the graph and, with ``quant_op``, install the tensor-op quantizers
    (utils/layer_transform.py:161-197)."""
    global module_tensor_op
    for key in module_dict:
        for source, target in module_dict[key]:
            transformer.register(source, target)
        model = transformer.trans_layers(model, update=(key == 1))
    g = transformer._build_graph(model, data, ignore_layer)
    if not quant_op:
        return model, transformer
    module_tensor_op = CustomTensorOP(g.getGraph(), g.getBottoms(), tuple(ignore_op))
    dev = next((p.device for p in model.parameters()), torch.device("cpu"))
    module_tensor_op.to(dev)
    model.add_module("custom_tensor_op", module_tensor_op)
    return model, transformer


# ---------------------------------------------------------------------------
# set_quant_minmax (utils/layer_transform.py:356-618): QuantMeasure ranges from
# the BN statistics feeding each quantized input.  The per-channel statistics
# (rectified-Gaussian moments, min/max of mean -/+ N*std, the case (d.) affine)
# are HIP kernels; the branch walk and the scalar combination stay Python, as in
# the reference.
# ---------------------------------------------------------------------------
_EPS = 1e-6
#: QuantMeasures the last set_quant_minmax set through case (d.) (a conv/linear
#: between the BN and the quantizer; its GEMV order is MKL's in the reference)
CASE_D = []


class _MinMaxBatch:
    """set_quant_minmax's (min, max) readbacks in one D2H copy.  The walk's control
    flow never depends on the values, so it runs twice: ``record`` enqueues every
    statistic kernel and writes each (min, max) into its own slot of one device
    buffer (the walk sees placeholders and its range writes are discarded); one
    copy brings all slots back; ``replay`` runs the walk again on the host only,
    handing out the values in call order."""

    def __init__(self, cap, device):
        self.device = device
        self.bufs = [torch.empty(2 * cap, dtype=torch.float32, device=device)]
        self.cap, self.n, self.vals, self.replay = cap, 0, None, False

    def minmax(self, a, w, n_sigma, w_is_var):
        k = self.n
        self.n += 1
        if self.replay:
            return self.vals[2 * k], self.vals[2 * k + 1]
        b, j = divmod(k, self.cap)
        if b == len(self.bufs):
            self.bufs.append(torch.empty(2 * self.cap, dtype=torch.float32, device=self.device))
        _lib.require_device(a, w)
        rc = _lib.load().dfq_act_minmax(_lib.ptr(a), _lib.ptr(w), a.numel(), int(w_is_var), _EPS, float(n_sigma),
                                        self.bufs[b].data_ptr() + 8 * j, _lib.stream_of(a))
        _lib.check(rc, "dfq_act_minmax")
        return 0.0, 0.0

    def fetch(self):
        vals = []
        for b in self.bufs:
            vals += b.tolist()
        self.vals, self.n, self.replay = vals, 0, True


_MM: Optional[_MinMaxBatch] = None


class _NoWrites:
    def fill(self, buf, value):
        pass

    def flush(self):
        pass


def _moments(weight, bias, kind, sqrt_w=False, into=None):
    """(mean, var) of one BN branch: kind 0 (no activation), 1 (ReLU), 2 (ReLU6);
    ``into``: (mean, var) accumulated in place (mean += m; var += v)."""
    if _MM is not None and _MM.replay:   # host-only pass: the statistics already ran
        return into if into is not None else (None, None)
    _lib.require_device(weight, bias)
    n = bias.numel()
    if into is None:
        mean = torch.empty(n, dtype=torch.float32, device=bias.device)
        var = torch.empty_like(mean)
        acc = 0
    else:
        mean, var = into
        acc = 1
    rc = _lib.load().dfq_act_moments(_lib.ptr(weight), _lib.ptr(bias), n, kind, int(sqrt_w), _EPS, acc,
                                     _lib.ptr(mean), _lib.ptr(var), _lib.stream_of(bias))
    _lib.check(rc, "dfq_act_moments")
    return mean, var


def _moments_inplace(mean, var, kind):
    """mean, var <- calculate_mean(_6)(sqrt(var + eps), mean), calculate_var(_6)(...)."""
    if _MM is not None and _MM.replay:
        return
    rc = _lib.load().dfq_act_moments(_lib.ptr(var), _lib.ptr(mean), mean.numel(), kind, 1, _EPS, 0,
                                     _lib.ptr(mean), _lib.ptr(var), _lib.stream_of(mean))
    _lib.check(rc, "dfq_act_moments")


def _minmax(a, w, n_sigma, w_is_var=False):
    """(float(min(a - N*w)), float(max(a + N*w))), w := sqrt(w + eps) if w_is_var."""
    if _MM is not None:
        return _MM.minmax(a, w, n_sigma, w_is_var)
    _lib.require_device(a, w)
    out = torch.empty(2, dtype=torch.float32, device=a.device)
    rc = _lib.load().dfq_act_minmax(_lib.ptr(a), _lib.ptr(w), a.numel(), int(w_is_var), _EPS, float(n_sigma),
                                    _lib.ptr(out), _lib.stream_of(a))
    _lib.check(rc, "dfq_act_minmax")
    lo, hi = out.tolist()
    return lo, hi


def _get_min_value(bias, weight, n):
    return _minmax(bias, weight, n)[0]


def _get_max_value(bias, weight, n):
    return _minmax(bias, weight, n)[1]


def _through_layer(vec, layer_type, layer):
    """Case (d.): a statistic vector pushed through a conv (weight summed over
    KH*KW, groups) or linear layer with its bias (utils/layer_transform.py:470-479)."""
    if _MM is not None and _MM.replay:
        layer.bias.detach()   # AttributeError on a bias-less layer, as in the recording pass
        return None
    w = layer.weight.detach().data
    b = layer.bias.detach().data   # AttributeError on a bias-less layer, as the reference
    o, i2 = w.shape[0], w.shape[1]
    khw = w.numel() // (o * i2)
    groups = getattr(layer, "groups", 1) if layer_type == "conv" else 1
    out = torch.empty(o, dtype=torch.float32, device=w.device)
    _lib.require_device(vec, w, b)
    rc = _lib.load().dfq_act_affine(_lib.ptr(vec), _lib.ptr(w.contiguous()), _lib.ptr(b), o, i2, khw, groups,
                                    _lib.ptr(out), _lib.stream_of(w))
    _lib.check(rc, "dfq_act_affine")
    return out


class _RangeWrites:
    """The walk's ``running_min/max.fill_(v)`` calls, kept on the host and written
    at the end in one H2D copy plus one ``dfq_bc_chain`` COPY launch per 64
    buffers (instead of a torch fill kernel per buffer).  Last write wins, as with
    sequential fills; ``flush`` runs in a ``finally``, so the writes made before an
    error take effect, as in the reference."""

    def __init__(self):
        self.dst = {}

    def fill(self, buf, value):
        if buf.numel() != 1 or buf.dtype != torch.float32 or not buf.is_cuda:
            buf.fill_(value)   # not a QuantMeasure scalar: the plain op
            return
        self.dst[buf.data_ptr()] = (buf, float(value))

    def flush(self):
        if not self.dst:
            return
        bufs = [b for b, _ in self.dst.values()]
        dev = bufs[0].device
        src = torch.tensor([v for _, v in self.dst.values()], dtype=torch.float32).to(dev)
        ops = (_lib.BcOp * len(bufs))()
        for k, b in enumerate(bufs):
            ops[k].kind, ops[k].a, ops[k].out, ops[k].n = _lib.DFQ_BC_OP_COPY, src.data_ptr() + 4 * k, b.data_ptr(), 1
        failed = C.c_int32(-1)
        rc = _lib.load().dfq_bc_chain(ops, len(bufs), C.byref(failed), _lib.stream_of(src))
        _lib.check(rc, f"dfq_bc_chain (range write {failed.value})", RuntimeError)
        src.record_stream(torch.cuda.current_stream(dev))
        self.dst.clear()


def set_quant_minmax(graph, bottoms, is_detection=False, bn_type=torch.nn.BatchNorm2d, N=6, verbose=True):
    """Set every QuantMeasure's running_min / running_max from the statistics of
    the BatchNorms feeding it (utils/layer_transform.py:356-618): 1-to-1, 1-to-many
    (add: Gaussian moment sums; cat: min/max), many-to-many, and layers without a
    BN in between (case d.)."""
    if verbose:
        print("SET QUANT MIN MAX")
    global _MM
    batch = (_moments is _MOMENTS_DEV and _moments_inplace is _MOMENTS_INPLACE_DEV and _minmax is _MINMAX_DEV
             and _through_layer is _THROUGH_DEV and _MM is None)
    dev = next((m.fake_bias.device for m in graph.values() if isinstance(m, bn_type) and
                getattr(m, "fake_bias", None) is not None and m.fake_bias.is_cuda), None)
    if not batch or dev is None:   # injected statistics (oracle-backed tests) or nothing on the GPU
        CASE_D.clear()
        _set_quant_minmax_walk(graph, bottoms, is_detection, bn_type, N, _RangeWrites())
        return
    _MM = _MinMaxBatch(4 * len(graph) + 16, dev)
    try:
        CASE_D.clear()
        err = None
        try:
            _set_quant_minmax_walk(graph, bottoms, is_detection, bn_type, N, _NoWrites())   # record
        except Exception as e:   # the reference's own errors: replay up to them, then raise
            err = e
        _MM.fetch()
        CASE_D.clear()
        try:   # replay: the fills made before an error take effect, as in the reference
            _set_quant_minmax_walk(graph, bottoms, is_detection, bn_type, N, _RangeWrites())
        except Exception:
            if err is None:
                raise
        if err is not None:
            raise err
    finally:
        _MM = None


def _set_quant_minmax_walk(graph, bottoms, is_detection, bn_type, N, writes):
    """The walk of set_quant_minmax (utils/layer_transform.py:356-618); ``writes``
    receives the running_min / running_max fills."""

    def get_quant_module(layer, key):
        if type(layer) == str:
            if module_tensor_op is not None and key in module_tensor_op.offsets:
                return module_tensor_op.get(key)
            return None
        if hasattr(layer, "quant"):
            return [getattr(layer, "quant")]
        return None

    def kind_of(use_relu):
        return 1 if use_relu == "relu" else 2 if use_relu == "relu6" else 0

    bn_module, relu_attached = {}, {}
    try:
        for idx_layer in graph:
            bot = bottoms[idx_layer]
            if bot is None:
                continue
            node = graph[idx_layer]
            if type(node) == bn_type:
                bn_module[idx_layer] = node
                relu_attached[idx_layer] = "none"
                continue
            if type(node) == torch.nn.ReLU:
                relu_attached[bot[0]] = "relu"
            elif type(node) == torch.nn.ReLU6:
                relu_attached[bot[0]] = "relu6"
            quant_module = get_quant_module(node, idx_layer)
            if len(bot) == 1 and bot[0] == "Data":
                if is_detection:
                    writes.fill(quant_module[0].running_max, 1)
                    writes.fill(quant_module[0].running_min, -1)
                else:   # (1 - mean) / std and (0 - mean) / std of the data preprocessing
                    writes.fill(quant_module[0].running_max, 2.64)
                    writes.fill(quant_module[0].running_min, -2.11790393)
            elif quant_module is not None:
                bn_list, relu_attach_list, connect_type_list, targ_without_bn = find_prev_bn(
                    bn_module, relu_attached, graph, bottoms, bot[:])
                if len(quant_module) == len(bn_list):   # 1 to 1
                    for idx in range(len(bn_list)):
                        bias = getattr(bn_list[idx][0], "fake_bias").view(-1)
                        weight = getattr(bn_list[idx][0], "fake_weight").view(-1)
                        if bn_list[idx][1][0] in targ_without_bn:   # case (d.)
                            CASE_D.append(quant_module[idx])
                            layer_type, obj_layer = targ_without_bn[bn_list[idx][1][0]]
                            bias = _through_layer(bias, layer_type, obj_layer)
                            weight = _through_layer(weight, layer_type, obj_layer)
                            value_max = _get_max_value(bias, weight, N)
                            value_min = _get_min_value(bias, weight, N)
                        else:
                            lo, hi = _minmax(bias, weight, N)
                            value_min = max(0., lo) if "relu" in relu_attach_list[idx] else lo
                            value_max = min(6., hi) if "relu6" in relu_attach_list[idx] else hi
                        writes.fill(quant_module[idx].running_max, value_max)
                        writes.fill(quant_module[idx].running_min, value_min)
                else:   # 1 to many or many to many
                    bn_branch = {}
                    for idx, tmp in enumerate(bn_list):
                        _, bid = tmp
                        bn_branch.setdefault(bid[0], []).append((tmp, relu_attach_list[idx], connect_type_list[idx]))
                    bn_res = {}
                    for key in bn_branch:
                        tmp_list = sorted(bn_branch[key], key=lambda x: len(x[0][1]), reverse=True)
                        node_cur, use_relu, connect_type = tmp_list[0]
                        layer_cur, bid = node_cur
                        depth = len(bid)
                        tmp_list.pop(0)
                        bias = layer_cur.fake_bias.detach()   # read only: no clone needed
                        weight = layer_cur.fake_weight.detach()
                        mean = var = None
                        value_min = value_max = None
                        if "add" in connect_type:
                            mean, var = _moments(weight, bias, kind_of(use_relu))
                        else:
                            lo, hi = _minmax(bias, weight, N)
                            value_min = max(0., lo) if "relu" in use_relu else lo
                            value_max = min(6., hi) if "relu6" in use_relu else hi
                        while len(tmp_list) > 0:
                            idx_bound = 0
                            while idx_bound < len(tmp_list) and len(tmp_list[idx_bound][0][1]) == depth:
                                idx_bound += 1
                            if idx_bound == 0 and len(tmp_list) > 0:   # cut depth
                                depth = len(tmp_list[idx_bound][0][1])
                            else:
                                for idx in range(idx_bound):
                                    node_tmp, use_relu_tmp, connect_type = tmp_list[idx]
                                    bias = node_tmp[0].fake_bias.detach()
                                    weight = node_tmp[0].fake_weight.detach()
                                    if "add" in connect_type:
                                        _moments(weight, bias, kind_of(use_relu_tmp), into=(mean, var))
                                        if "relu6" in connect_type:
                                            _moments_inplace(mean, var, 2)
                                        elif "relu" in connect_type:
                                            _moments_inplace(mean, var, 1)
                                    else:
                                        lo, hi = _minmax(bias, weight, N)
                                        if "cat" == connect_type:
                                            value_min = min(value_min, max(0., lo) if "relu" in use_relu_tmp else lo)
                                            value_max = max(value_max, min(6., hi) if "relu6" in use_relu_tmp else hi)
                                        else:
                                            value_min += max(0., lo) if use_relu_tmp else lo
                                            value_max += hi
                                tmp_list = tmp_list[idx_bound:]
                                if "one" == connect_type:
                                    value_min /= (idx_bound + 1)
                                    value_max /= (idx_bound + 1)
                        if "add" in connect_type:
                            bn_res[key] = (connect_type, mean, var)
                        else:
                            bn_res[key] = (connect_type, value_min, value_max)

                    if len(quant_module) == 1 and len(quant_module) < len(bn_list):   # 1 to many
                        assert len(list(bn_res.keys())) == 1, "Error occurs when setting min/max, should be 1 to many"
                        first = list(bn_res.values())[0]
                        if "add" in first[0]:
                            _, mean, var = first
                            value_min, value_max = _minmax(mean, var, N, w_is_var=True)
                        else:
                            _, value_min, value_max = first
                        writes.fill(quant_module[0].running_max, value_max)
                        writes.fill(quant_module[0].running_min, value_min)
                    elif len(quant_module) < len(bn_list):   # many to many
                        assert len(bn_res) == len(quant_module), "LENGTH NOT EQUAL {} vs {}".format(
                            len(bn_res), len(quant_module))
                        for idx in range(len(bn_res)):
                            entry = bn_res[str(idx)]
                            if "add" in entry[0]:
                                _, mean, var = entry
                                value_min, value_max = _minmax(mean, var, N, w_is_var=True)
                            else:
                                _, value_min, value_max = entry
                            writes.fill(quant_module[idx].running_max, value_max)
                            writes.fill(quant_module[idx].running_min, value_min)
                    else:
                        assert False, "Unknown error occured while setting min/max"
    finally:
        writes.flush()


_MOMENTS_DEV, _MOMENTS_INPLACE_DEV, _MINMAX_DEV, _THROUGH_DEV = _moments, _moments_inplace, _minmax, _through_layer

_RAW_OPS = {}
_IN_QUANT = False   # re-entrancy guard: ops inside a quantizer are never intercepted


def _quantized_call(func, kind, args, kwargs):
    """Apply the op node's QuantMeasures to the call's tensor inputs (the reference's
    ___add__ / torch_cat / torch_mean / F_interpolate / F_softmax,
    utils/layer_transform.py:18-124), then run the original op."""
    global _IN_QUANT
    key = module_tensor_op.next_name()
    qs = module_tensor_op.get(key)
    _IN_QUANT = True
    try:
        if kind == "add":
            args = (qs[0](args[0]), qs[1](args[1])) + tuple(args[2:])
        elif kind == "cat":
            seq = args[0] if args else kwargs.pop("tensors")
            args = (type(seq)(q(t) for q, t in zip(qs, seq)),) + tuple(args[1:])
        else:
            args = (qs[0](args[0]),) + tuple(args[1:])
    finally:
        _IN_QUANT = False
    return func(*args, **kwargs)


def _wrap(raw, kind):
    """The patched op: intercepted only when the graph's next op node is this kind
    (execution order, as the reference's name check does without inspect.stack)."""
    def op(*args, **kwargs):
        m = module_tensor_op
        if not _IN_QUANT and m is not None and m.names and kind in m.names[m.idx_name_tensor_op]:
            return _quantized_call(raw, kind, args, kwargs)
        return raw(*args, **kwargs)
    op.__name__ = getattr(raw, "__name__", kind)
    op.__wrapped__ = raw
    return op


# (owner, attribute, kind): Tensor.__add__ / __iadd__ / add, torch.add, torch.cat,
# torch.mean, F.interpolate, F.softmax -- the reference's tensor_magic_op_supported,
# torch_op_supported and func_op_sopprted lists (utils/layer_transform.py:128-144)
_PATCHES = [(torch.Tensor, "__add__", "add"), (torch.Tensor, "__iadd__", "add"), (torch.Tensor, "add", "add"),
            (torch, "add", "add"), (torch, "cat", "cat"), (torch, "mean", "mean"),
            (torch.nn.functional, "interpolate", "interpolate"), (torch.nn.functional, "softmax", "softmax")]


def replace_op():
    """Quantize the inputs of tensor ops during inference
    (utils/layer_transform.py:128-144): patch the eight ops above with wrappers that
    match each call to the next op node of the graph (no call-stack inspection);
    every other op runs untouched."""
    if _RAW_OPS:
        return
    for owner, name, kind in _PATCHES:
        raw = getattr(owner, name)
        _RAW_OPS[(owner, name)] = raw
        setattr(owner, name, _wrap(raw, kind))


def restore_op():
    """Undo replace_op (utils/layer_transform.py:147-158)."""
    for (owner, name), raw in list(_RAW_OPS.items()):
        setattr(owner, name, raw)
    _RAW_OPS.clear()


__all__ = ["merge_batchnorm", "quantize_targ_layer", "find_prev_bn", "switch_layers", "replace_op", "restore_op",
           "set_quant_minmax", "CustomTensorOP", "TorchTransformer", "QuantMeasure"]
