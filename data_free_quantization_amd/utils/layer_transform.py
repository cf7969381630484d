"""Drop-in for the DFQ-path functions of the reference's ``utils/layer_transform.py``:

* ``merge_batchnorm``     (utils/layer_transform.py:240-285) -> HIP ``dfq_bn_fold``
* ``quantize_targ_layer`` (utils/layer_transform.py:288-305) -> one grouped HIP sweep
* ``find_prev_bn``        (utils/layer_transform.py:308-353) host graph walk
* ``switch_layers``       (utils/layer_transform.py:161-197) with this package's tracer

Graph/bottoms follow SURVEY.md 8b.  Target tensors must be on a ROCm device.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import torch
import torch.nn as nn

from .. import _lib
from ..sweep import SweepItem, SweepPlan, khw_of
from .quantize import (QConv2d, QLinear, QuantConv2d, QuantLinear, QuantMeasure, QuantNConv2d,
                       QuantNLinear)
from .tracer import TorchTransformer

_CONV_TYPES = (nn.Conv2d, QConv2d, QuantConv2d, QuantNConv2d)
_LINEAR_TYPES = (nn.Linear, QLinear, QuantLinear, QuantNLinear)


def merge_batchnorm(model, graph, bottoms, targ_type=[QConv2d]):
    """Fold each BatchNorm2d into the target layer feeding it, keep |gamma| and beta
    as ``fake_weight``/``fake_bias`` buffers, and turn the BN into an identity."""
    with torch.no_grad():
        for layer_idx in graph:
            if bottoms[layer_idx] is None:
                continue
            for bot_idx in bottoms[layer_idx]:
                bn, layer = graph[layer_idx], graph[bot_idx]
                if type(bn) != nn.BatchNorm2d or type(layer) not in targ_type:
                    continue
                w = layer.weight
                _lib.require_device(w, bn.weight, bn.bias, bn.running_mean, bn.running_var)
                if layer.bias is None:   # :262-263
                    layer.bias = nn.Parameter(torch.zeros(w.size(0), dtype=torch.float32, device=w.device),
                                              requires_grad=False)
                fake_w = torch.empty_like(bn.weight)
                fake_b = torch.empty_like(bn.bias)
                rows = w.size(0)
                rc = _lib.load().dfq_bn_fold(
                    _lib.ptr(w), _lib.ptr(layer.bias), _lib.ptr(bn.weight), _lib.ptr(bn.bias),
                    _lib.ptr(bn.running_mean), _lib.ptr(bn.running_var), _lib.ptr(fake_w), _lib.ptr(fake_b),
                    float(bn.eps), rows, w.numel() // rows, _lib.stream_of(w))
                _lib.check(rc, "dfq_bn_fold")
                bn.register_buffer("fake_weight", fake_w)
                bn.register_buffer("fake_bias", fake_b)
                bn.eps = 0
                break
    return model


def quantize_targ_layer(graph, bit_weight=8, bits_bias=16, targ_type=None, *, granularity="tensor",
                        symmetric=False, clip=None, state: Optional[Dict] = None):
    """Fake-quantize every target layer's weight (and bias when bits_bias < 32) in
    place, all layers in one grouped launch.

    Reference semantics by default (per-tensor asymmetric with float(min)/float(max),
    utils/layer_transform.py:298-303).  Extensions: ``granularity="channel"``,
    ``symmetric=True``, ``clip=(lo, hi)`` fused (the clip_weight clamp), and
    ``state`` -- a dict filled with per-layer codes/scale/zero and the BC error
    sums E[o,i] of this quantization.
    """
    print("Quantizing Layer parameters")
    if bits_bias == 32:
        print("Skipping bias quantization (32 bits)")
    assert targ_type is not None, "targ_type cannot be None!"
    per_channel = granularity == "channel"
    if granularity not in ("tensor", "channel"):
        raise ValueError("granularity must be 'tensor' or 'channel'")
    items = []
    keys = []
    for layer_idx in graph:
        layer = graph[layer_idx]
        if type(layer) not in targ_type:
            continue
        w = layer.weight.data
        rows = w.size(0) if per_channel else 1
        npar = rows
        khw = khw_of(w)
        want = state is not None
        it = SweepItem(src=w, dst=w, bits=bit_weight, per_channel=per_channel, symmetric=symmetric, clip=clip,
                       khw=khw, rows=rows)
        if want:
            cdt = (torch.int8 if symmetric else torch.uint8) if bit_weight <= 8 else torch.int16
            it.codes = torch.empty(w.shape, dtype=cdt, device=w.device)
            it.scale = torch.empty(npar, dtype=torch.float32, device=w.device)
            it.zero = torch.empty(npar, dtype=torch.float32, device=w.device)
            it.esum = torch.empty(w.numel() // khw, dtype=torch.float32, device=w.device)
        items.append(it)
        keys.append(layer_idx)
        if layer.bias is not None and bits_bias < 32:
            b = layer.bias.data
            items.append(SweepItem(src=b, dst=b, bits=bits_bias, per_channel=False, symmetric=False, rows=1))
            keys.append(None)
    if not items:
        return graph
    plan = SweepPlan(items)
    plan.execute()
    plan.destroy()   # synchronises before releasing the task tables
    if state is not None:
        for k, it in zip(keys, items):
            if k is not None:
                state[k] = dict(codes=it.codes, scale=it.scale, zero=it.zero, esum=it.esum, khw=it.khw)
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


def switch_layers(model, transformer, data, module_dict, ignore_layer=[], ignore_op=["pad"], quant_op=True):
    """Swap layer types (module_dict {1: [(Conv2d, QuantConv2d), ...], 0: [(ReLU6, ReLU)]})
    and build the graph (utils/layer_transform.py:161-197).  Activation-op
    interception (CustomTensorOP) is not on the weight path and is not installed."""
    for key in module_dict:
        for source, target in module_dict[key]:
            transformer.register(source, target)
        model = transformer.trans_layers(model, update=(key == 1))
    transformer._build_graph(model, data, ignore_layer)
    return model, transformer


def replace_op():
    """Activation-op interception (utils/layer_transform.py:128-144) belongs to the
    activation/inference path, out of scope for the weight path."""
    return None


def restore_op():
    return None


__all__ = ["merge_batchnorm", "quantize_targ_layer", "find_prev_bn", "switch_layers", "replace_op", "restore_op",
           "TorchTransformer", "QuantMeasure"]
