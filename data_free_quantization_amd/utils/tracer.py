"""Graph capture for the DFQ path (replaces the empty PyTransformer submodule).

The reference builds its layer graph with PyTransformer's
``TorchTransformer._build_graph`` and reads it back through
``transformer.log.getGraph()/getBottoms()`` (main_dfq.py:149-175,
utils/layer_transform.py:161-197).  The submodule is empty in the reference tree
(.gitmodules:1-4), so this module re-creates the data model the DFQ functions
consume:

* ``graph``: OrderedDict key -> nn.Module (leaf layer call) or str (op node,
  value == key); ``"Data"`` is the root.
* ``bottoms``: key -> list of input keys; ``bottoms["Data"] = None``.
* op keys carry the op name the reference greps for: ``add_<pos>``,
  ``torch.cat_<pos>``, ``torch.mean_<pos>``, ``F.pad_<pos>``,
  ``F.interpolate_<pos>`` (utils/layer_transform.py:325-334, utils/relation.py:54).

Keys come in two flavours.  ``key_mode="opaque"`` (default, like PyTransformer)
names a module call by its qualified module path; ``key_mode="positional"`` uses
the node's position (int), which makes ``bias_correction``'s
``enumerate(graph.values())`` index equal the key so its arithmetic runs
(bias_correction.py:185-190).

Tracing uses torch.fx: leaf modules become nodes; view/size/reshape/flatten/
getitem/contiguous are transparent.
"""
from __future__ import annotations

import operator
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch
import torch.fx as fx
import torch.nn as nn
import torch.nn.functional as F

_TRANSPARENT_METHODS = {"view", "size", "reshape", "flatten", "contiguous", "dim", "float", "detach", "clone"}
_TRANSPARENT_FUNCS = {operator.getitem, getattr, torch.flatten, torch.reshape}
_OPS = {
    operator.add: "add", operator.iadd: "add", torch.add: "add",
    torch.cat: "torch.cat", torch.mean: "torch.mean",
    F.pad: "F.pad", F.interpolate: "F.interpolate", F.softmax: "F.softmax",
}
_METHOD_OPS = {"add": "add", "add_": "add", "__add__": "add", "__iadd__": "add", "mean": "torch.mean"}


class _LeafTracer(fx.Tracer):
    """Every module without children is a leaf, plus conv/linear subclasses that
    carry a QuantMeasure child (QuantConv2d / QuantLinear, utils/quantize.py)."""

    def is_leaf_module(self, m: nn.Module, qualname: str) -> bool:
        if isinstance(m, (nn.Conv2d, nn.Linear, nn.BatchNorm2d)):
            return True
        return len(list(m.children())) == 0


def _tensor_args(args) -> List[fx.Node]:
    out = []
    for a in args:
        if isinstance(a, fx.Node):
            out.append(a)
        elif isinstance(a, (list, tuple)):
            out.extend(_tensor_args(a))
    return out


class TorchGraph:
    """Result of a trace; mirrors ``transformer.log`` (getGraph / getBottoms)."""

    def __init__(self, graph: "OrderedDict", bottoms: Dict, record_ops: List[Tuple[str, str]]):
        self._graph = graph
        self._bottoms = bottoms
        self._ops = record_ops

    def getGraph(self):
        return self._graph

    def getBottoms(self):
        return self._bottoms

    def getRecordTensorOP(self):
        return list(self._ops)


def build_graph(model: nn.Module, key_mode: str = "opaque") -> TorchGraph:
    """Trace ``model`` and return its DFQ graph/bottoms (see module doc)."""
    if key_mode not in ("opaque", "positional"):
        raise ValueError("key_mode must be 'opaque' or 'positional'")
    tracer = _LeafTracer()
    fxg = tracer.trace(model)
    modules = dict(model.named_modules())

    graph: "OrderedDict" = OrderedDict()
    bottoms: Dict = OrderedDict()
    producer: Dict[fx.Node, Optional[object]] = {}   # fx node -> graph key (None: not a tensor)
    ops: List[Tuple[str, str]] = []
    used_names: Dict[str, int] = {}

    def add(key, value, bots):
        graph[key] = value
        bottoms[key] = bots

    def key_for(pos: int, name: str):
        if key_mode == "positional":
            return pos
        k = name
        if k in used_names:
            used_names[k] += 1
            k = f"{name}#{used_names[name]}"
        else:
            used_names[k] = 0
        return k

    def bots_of(args) -> List:
        res = []
        for a in _tensor_args(args):
            k = producer.get(a)
            if k is not None:
                res.append(k)
        return res

    for node in fxg.nodes:
        pos = len(graph)
        if node.op == "placeholder":
            if "Data" not in graph:
                add("Data", "Data", None)
            producer[node] = "Data"
        elif node.op == "call_module":
            mod = modules[node.target]
            key = key_for(pos, node.target)
            b = bots_of(node.args)
            add(key, mod, b[:1] if b else ["Data"])
            producer[node] = key
        elif node.op in ("call_function", "call_method"):
            tgt = node.target
            opname = _OPS.get(tgt) if node.op == "call_function" else _METHOD_OPS.get(tgt)
            if opname is not None:
                key = f"{opname}_{pos}"
                add(key, key, bots_of(node.args))
                producer[node] = key
                ops.append((key, f"{opname}_{len(bots_of(node.args))}"))
            elif (node.op == "call_method" and tgt in _TRANSPARENT_METHODS) or \
                    (node.op == "call_function" and tgt in _TRANSPARENT_FUNCS):
                src = _tensor_args(node.args[:1])
                producer[node] = producer.get(src[0]) if src else None
                if tgt in ("size", "dim") or (tgt is operator.getitem and producer[node] is None):
                    producer[node] = None
            else:
                # any other tensor op becomes an opaque op node so walks stop there
                b = bots_of(node.args)
                if b:
                    name = getattr(tgt, "__name__", str(tgt))
                    key = f"{name}_{pos}"
                    add(key, key, b)
                    producer[node] = key
                else:
                    producer[node] = None
        elif node.op == "get_attr":
            producer[node] = None
    return TorchGraph(graph, bottoms, ops)


class TorchTransformer:
    """Minimal stand-in for PyTransformer's TorchTransformer as used by
    main_dfq.py:149-175 / utils/layer_transform.py:161-197: register layer swaps,
    apply them, build the graph."""

    def __init__(self, key_mode: str = "opaque"):
        self._swaps: List[Tuple[type, type]] = []
        self.key_mode = key_mode
        self.log: Optional[TorchGraph] = None

    def register(self, source: type, target: type):
        self._swaps.append((source, target))

    def trans_layers(self, model: nn.Module, update: bool = True) -> nn.Module:
        swaps, self._swaps = self._swaps, []
        for name, child in list(model.named_children()):
            replaced = False
            for src, dst in swaps:
                if type(child) is src:
                    setattr(model, name, _convert(child, dst, update))
                    replaced = True
                    break
            if not replaced:
                self._swaps = swaps
                self.trans_layers(child, update)
        self._swaps = swaps
        return model

    def _build_graph(self, model: nn.Module, data=None, ignore_layer=()) -> TorchGraph:
        self.log = build_graph(model, self.key_mode)
        return self.log


def _convert(child: nn.Module, dst: type, update: bool) -> nn.Module:
    """Swap a layer for ``dst`` (ReLU6 -> ReLU, Conv2d -> QuantConv2d, Linear ->
    QuantLinear), carrying weights/bias over when ``update``."""
    if isinstance(child, nn.Conv2d) and issubclass(dst, nn.Conv2d):
        new = dst(child.in_channels, child.out_channels, child.kernel_size, stride=child.stride,
                  padding=child.padding, dilation=child.dilation, groups=child.groups,
                  bias=child.bias is not None)
    elif isinstance(child, nn.Linear) and issubclass(dst, nn.Linear):
        new = dst(child.in_features, child.out_features, bias=child.bias is not None)
    else:
        try:
            new = dst(inplace=getattr(child, "inplace", False))
        except TypeError:
            new = dst()
        return new
    if update:
        with torch.no_grad():
            new.weight.copy_(child.weight)
            if child.bias is not None:
                new.bias.copy_(child.bias)
    new = new.to(child.weight.device)
    new.train(child.training)
    return new
