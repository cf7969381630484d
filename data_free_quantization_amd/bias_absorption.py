"""Drop-in for the reference's ``bias_absorption.py`` (bias_absorption.py:9-121):
high-bias absorption across equalized pairs with a ReLU in between.

Per relation: c = clamp(beta - N*gamma, 0) from the BN's fake stats;
b2 += sum_i (sum_k W2[o,i,k]) * c[i]  (HIP GEMV, one wave per output row);
b1 -= c; beta -= c (HIP, per channel).
"""
from __future__ import annotations

import ctypes as C
import warnings

import torch
import torch.nn as nn

from . import _lib


def _has_relu_between(layer_second, layer_first, graph, bottoms):
    """bias_absorption.py:10-18: any ReLU on the single-input path second -> first."""
    idx = layer_second
    while idx != layer_first:
        if isinstance(graph[bottoms[idx][0]], torch.nn.ReLU):
            return True
        idx = bottoms[idx][0]
    return False


def bias_absorption(graph, relations, bottoms, N=3, visualize=False):
    """Every absorbing relation in ONE dfq_bias_absorb_batch call (two launches;
    the same per-element fp32 order as one call per relation)."""
    print("Start bias absorption")
    if visualize:
        warnings.warn("bias-absorption histograms are visualization, not part of the weight path; skipped")
    with torch.no_grad():
        todo = []
        for rel in relations:
            first, second, bn_idx = rel.get_idxs()
            if not _has_relu_between(second, first, graph, bottoms):
                continue
            l1, l2, bn = graph[first], graph[second], graph[bn_idx]
            for layer in (l1, l2):
                if layer.bias is None:
                    layer.bias = nn.Parameter(torch.zeros(layer.weight.size(0), dtype=torch.float32,
                                                          device=layer.weight.device), requires_grad=False)
            todo.append((l1, l2, bn))
        if not todo:
            print("Bias absorption done")
            return
        descs = (_lib.AbsorbDesc * len(todo))()
        for j, (l1, l2, bn) in enumerate(todo):
            w2 = l2.weight.data
            _lib.require_device(w2, l1.bias, l2.bias, bn.fake_weight, bn.fake_bias)
            d = descs[j]
            d.w2, d.b1, d.b2 = w2.data_ptr(), l1.bias.data.data_ptr(), l2.bias.data.data_ptr()
            d.bn_w, d.bn_b = bn.fake_weight.data_ptr(), bn.fake_bias.data_ptr()
            d.c1, d.o2, d.i2 = l1.weight.size(0), w2.shape[0], w2.shape[1]
            d.khw2 = w2.numel() // (w2.shape[0] * w2.shape[1])
        L = _lib.load()
        stream = _lib.stream_of(todo[0][1].weight)
        nb = int(L.dfq_bias_absorb_ws_bytes(descs, len(todo)))
        if nb >= 0:
            ws = torch.empty(max(nb, 256), dtype=torch.uint8, device=todo[0][1].weight.device)   # stream-ordered
            failed = C.c_int32(-1)
            rc = L.dfq_bias_absorb_batch(descs, len(todo), float(N), ws.data_ptr(), ws.numel(), C.byref(failed),
                                         stream)
            if rc != _lib.DFQ_ERR_UNSUPPORTED:
                _lib.check(rc, f"dfq_bias_absorb_batch (relation {failed.value})")
                print("Bias absorption done")
                return
        for d in descs:   # invalid shapes (the per-relation call raises the reference's error) or a shared BN
            _lib.check(L.dfq_bias_absorb(d.w2, d.b1, d.b2, d.bn_w, d.bn_b, d.c1, d.o2, d.i2, d.khw2, float(N), stream),
                       "dfq_bias_absorb")
    print("Bias absorption done")
