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


def _state(m, name):
    """A module's registered buffer without Module.__getattr__ (else getattr)."""
    b = getattr(m, "_buffers", None)
    if b is not None and name in b:
        return b[name]
    return getattr(m, name)


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
    _lib.weights_changed()
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
                lp = layer._parameters   # no Module.__getattr__ per access
                if lp.get("bias") is None:
                    w = lp["weight"]
                    layer.bias = nn.Parameter(torch.zeros(w.size(0), dtype=torch.float32, device=w.device),
                                              requires_grad=False)
            todo.append((l1, l2, bn))
        if not todo:
            print("Bias absorption done")
            return
        descs = (_lib.AbsorbDesc * len(todo))()
        for j, (l1, l2, bn) in enumerate(todo):
            p1, p2 = l1._parameters, l2._parameters
            w2, b1, b2 = p2["weight"], p1["bias"], p2["bias"]
            fw, fb = _state(bn, "fake_weight"), _state(bn, "fake_bias")
            _lib.require_device(w2, b1, b2, fw, fb)
            s2 = w2.shape
            d = descs[j]
            d.w2, d.b1, d.b2 = w2.data_ptr(), b1.data_ptr(), b2.data_ptr()
            d.bn_w, d.bn_b = fw.data_ptr(), fb.data_ptr()
            d.c1, d.o2, d.i2 = p1["weight"].size(0), s2[0], s2[1]
            d.khw2 = w2.numel() // (s2[0] * s2[1])
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
