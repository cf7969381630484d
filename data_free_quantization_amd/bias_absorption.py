"""Drop-in for the reference's ``bias_absorption.py`` (bias_absorption.py:9-121):
high-bias absorption across equalized pairs with a ReLU in between.

Per relation: c = clamp(beta - N*gamma, 0) from the BN's fake stats;
b2 += sum_i (sum_k W2[o,i,k]) * c[i]  (HIP GEMV, one wave per output row);
b1 -= c; beta -= c (HIP, per channel).
"""
from __future__ import annotations

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
    print("Start bias absorption")
    if visualize:
        warnings.warn("bias-absorption histograms are visualization, not part of the weight path; skipped")
    with torch.no_grad():
        for rel in relations:
            first, second, bn_idx = rel.get_idxs()
            if not _has_relu_between(second, first, graph, bottoms):
                continue
            l1, l2, bn = graph[first], graph[second], graph[bn_idx]
            for layer in (l1, l2):
                if layer.bias is None:
                    layer.bias = nn.Parameter(torch.zeros(layer.weight.size(0), dtype=torch.float32,
                                                          device=layer.weight.device), requires_grad=False)
            w2 = l2.weight.data
            _lib.require_device(w2, l1.bias, l2.bias, bn.fake_weight, bn.fake_bias)
            c1 = l1.weight.size(0)
            o2, i2 = w2.shape[0], w2.shape[1]
            rc = _lib.load().dfq_bias_absorb(
                _lib.ptr(w2), _lib.ptr(l1.bias.data), _lib.ptr(l2.bias.data), _lib.ptr(bn.fake_weight),
                _lib.ptr(bn.fake_bias), c1, o2, i2, w2.numel() // (o2 * i2), float(N), _lib.stream_of(w2))
            _lib.check(rc, "dfq_bias_absorb")
    print("Bias absorption done")
