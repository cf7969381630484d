"""Drop-in for the reference's ``clip_weight.py`` (clip_weight.py:4-33): clamp
every target layer's weight to [lo, hi] in place (HIP ``dfq_clamp_batch``: one
call, 64 weights per launch).  The same
clamp is also available fused into the quantize sweep
(``quantize_targ_layer(..., clip=(lo, hi))``)."""
from __future__ import annotations

import ctypes as C

import torch.nn as nn

from . import _lib


def clip_weight(graph, range_clip=None, targ_type=[nn.Conv2d, nn.Linear]):
    if range_clip is None:
        range_clip = [-15, 15]
    assert isinstance(range_clip, (list, tuple)) and len(range_clip) == 2, \
        "range_clip should be a list or tuple of two elements"
    lo, hi = float(range_clip[0]), float(range_clip[1])
    _lib.weights_changed()
    ws = []
    for idx, layer in graph.items():
        if isinstance(layer, tuple(targ_type)):
            if hasattr(layer, "weight"):
                w = layer.weight.data
                _lib.require_device(w)
                ws.append(w)
            else:
                print(f"Warning: Layer at index {idx} does not have 'weight' attribute")
        else:
            print(f"Warning: Layer at index {idx} is not in the target type list for clipping")
    if ws:   # every clamp in one call (64 weights per launch)
        ptrs = (C.c_void_p * len(ws))(*[w.data_ptr() for w in ws])
        ns = (C.c_int64 * len(ws))(*[w.numel() for w in ws])
        _lib.check(_lib.load().dfq_clamp_batch(ptrs, ns, len(ws), lo, hi, _lib.stream_of(ws[0])), "dfq_clamp_batch")
