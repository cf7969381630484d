"""Drop-in for the reference's ``clip_weight.py`` (clip_weight.py:4-33): clamp
every target layer's weight to [lo, hi] in place (HIP ``dfq_clamp``).  The same
clamp is also available fused into the quantize sweep
(``quantize_targ_layer(..., clip=(lo, hi))``)."""
from __future__ import annotations

import torch.nn as nn

from . import _lib


def clip_weight(graph, range_clip=None, targ_type=[nn.Conv2d, nn.Linear]):
    if range_clip is None:
        range_clip = [-15, 15]
    assert isinstance(range_clip, (list, tuple)) and len(range_clip) == 2, \
        "range_clip should be a list or tuple of two elements"
    lo, hi = float(range_clip[0]), float(range_clip[1])
    for idx, layer in graph.items():
        if isinstance(layer, tuple(targ_type)):
            if hasattr(layer, "weight"):
                w = layer.weight.data
                _lib.require_device(w)
                _lib.check(_lib.load().dfq_clamp(_lib.ptr(w), w.numel(), lo, hi, _lib.stream_of(w)), "dfq_clamp")
            else:
                print(f"Warning: Layer at index {idx} does not have 'weight' attribute")
        else:
            print(f"Warning: Layer at index {idx} is not in the target type list for clipping")
