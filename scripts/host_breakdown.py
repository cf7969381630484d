"""Where the host time of the host-bound pipeline stages goes (warm, MobileNetV2):
merge_batchnorm's graph walk / descriptor build / C call / buffer and hook
bookkeeping, bias_absorption, quantize_targ_layer and bias_correction, each timed
with the GPU idle before and after (diagnostic)."""
import contextlib
import io
import json
import logging
import sys
import time
from pathlib import Path

import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from data_free_quantization_amd import zoo, _lib  # noqa: E402
from data_free_quantization_amd.utils import layer_transform as LT  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
T = (nn.Conv2d, nn.Linear)
acc = {}


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
    return w


L = _lib.load()
LT._identity_forward = timed("bn.identity_forward", LT._identity_forward)
LT._carve = timed("bn.carve", LT._carve)
_lib.require_device = timed("require_device", _lib.require_device)
for rep in range(3):
    acc.clear()
    m = zoo.build("mobilenetv2", seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    G, B = g.getGraph(), g.getBottoms()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    LT.merge_batchnorm(m, G, B, T)
    torch.cuda.synchronize()
    acc["bn1.total"] = time.perf_counter() - t0
print(json.dumps({k: round(v * 1e3, 3) for k, v in acc.items()}))
