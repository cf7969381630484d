"""Achievable-ceiling probes next to the sweep, on one box (diagnostic).

Prints algorithmic GB/s for: the sweep (MobileNetV2 x155 batch), the flat
same-mix stream (bench.py's probe), the sweep's own memory pattern without
arithmetic (LDS-DMA in, non-temporal out), and plain copies."""
import os
os.environ.setdefault("DFQ_LIB", "diag")   # A/B variants, switches and probes: libdfq_diag.so
import ctypes as C
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from data_free_quantization_amd import _lib  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)
L = _lib.load()
s = C.c_void_p(stream.cuda_stream)


def timed(fn, reps=10):
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        best = ms if best is None else min(best, ms)
    return best


out = {}
items, _, per_copy, copies = bench.build_batch("mobilenetv2", dev)
plan = SweepPlan(items)
ms = timed(lambda: plan.execute(stream))
out["sweep_mbv2"] = round(plan.stats["algo_bytes"] / ms / 1e6, 1)
plan.destroy()
del items, plan
torch.cuda.empty_cache()
n = per_copy * copies // 2048 * 2048
x = torch.randn(n, device=dev)
y = torch.empty_like(x)
cds = torch.empty(n, dtype=torch.uint8, device=dev)
e = torch.empty_like(x)
P = lambda t: C.c_void_p(t.data_ptr())
for blocks in (2048, 8192):
    ms = timed(lambda: L.dfq_probe_stream(P(x), P(y), P(cds), P(e), n, blocks, s))
    out[f"flat_mix_{blocks}"] = round(13 * n / ms / 1e6, 1)
ms = timed(lambda: L.dfq_probe_stream(P(x), P(y), P(cds), P(e), n, -4096, s))
out["flat_mix_4deep"] = round(13 * n / ms / 1e6, 1)
for blocks in (1024, 2048, 4096):
    ms = timed(lambda: L.dfq_probe_lds(P(x), P(y), P(cds), P(e), n, 0, blocks, s))
    out[f"lds_mix_{blocks}"] = round(13 * n / ms / 1e6, 1)
    ms = timed(lambda: L.dfq_probe_lds(P(x), P(y), None, None, n, 1, blocks, s))
    out[f"lds_copy_{blocks}"] = round(8 * n / ms / 1e6, 1)
for blocks in (2048, 8192):
    ms = timed(lambda: L.dfq_probe_stream(P(x), P(y), None, None, n, blocks, s))
    out[f"flat_copy_{blocks}"] = round(8 * n / ms / 1e6, 1)
print(json.dumps(out))
