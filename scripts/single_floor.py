"""Single-model latency floor (diagnostic, GPU): the W8 row's sweep next to
kernels that only move the same bytes, at the same size, kernel to kernel (HIP
graph replays).  For MobileNetV2 / DeepLab one weight set: read x (4 B/elem),
write dq (4 B) + codes (1 B) -- 9 algorithmic B/elem.
usage: python scripts/single_floor.py [model ...]"""
import os
os.environ.setdefault("DFQ_LIB", "diag")   # the probes live in libdfq_diag.so
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
L = _lib.load()


def graph_us(fn, per_graph=50, replays=8):
    cs = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(g, stream=cs):
        for _ in range(per_graph):
            fn(cs)
    g.replay()
    torch.cuda.synchronize(dev)
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        cur = torch.cuda.current_stream(dev)
        e0.record(cur)
        for _ in range(replays):
            g.replay()
        e1.record(cur)
        torch.cuda.synchronize(dev)
        us = e0.elapsed_time(e1) / (replays * per_graph) * 1e3
        best = us if best is None else min(best, us)
    return round(best, 2)


P = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
S = lambda cs: C.c_void_p(cs.cuda_stream)
for model in sys.argv[1:] or ["mobilenetv2", "deeplab"]:
    items, _, _, _ = bench.build_batch(model, dev, copies=1, seed=5)
    plan = SweepPlan(items)
    n = sum(it.src.numel() for it in items)
    row = {"model": model, "elems": n, "algo_MB": round(9 * n / 1e6, 1),
           "sweep_w8": graph_us(lambda cs: plan.execute(cs))}
    plan.destroy()
    n16 = n // 2048 * 2048
    x = torch.randn(n16, device=dev)
    y = torch.empty_like(x)
    cds = torch.empty(n16, dtype=torch.uint8, device=dev)
    e = torch.empty_like(x)
    row["torch_copy_8B"] = graph_us(lambda cs: y.copy_(x))
    for blocks in (1024, 2048, 4096, n16 // 1024):
        row[f"stream_9B_{blocks}"] = graph_us(lambda cs: L.dfq_probe_stream(P(x), P(y), P(cds), None, n16, blocks, S(cs)))
    row["stream4_9B_1024"] = graph_us(lambda cs: L.dfq_probe_stream(P(x), P(y), P(cds), None, n16, -1024, S(cs)))
    row["stream_4B_read_only_like_copy"] = graph_us(lambda cs: L.dfq_probe_stream(P(x), P(y), None, None, n16,
                                                                                  n16 // 1024, S(cs)))
    for blocks in (n16 // 8192, n16 // 2048 // 4 * 2):
        row[f"lds_copy_8B_{blocks}"] = graph_us(lambda cs: L.dfq_probe_lds(P(x), P(y), None, None, n16, 1, blocks,
                                                                           S(cs)))
    row["lds_mix_13B"] = graph_us(lambda cs: L.dfq_probe_lds(P(x), P(y), P(cds), P(e), n16, 0, n16 // 8192, S(cs)))
    row["empty_like_launch"] = graph_us(lambda cs: L.dfq_probe_stream(P(x), P(y), None, None, 4, 1, S(cs)))
    print(json.dumps(row), flush=True)
    del x, y, cds, e, items
    torch.cuda.empty_cache()
