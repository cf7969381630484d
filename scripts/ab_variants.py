"""A/B the sweep kernel variants in ONE process on the same data (interleaved
rounds, median and min per variant; cdna_hip_programming.md 5.4 rule 24)."""
import os
os.environ.setdefault("DFQ_LIB", "diag")   # A/B variants, switches and probes: libdfq_diag.so
import json
import os
import statistics
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="0,2,4,5")
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--model", default="mobilenetv2")
    p.add_argument("--no-esum", action="store_true")
    p.add_argument("--asym", action="store_true")
    p.add_argument("--tensor", action="store_true", help="per-tensor ranges (quantize_targ_layer's mode)")
    a = p.parse_args()
    import bench
    from data_free_quantization_amd.sweep import SweepPlan
    dev = torch.device("cuda:0")
    items, shapes, per_copy, copies = bench.build_batch(a.model, dev, channel=not a.tensor, sym=not a.asym,
                                                          esum=not a.no_esum)
    plans = {}
    for v in [int(x) for x in a.variants.split(",")]:
        os.environ["DFQ_SWEEP_VARIANT"] = str(v)
        plans[v] = SweepPlan(items)
    stream = torch.cuda.current_stream(dev)
    times = {v: [] for v in plans}
    for v, pl in plans.items():
        for _ in range(3):
            pl.execute(stream)
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for v, pl in plans.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                pl.execute(stream)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.reps)
    # same-mix streaming probe (13 B / element: read 4, write 4 + 1 + 4)
    import ctypes as C
    from data_free_quantization_amd import _lib
    n = per_copy * copies // 16 * 16
    x = torch.randn(n, device=dev)
    y = torch.empty_like(x)
    cds = torch.empty(n, dtype=torch.uint8, device=dev)
    e = torch.empty_like(x)
    L = _lib.load()
    pt = []
    for blocks in (2048, 8192, -2048, -4096, -8192):
        for r in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                _lib.check(L.dfq_probe_stream(_lib.ptr(x), _lib.ptr(y), None if a.no_esum else C.c_void_p(cds.data_ptr()),
                                              None if a.no_esum else _lib.ptr(e), n, blocks, _lib.stream_of(x)), "probe")
            e1.record(stream)
            torch.cuda.synchronize()
            pt.append((e0.elapsed_time(e1) / a.reps, blocks))
    best = min(pt)
    probe_bytes = (4 + 4 + (0 if a.no_esum else 5)) * n
    probe = dict(ms=round(best[0], 4), blocks=best[1], GBs=round(probe_bytes / (best[0] / 1e3) / 1e9, 1))
    out = {}
    for v, pl in plans.items():
        med = statistics.median(times[v])
        gbs = pl.stats["algo_bytes"] / (med / 1e3) / 1e9
        out[v] = dict(median_ms=round(med, 4), min_ms=round(min(times[v]), 4), algo_GBs=round(gbs, 1),
                      frac=round(gbs / 8000, 4), tasks=pl.stats["n_tasks_main"], grid=pl.stats["grid_blocks"])
    print(json.dumps(dict(model=a.model, copies=copies, no_esum=a.no_esum, probe=probe, variants=out)))


if __name__ == "__main__":
    main()
