"""Sweep-kernel throughput per layer-shape family (diagnostic, GPU).

Each family is a >= 1 GiB batch of identical conv/linear weights; per-channel sym
INT8 + codes + clip, with and without the BC error sums.  Prints one JSON line
per (family, esum): algorithmic GB/s of one execute() and the plan's task mix.
"""
import os
os.environ.setdefault("DFQ_LIB", "diag")   # A/B variants, switches and probes: libdfq_diag.so
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from data_free_quantization_amd.sweep import SweepPlan, allocate, khw_of  # noqa: E402

FAMILIES = {
    "1x1_256x256": (256, 256, 1, 1),
    "1x1_1024x2048": (1024, 2048, 1, 1),
    "3x3_256x64(row576)": (256, 64, 3, 3),
    "3x3_256x128(row1152)": (256, 128, 3, 3),
    "3x3_256x256(row2304)": (256, 256, 3, 3),
    "3x3_256x320(row2880)": (256, 320, 3, 3),
    "3x3_512x512(row4608)": (512, 512, 3, 3),
    "dw3x3_960x1": (960, 1, 3, 3),
    "fc_256x4096(row4096)": (256, 4096),
    "fc_256x1024(row1024)": (256, 1024),
    "fc_256x1152(row1152)": (256, 1152),
    "fc_256x2304(row2304)": (256, 2304),
    "fc_256x576(row576)": (256, 576),
    "fc_1000x1280(row1280)": (1000, 1280),
    "1x1_960x160": (960, 160, 1, 1),
    "1x1_160x960": (160, 960, 1, 1),
}


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    only = sys.argv[1:] or list(FAMILIES)
    for name in only:
        shp = FAMILIES[name]
        n = int(torch.Size(shp).numel())
        copies = max(1, (1 << 30) // (4 * n))
        ws = torch.randn((copies,) + shp, device=dev) * 0.05
        for esum in (True, False):
            items = [allocate(ws[c], bits=8, per_channel=True, symmetric=True, khw=khw_of(ws[c]), want_esum=esum,
                              clip=(-15.0, 15.0)) for c in range(copies)]
            plan = SweepPlan(items)
            for _ in range(3):
                plan.execute(stream)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record(stream)
            for _ in range(reps):
                plan.execute(stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / reps
            st = plan.stats
            print(json.dumps({"family": name, "esum": esum, "copies": copies, "ms": round(ms, 4),
                              "algo_GBs": round(st["algo_bytes"] / ms / 1e6, 1),
                              "weight_GBs": round(4 * n * copies / ms / 1e6, 1), "tasks": st["n_tasks_main"],
                              "reduce_tasks": st["n_tasks_reduce"], "launches": st["launches"],
                              "variant": st["variant"], "blockrow": os.environ.get("DFQ_SWEEP_BLOCKROW", "1")}),
                  flush=True)
            plan.destroy()
            del items, plan
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
