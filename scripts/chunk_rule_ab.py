"""Task size against list size: variant 6 (2,048-element tasks) vs 10 (1,536) over
lists of 1..64 weight sets, device us per execute from HIP-graph replays, both
variants alternated twice in the same process.  Evidence for build_planned's rule
(csrc/dfq_sweep.hip).  usage: python scripts/chunk_rule_ab.py  (diagnostics library)"""
import os
os.environ.setdefault("DFQ_LIB", "diag")
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)
CASES = [("mobilenetv2", c) for c in (1, 2, 3, 4, 6, 8, 16, 32, 64)] + \
        [("deeplab", c) for c in (1, 2, 3, 4, 8)] + [("resnet50", c) for c in (1, 2, 4)]
for model, copies in CASES:
    items, _, _, _ = bench.build_batch(model, dev, copies=copies, seed=5, esum=False)
    row = {"model": model, "copies": copies}
    for rep in range(2):
        for v in ("6", "10", ""):
            os.environ["DFQ_SWEEP_VARIANT"] = v
            plan = SweepPlan(items)
            bench.time_plan(plan, stream, dev, 10, 3)
            us = round(bench.time_plan_graph(plan, dev) * 1e3, 2)
            key = f"v{v or 'auto'}"
            row.setdefault(key, []).append(us)
            row[key + "_grid"] = plan.stats["grid_blocks"]
            row[key + "_variant"] = plan.stats["variant"]
            plan.destroy()
    print(json.dumps(row), flush=True)
    del items
    torch.cuda.empty_cache()
