"""Single-model W8 rows (no E) against the whole-row task cap (diagnostic, GPU;
DFQ_SWEEP_TASK_CAP, diagnostics library): kernel-to-kernel us per execute.
usage: python scripts/single_cap.py cap [cap ...]"""
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
caps = [int(c) for c in sys.argv[1:]] or [2048, 1024]
for model in ("mobilenetv2", "deeplab", "resnet50"):
    items, _, _, _ = bench.build_batch(model, dev, copies=1, seed=5, esum=False)
    row = {"model": model}
    for c in caps:
        os.environ["DFQ_SWEEP_TASK_CAP"] = str(c)
        plan = SweepPlan(items)
        bench.time_plan_graph(plan, dev)
        row[str(c)] = round(bench.time_plan_graph(plan, dev) * 1e3, 2)
        row[f"{c}_grid"] = plan.stats["grid_blocks"]
        plan.destroy()
    print(json.dumps(row), flush=True)
