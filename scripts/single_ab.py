"""Single-model sweep latency per kernel variant: one weight set,
per-channel sym INT8 + codes + clip + BC sums, device us per execute from HIP
graph replays (a Python execute() alone costs more than one small sweep).
usage: python scripts/single_ab.py [variants...]   (env DFQ_SWEEP_BLOCKS_PER_CU applies;
DFQ_SINGLE_ESUM=0: no E, the W8 rows)"""
import os
os.environ.setdefault("DFQ_LIB", "diag")   # A/B variants, switches and probes: libdfq_diag.so
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

variants = [int(v) for v in sys.argv[1:]] or [6]
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)
for model in ("mobilenetv2", "resnet50", "deeplab"):
    esum = os.environ.get("DFQ_SINGLE_ESUM", "1") != "0"   # 0: BASELINE.md's W8 rows (no E)
    items, _, _, _ = bench.build_batch(model, dev, copies=1, seed=5, esum=esum)
    row = {"model": model, "esum": esum, "bpc": os.environ.get("DFQ_SWEEP_BLOCKS_PER_CU", "64")}
    for v in variants:
        os.environ["DFQ_SWEEP_VARIANT"] = str(v)
        plan = SweepPlan(items)
        bench.time_plan(plan, stream, dev, 20, 5)                 # warm (host-paced rate: not reported)
        ms = bench.time_plan_graph(plan, dev)                      # kernel-to-kernel (HIP graph replays)
        row[f"v{v}"] = round(ms * 1e3, 2)
        row[f"v{v}_grid"] = plan.stats["grid_blocks"]
        plan.destroy()
    print(json.dumps(row), flush=True)
