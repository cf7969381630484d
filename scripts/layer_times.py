"""Per-layer sweep time of one model (diagnostic): one plan per target layer."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "deeplab"
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)
items, shapes, _, _ = bench.build_batch(model, dev, copies=1, seed=5)
res = []
for it, shp in zip(items, shapes):
    plan = SweepPlan([it])
    ms = bench.time_plan(plan, stream, dev, 50, 5)
    res.append((ms * 1e3, shp, plan.stats["n_tasks_main"], plan.stats["launches"]))
    plan.destroy()
for us, shp, tasks, l in sorted(res, reverse=True)[:10]:
    print(f"{us:8.2f} us  {shp}  tasks={tasks} launches={l}")
print("sum of per-layer us:", round(sum(r[0] for r in res), 1))
