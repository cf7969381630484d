"""Single-model sweep time for subsets of a model's layers (diagnostic)."""
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
pairs = list(zip(items, shapes))
subsets = {
    "all": pairs,
    "dw only": [p for p in pairs if len(p[1]) == 4 and p[1][1] == 1],
    "no dw": [p for p in pairs if not (len(p[1]) == 4 and p[1][1] == 1)],
    "3x3 dense": [p for p in pairs if len(p[1]) == 4 and p[1][2] == 3 and p[1][1] > 1],
    "1x1": [p for p in pairs if len(p[1]) == 4 and p[1][2] == 1],
}
for name, sub in subsets.items():
    if not sub:
        continue
    plan = SweepPlan([p[0] for p in sub])
    ms = bench.time_plan(plan, stream, dev, 100, 10)
    st = plan.stats
    print(f"{name:10s} layers={len(sub):3d} us={ms * 1e3:8.2f} tasks={st['n_tasks_main']} grid={st['grid_blocks']} "
          f"launches={st['launches']} GB/s={st['algo_bytes'] / ms / 1e6:.0f}")
    plan.destroy()
big = sorted(pairs, key=lambda p: -p[0].src.numel())[:5]
print("largest:", [p[1] for p in big])
