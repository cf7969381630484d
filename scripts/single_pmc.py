"""Single-model sweep executes for a PMC pass (one weight set, per-channel W8 +
codes and, unless "w8", the BC error sums): run under
`rocprofv3 --pmc ... --kernel-include-regex sweep_main -- python3 scripts/single_pmc.py [lib.so|-] [model] [w8]`
("w8": without the E sums, BASELINE.md's W8 rows).
An optional library path selects an A/B build (scripts/ab_variant_libs.py)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from data_free_quantization_amd import _lib  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] not in ("", "-"):
    _lib.LIB_PATH = Path(sys.argv[1])
model = sys.argv[2] if len(sys.argv) > 2 else "mobilenetv2"
import bench  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

dev = torch.device("cuda:0")
w8 = len(sys.argv) > 3 and sys.argv[3] == "w8"   # BASELINE.md's W8 rows: no E
items, _, _, _ = bench.build_batch(model, dev, copies=1, seed=5, esum=not w8)
plan = SweepPlan(items)
s = torch.cuda.current_stream(dev)
for _ in range(20):
    plan.execute(s)
torch.cuda.synchronize()
plan.destroy()
print("ok", model, _lib.LIB_PATH)
