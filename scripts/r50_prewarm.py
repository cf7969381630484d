"""ResNet-50 x22 secondary config (bench.py SECONDARY[0]) timed as the bench times
it -- after a GPU-idle stretch, 100 ms pre-warm -- and again with longer pre-warms
and back to back, in one process (diagnostic, GPU): does the in-bench figure sit
below the fresh-process one (scripts/r50_spread.py) because the clocks have not
ramped after the host-bound pipeline legs?  Prints one JSON line."""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
items, _, per_copy, copies = bench.build_batch("resnet50", dev, bits=8, channel=True, sym=True, esum=True, seed=99)
plan = SweepPlan(items)
frac = lambda ms: round(plan.stats["algo_bytes"] / ms / 1e6 / bench.HBM_PEAK_GBS, 4)
out = {}
for label, idle_s, pre in (("idle2s_pre100", 2.0, 100.0), ("next_pre100", 0.0, 100.0), ("idle2s_pre600", 2.0, 600.0),
                           ("idle2s_pre100_again", 2.0, 100.0), ("next_pre0", 0.0, 0.0)):
    torch.cuda.synchronize(dev)
    time.sleep(idle_s)
    out[label] = frac(bench.time_plan(plan, s, dev, 20, 3, prewarm_ms=pre))
print(json.dumps(out), flush=True)
plan.destroy()
