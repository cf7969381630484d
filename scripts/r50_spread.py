"""Where the ResNet-50 x22 sweep's box-to-box spread comes from:
the same secondary config timed in several FRESH processes on one box (each
process allocates its tensors anew, so each lands at a different physical
placement) and, inside each process, over repeated plans on reallocated tensors.
Spread across processes >> spread inside one process -> placement; equal ->
the box.  Prints one JSON line per process and a summary."""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CHILD = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
import bench
from data_free_quantization_amd.sweep import SweepPlan
dev = torch.device("cuda:0"); s = torch.cuda.current_stream(dev)
out = []
for rep in range(3):   # three allocations in this process
    items, _, per_copy, copies = bench.build_batch("resnet50", dev, seed=99 + rep)
    plan = SweepPlan(items)
    ms = bench.time_plan(plan, s, dev, 20, 3, prewarm_ms=200.0)
    out.append(round(plan.stats["algo_bytes"] / ms / 1e6 / bench.HBM_PEAK_GBS, 4))
    plan.destroy(); del items, plan; torch.cuda.empty_cache()
print(json.dumps({"fracs": out}))
"""

res = []
for p in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    r = subprocess.run([sys.executable, "-c", CHILD, str(ROOT)], capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not line:
        print(r.stderr[-2000:])
        sys.exit(1)
    d = json.loads(line[-1])
    d["process"] = p
    print(json.dumps(d), flush=True)
    res.append(d["fracs"])
inside = max(max(f) - min(f) for f in res)
across = max(max(f) for f in res) - min(min(f) for f in res)
print(json.dumps({"max_spread_inside_a_process": round(inside, 4), "spread_across_processes": round(across, 4),
                  "all": res}))
