"""Per-task timeline of one single-model sweep (diagnostic, GPU; variant 13).

usage: python scripts/timeline.py [model] [copies]
Prints the kernel span and, per phase, when tasks started / had their data /
finished (us from the first task start), plus latency percentiles.  Timestamps
are s_memrealtime (100 MHz, 10 ns resolution)."""
import os
os.environ.setdefault("DFQ_LIB", "diag")   # A/B variants, switches and probes: libdfq_diag.so
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ["DFQ_SWEEP_VARIANT"] = "13"
import bench  # noqa: E402
from data_free_quantization_amd import _lib  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "mobilenetv2"
copies = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)
esum = os.environ.get("DFQ_SINGLE_ESUM", "1") != "0"   # 0: BASELINE.md's W8 rows (no E)
items, _, _, _ = bench.build_batch(model, dev, copies=copies, seed=5, esum=esum)
plan = SweepPlan(items)
n = plan.stats["n_tasks_main"]
buf = torch.zeros(8 * n, dtype=torch.int64, device=dev)
L = _lib.load()
us = bench.time_plan(plan, stream, dev, 100, 10) * 1e3
_lib.check(L.dfq_debug_timeline(buf.data_ptr(), n), "timeline")
for _ in range(3):
    plan.execute(stream)
torch.cuda.synchronize(dev)
_lib.check(L.dfq_debug_timeline(None, 0), "timeline off")
r = buf.view(n, 8).cpu().numpy().astype(np.int64)
t0 = r[:, 0].min()
start, landed, params, quant, done = [(r[:, k] - t0) / 100.0 for k in range(5)]   # us
has_sub = r[:, 6] > 0   # whole-row tasks: first rows' ranges reduced, their parameters built
ranged, built = [(r[:, k] - t0) / 100.0 for k in (6, 7)]
q = lambda a: [round(float(np.percentile(a, p)), 2) for p in (0, 10, 50, 90, 99, 100)]
out = {"model": model, "copies": copies, "tasks": n, "grid": plan.stats["grid_blocks"], "event_us": round(us, 2),
       "span_us": round(float(done.max()), 2),
       "start_pct": q(start), "landed_pct": q(landed), "done_pct": q(done),
       "load_lat_pct": q(landed - start), "compute_pct": q(done - landed),
       "row_params_pct": q(params - landed), "quant_loop_pct": q(quant - params), "esum_tail_pct": q(done - quant),
       "whole_row_tasks": int(has_sub.sum()),
       "row_reduce_pct": q((ranged - landed)[has_sub]) if has_sub.any() else None,
       "make_qparams_pct": q((built - ranged)[has_sub]) if has_sub.any() else None,
       "params_sync_pct": q((params - built)[has_sub]) if has_sub.any() else None}
# how many waves were live over time (1 us bins)
bins = np.arange(0, done.max() + 1.0, 1.0)
live = [int(((start <= b) & (done > b)).sum()) for b in bins]
out["live_tasks_per_us"] = live
xcc = (r[:, 5] >> 32) & 0xFF
out["tasks_per_xcc"] = np.bincount(xcc, minlength=8).tolist()
# per task kind (float4 rows / scalar rows, row length): where the compute goes
tix = r[:, 5] >> 40
kinds = {}
for ti in np.unique(tix):
    w = items[int(ti)].src
    rl = int(w[0].numel()) if w.dim() > 1 else int(w.numel())
    key = f"{'vec' if rl % 4 == 0 else 'scalar'}_len{rl if rl <= 64 else ('<=576' if rl <= 576 else '>576')}"
    kinds.setdefault(key, []).append(ti)
for key, tis in sorted(kinds.items()):
    m = np.isin(tix, tis)
    out["kind_" + key] = {"tasks": int(m.sum()), "compute_p50": round(float(np.median((done - landed)[m])), 2),
                          "row_params_p50": round(float(np.median((params - landed)[m])), 2),
                          "quant_p50": round(float(np.median((quant - params)[m])), 2),
                          "done_p90": round(float(np.percentile(done[m], 90)), 2)}
# the last tasks to finish: what they are and where their time went
kind_of = {}
for key, tis in kinds.items():
    for ti in tis:
        kind_of[int(ti)] = key
last = np.argsort(done)[-12:][::-1]
out["last_tasks"] = [{"kind": kind_of[int(tix[i])], "tensor": int(tix[i]), "start": round(float(start[i]), 2),
                      "landed": round(float(landed[i]), 2), "params": round(float(params[i]), 2),
                      "quant": round(float(quant[i]), 2), "done": round(float(done[i]), 2)} for i in last]
print(json.dumps(out))
plan.destroy()
