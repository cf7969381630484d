"""Row groups vs whole-row tasks / block-row pieces (diagnostics library,
DFQ_SWEEP_GROUP_ROWS) on the bench's secondary configs: device ms per execute,
interleaved on one box."""
import json
import os
import sys
from pathlib import Path

os.environ["DFQ_LIB"] = "diag"
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import bench  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)
out = []
for name, model, bits, ch, sym, es, *pack in bench.SECONDARY[:4] + [("mobilenetv2 bench", "mobilenetv2", 8, True, True,
                                                                      True)]:
    items, _, per_copy, copies = bench.build_batch(model, dev, bits=bits, channel=ch, sym=sym, esum=es, seed=99,
                                                   pack=bool(pack and pack[0]))
    plans = {}
    for g in ("0", "1"):
        os.environ["DFQ_SWEEP_GROUP_ROWS"] = g
        plans[g] = SweepPlan(items)
    res = {"0": [], "1": []}
    for rep in range(4):
        for g in ("0", "1"):
            res[g].append(bench.time_plan(plans[g], stream, dev, 15, 3))
    row = {"config": name}
    for g in ("0", "1"):
        ms = min(res[g])
        row[f"group{g}_ms"] = round(ms, 4)
        row[f"group{g}_frac"] = round(plans[g].stats["algo_bytes"] / ms / 1e9 / 8.0, 4)
        row[f"group{g}_tasks"] = plans[g].stats["n_tasks_main"]
        plans[g].destroy()
    out.append(row)
    del items, plans
    torch.cuda.empty_cache()
print(json.dumps(out))
