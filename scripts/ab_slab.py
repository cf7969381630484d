"""Per-tensor (quantize_targ_layer's mode) sweep on the replicated MobileNetV2
bench list: device ms per execute for several slab sizes of the two-stream
reduce / quantize pipeline (diagnostics library: DFQ_SWEEP_SLAB_MB), interleaved."""
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
items, _, per_copy, copies = bench.build_batch("mobilenetv2", dev, bits=8, channel=False, sym=False, esum=False,
                                               seed=99)
sizes = [int(x) for x in (sys.argv[1:] or ["0", "16", "32", "64", "128", "256"])]
plans = {}
for mb in sizes:
    os.environ["DFQ_SWEEP_SLAB_MB"] = str(mb)
    plans[mb] = SweepPlan(items)
res = {mb: [] for mb in sizes}
for rep in range(3):
    for mb in sizes:
        ms = bench.time_plan(plans[mb], stream, dev, 20, 3)
        res[mb].append(ms)
out = []
for mb in sizes:
    ms = min(res[mb])
    st = plans[mb].stats
    out.append({"slab_mb": mb, "ms": round(ms, 4), "launches": st["launches"],
                "algo_TBs": round(st["algo_bytes"] / ms / 1e9, 3), "frac": round(st["algo_bytes"] / ms / 1e9 / 8.0, 4)})
print(json.dumps(out))
