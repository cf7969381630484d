"""Single-model sweep attribution by ablation (diagnostic, GPU): BASELINE.md's W8
rows (one weight set, per-channel W8 + codes + clip, no E) timed kernel to kernel
(HIP graph replays) with variant 13's ablation bits -- 1 no row reduce, 2 stores
without the quantize arithmetic, 4 no quantize loop, 8 no input loads, 16 the
launch alone, 32 task / tensor records (and loads) without compute -- next to
the product variant and a stream of the same bytes.  Ablated outputs are wrong;
only the times mean anything.
usage: python scripts/single_ablate.py [model ...]"""
import os
os.environ.setdefault("DFQ_LIB", "diag")
import ctypes as C
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from data_free_quantization_amd import _lib  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

dev = torch.device("cuda:0")
L = _lib.load()
ABL = {"full": 0, "no_reduce": 1, "no_arith": 2, "no_quant": 4, "no_load": 8, "no_reduce_arith": 3,
       "no_reduce_quant": 5, "nothing": 13, "records_loads": 32, "records_only": 40, "launch_only": 16,
       "arith_no_store": 68}

for model in sys.argv[1:] or ["mobilenetv2", "deeplab", "resnet50"]:
    items, _, _, _ = bench.build_batch(model, dev, copies=1, seed=5, esum=False)
    row = {"model": model}
    os.environ["DFQ_SWEEP_VARIANT"] = "6"
    plan = SweepPlan(items)
    bench.time_plan_graph(plan, dev)
    row["v6"] = round(bench.time_plan_graph(plan, dev) * 1e3, 2)
    plan.destroy()
    os.environ["DFQ_SWEEP_VARIANT"] = "13"
    _lib.check(L.dfq_debug_timeline(None, 0), "timeline off")
    plan = SweepPlan(items)
    for name, bits in ABL.items():
        _lib.check(L.dfq_debug_ablate(bits), "ablate")
        bench.time_plan_graph(plan, dev)
        row[name] = round(bench.time_plan_graph(plan, dev) * 1e3, 2)
    _lib.check(L.dfq_debug_ablate(0), "ablate off")
    plan.destroy()
    n = sum(it.src.numel() for it in items) // 2048 * 2048
    x = torch.randn(n, device=dev)
    y = torch.empty_like(x)
    cds = torch.empty(n, dtype=torch.uint8, device=dev)

    class _P:   # a stand-in plan for time_plan_graph: the same bytes as a plain stream
        def execute(self, cs):
            L.dfq_probe_stream(C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(cds.data_ptr()), None,
                               n, 1024, C.c_void_p(cs.cuda_stream))
    bench.time_plan_graph(_P(), dev)
    row["stream_same_bytes"] = round(bench.time_plan_graph(_P(), dev) * 1e3, 2)
    print(json.dumps(row), flush=True)
    del items, x, y, cds
    torch.cuda.empty_cache()
