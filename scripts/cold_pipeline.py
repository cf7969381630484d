"""Cold vs warm full-DFQ pipeline (main_dfq's stage order) in a fresh process:
stage milliseconds of the first run (library and kernel loading, first
allocations, CLE graph capture) and of the second."""
import contextlib
import io
import json
import logging
import sys
import time
from pathlib import Path

import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from data_free_quantization_amd import _lib, zoo  # noqa: E402
from data_free_quantization_amd.pipeline import run_dfq  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
args = [a for a in sys.argv[1:] if not a.startswith("--")]
name = args[0] if args else "mobilenetv2"
torch.zeros(1, device="cuda:0")   # the CUDA context is not the DFQ path's cost
out = {}
if "--preload" in sys.argv:       # what main_dfq does before its timer
    t0 = time.perf_counter()
    _lib.preload()
    out["preload_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
for rep in ("cold", "warm"):
    m = zoo.build(name, seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    t = {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True,
                bc_mode="fused", timings=t)
    torch.cuda.synchronize()
    out[rep] = {k: round(v * 1e3, 3) for k, v in t.items()}
    out[rep]["total"] = round((time.perf_counter() - t0) * 1e3, 3)
print(json.dumps(out))
