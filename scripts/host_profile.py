"""cProfile of one warm full-DFQ pipeline (host-side hot spots per stage)."""
import contextlib
import cProfile
import io
import logging
import pstats
import sys
from pathlib import Path

import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from data_free_quantization_amd import zoo  # noqa: E402
from data_free_quantization_amd.pipeline import run_dfq  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
name = sys.argv[1] if len(sys.argv) > 1 else "mobilenetv2"
for rep in range(3):
    m = zoo.build(name, seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    torch.cuda.synchronize()
    pr = cProfile.Profile() if rep == 2 else None
    t = {}
    if pr:
        pr.enable()
    with contextlib.redirect_stdout(io.StringIO()):
        run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True,
                bc_mode="fused", timings=t)
    torch.cuda.synchronize()
    if pr:
        pr.disable()
    print(rep, {k: round(v * 1e3, 3) for k, v in t.items()}, flush=True)
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
print(s.getvalue())
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
print(s.getvalue())
