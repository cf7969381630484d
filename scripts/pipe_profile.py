"""cProfile of a warm run_dfq (MobileNetV2, per-channel, fused BC): the host-side
cost of every stage, sorted by own time."""
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
from data_free_quantization_amd import _lib, zoo  # noqa: E402
from data_free_quantization_amd.pipeline import run_dfq  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
_lib.preload()
pr = cProfile.Profile()
for rep in range(3):
    m = zoo.build("mobilenetv2", seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    G, B = g.getGraph(), g.getBottoms()
    torch.cuda.synchronize()
    if rep == 2:
        pr.enable()
    with contextlib.redirect_stdout(io.StringIO()):
        run_dfq(m, G, B, (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True, bc_mode="fused")
    torch.cuda.synchronize()
    if rep == 2:
        pr.disable()
s = io.StringIO()
st = pstats.Stats(pr, stream=s)
st.sort_stats("tottime").print_stats(40)
st.sort_stats("cumtime").print_stats(40)
print(s.getvalue())
