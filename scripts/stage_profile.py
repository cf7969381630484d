"""cProfile of one warm pipeline stage's host work (argv[1]: bias_correction,
quantize_targ_layer, merge_batchnorm, bias_absorption; default bias_correction)."""
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
from data_free_quantization_amd import bias_correction as BC  # noqa: E402
from data_free_quantization_amd import pipeline  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
_lib.preload()
pr = cProfile.Profile()
fname = sys.argv[1] if len(sys.argv) > 1 else "bias_correction"
orig = getattr(pipeline, fname)


def prof_bc(*a, **k):
    pr.enable()
    try:
        return orig(*a, **k)
    finally:
        pr.disable()


for rep in range(3):
    if rep == 2:
        setattr(pipeline, fname, prof_bc)
    m = zoo.build("mobilenetv2", seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    with contextlib.redirect_stdout(io.StringIO()):
        pipeline.run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel",
                         symmetric=True, bc_mode="fused")
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats(sys.argv[2] if len(sys.argv) > 2 else "cumtime").print_stats(30)
print(s.getvalue())
