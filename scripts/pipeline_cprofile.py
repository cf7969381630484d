"""cProfile of one warm full-DFQ pipeline (host overheads per stage; diagnostic, GPU)."""
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
for rep in range(2):
    m = zoo.build(name, seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    t = {}
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    with contextlib.redirect_stdout(io.StringIO()):
        pr.enable()
        run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True,
                bc_mode="fused", timings=t)
        torch.cuda.synchronize()
        pr.disable()
    print(rep, {k: round(v * 1e3, 3) for k, v in t.items()})
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
print("---- callees of _fold_batch / merge_batchnorm")
st.sort_stats("cumulative").print_callees("_fold_batch")
st.print_callees("merge_batchnorm")
