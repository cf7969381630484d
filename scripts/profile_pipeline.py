"""One warm full-DFQ pipeline on MobileNetV2 (for rocprofv3 kernel traces)."""
import contextlib
import io
import logging
import sys
import time
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
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True,
                bc_mode="fused", timings=t)
    torch.cuda.synchronize()
    from data_free_quantization_amd import Cross_layer_equal as cle
    print(rep, {k: round(v * 1e3, 3) for k, v in t.items()}, round((time.perf_counter() - t0) * 1e3, 3),
          {k: v for k, v in cle.LAST_RUN.items() if k != "diffs"}, flush=True)
