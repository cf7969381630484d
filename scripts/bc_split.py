"""Where the bias-correction stage's time goes (warm run): host walk until the
chain is flushed, the flush call itself, and the device drain after it."""
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
from data_free_quantization_amd import bias_correction as BC  # noqa: E402
from data_free_quantization_amd.pipeline import run_dfq  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
name = sys.argv[1] if len(sys.argv) > 1 else "mobilenetv2"
_lib.preload()
rec = {}
orig = BC._BcChain.flush


def flush(self, stream):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rec["ops"] = len(self.ops)
    orig(self, stream)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    rec["flush_ms"] = round((t1 - t0) * 1e3, 3)
    rec["drain_ms"] = round((t2 - t1) * 1e3, 3)


BC._BcChain.flush = flush
for rep in range(3):
    m = zoo.build(name, seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    t = {}
    with contextlib.redirect_stdout(io.StringIO()):
        run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True,
                bc_mode="fused", timings=t)
    rec["bc_ms"] = round(t["bc"] * 1e3, 3)
    print(json.dumps(rec))
