"""A/B of the launched (asynchronous) CLE loop against the blocking run, in one
process (diagnostic, GPU): per model, the staged CLE stage time and the
end-to-end run_dfq time (no stage syncs), median of 4 after a warm-up.

    python scripts/cle_async_ab.py [tag]      # tag: printed with the line
"""
import contextlib
import io
import json
import logging
import os
import statistics
import sys
import time
from pathlib import Path

import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from data_free_quantization_amd import Cross_layer_equal as cle, zoo  # noqa: E402
from data_free_quantization_amd.pipeline import run_dfq  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
tag = sys.argv[1] if len(sys.argv) > 1 else ""


def once(name, staged):
    m = zoo.build(name, seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    t = {} if staged else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True,
                bc_mode="fused", timings=t)
    torch.cuda.synchronize()
    total = (time.perf_counter() - t0) * 1e3
    return total, (t["cle"] * 1e3 if staged else None), cle.LAST_RUN.get("host_ms")


_orig = cle.cross_layer_equalization


def _join_first(*a, **k):   # launched, then joined at once (the host idles during the loop)
    _orig(*a, **k)
    cle.wait()


MODES = {"blocking": (False, _orig), "async": (True, _orig), "async_join_first": (True, _join_first)}
if os.environ.get("DFQ_AB_MODES"):   # a subset (DFQ_CLE_ASYNC_NOWAIT runs join-first only)
    MODES = {k: v for k, v in MODES.items() if k in os.environ["DFQ_AB_MODES"].split(",")}
for name in ("mobilenetv2", "resnet50"):
    res = {}
    for rep in range(5):
        for mode, (asy, fn) in MODES.items():
            cle.ASYNC = asy
            cle.cross_layer_equalization = fn
            st_total, st_cle, host = once(name, True)
            e2e, _, _ = once(name, False)
            if rep:
                r = res.setdefault(mode, {"staged_total": [], "staged_cle": [], "end_to_end": []})
                r["staged_total"].append(st_total)
                r["staged_cle"].append(st_cle)
                r["end_to_end"].append(e2e)
    out = {"tag": tag, "model": name}
    for mode, r in res.items():
        out[mode] = {k: round(statistics.median(v), 3) for k, v in r.items()}
    print(json.dumps(out), flush=True)
