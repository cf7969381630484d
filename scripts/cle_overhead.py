"""Host-side breakdown of one device CLE call (plan create / run / destroy) on a
model after BN folding: where the non-kernel time of the CLE stage goes."""
import os
os.environ.setdefault("DFQ_LIB", "diag")   # A/B variants, switches and probes: libdfq_diag.so
import contextlib
import io
import sys
import time
from pathlib import Path

import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from data_free_quantization_amd import _lib, zoo  # noqa: E402
from data_free_quantization_amd import Cross_layer_equal as cle  # noqa: E402
from data_free_quantization_amd.utils.layer_transform import merge_batchnorm  # noqa: E402
from data_free_quantization_amd.utils.relation import create_relation  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "mobilenetv2"
L = _lib.load()
acc = {}
for fn in ("dfq_cle_plan_create", "dfq_cle_plan_run", "dfq_cle_plan_destroy"):
    orig = getattr(L, fn)

    def wrap(*a, _o=orig, _n=fn):
        t0 = time.perf_counter()
        r = _o(*a)
        acc[_n] = acc.get(_n, 0.0) + time.perf_counter() - t0
        return r
    setattr(L, fn, wrap)
for rep in range(3):
    acc.clear()
    m = zoo.build(name, seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    graph, bottoms = g.getGraph(), g.getBottoms()
    with contextlib.redirect_stdout(io.StringIO()):
        merge_batchnorm(m, graph, bottoms, (nn.Conv2d, nn.Linear))
        rels = create_relation(graph, bottoms, (nn.Conv2d, nn.Linear))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cle.cross_layer_equalization(graph, rels, (nn.Conv2d, nn.Linear), Save_state=False)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    print(rep, name, "total_ms", round(tot * 1e3, 3), {k: round(v * 1e3, 3) for k, v in acc.items()},
          cle.LAST_RUN.get("iterations"), flush=True)
