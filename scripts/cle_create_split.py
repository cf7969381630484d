"""Host time of the CLE plan creation on the GPU box: fresh MobileNetV2 / ResNet-50
models (BN-folded, relations built), then Cross_layer_equal._create_plan under
DFQ_CLE_TIMING (the Python split: relations / tables + workspace / plan_create)
and the plan's destroy, 20 times; medians per segment.

  DFQ_CLE_TIMING=1 python scripts/cle_create_split.py [models...]
"""
import contextlib
import io
import json
import os
import re
import statistics
import sys
from pathlib import Path

os.environ.setdefault("DFQ_CLE_TIMING", "1")
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from data_free_quantization_amd import zoo, _lib, Cross_layer_equal as cle  # noqa: E402
from data_free_quantization_amd.utils.layer_transform import merge_batchnorm  # noqa: E402
from data_free_quantization_amd.utils.relation import create_relation  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

T = (nn.Conv2d, nn.Linear)
dev = torch.device("cuda:0")
for name in sys.argv[1:] or ["mobilenetv2", "resnet50"]:
    preps = []
    for _ in range(21):
        m = zoo.build(name, seed=0, relu=True).to(dev)
        g = build_graph(m, "positional")
        G, B = g.getGraph(), g.getBottoms()
        with contextlib.redirect_stdout(io.StringIO()):
            merge_batchnorm(m, G, B, T)
        preps.append((m, G, create_relation(G, B, T)))
    torch.cuda.synchronize()
    rows = []
    for i, (m, G, rels) in enumerate(preps):
        err = io.StringIO()
        with contextlib.redirect_stderr(err):
            plan, ws, _ = cle._create_plan(G, rels, T, [1e-8, 1e8], False, 0)
        _lib.load().dfq_cle_plan_destroy(plan)
        torch.cuda.synchronize()
        mt = re.search(r"relations ([\d.]+) us, tables \+ workspace ([\d.]+) us, plan_create ([\d.]+) us", err.getvalue())
        if i and mt:
            rows.append([float(x) for x in mt.groups()])
    med = [round(statistics.median(c), 1) for c in zip(*rows)]
    print(json.dumps({"model": name, "python_relations_us": med[0], "tables_workspace_us": med[1],
                      "plan_create_us": med[2], "runs": len(rows)}), flush=True)
