"""The CLE device loop alone (blocking, the product schedule) on a fresh model
after the first BN fold, ``--reps`` times; one JSON line per run with the
iterations, the iteration groups launched, the loop's device ms (one HIP event
pair: Cross_layer_equal.DEVICE_TIMING) and the algorithmic bytes per iteration.
The process under scripts/cle_pmc.sh's rocprofv3 passes.

  python scripts/cle_loop_once.py [--model mobilenetv2] [--reps 2]
"""
import argparse
import contextlib
import io
import json
import sys
from pathlib import Path

import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from data_free_quantization_amd import zoo, Cross_layer_equal as cle  # noqa: E402
from data_free_quantization_amd.utils.layer_transform import merge_batchnorm  # noqa: E402
from data_free_quantization_amd.utils.relation import create_relation  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="mobilenetv2")
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
T = (nn.Conv2d, nn.Linear)
dev = torch.device("cuda:0")
cle.DEVICE_TIMING = True
for rep in range(a.reps):
    m = zoo.build(a.model, seed=0, relu=True).to(dev)
    g = build_graph(m, "positional")
    G, B = g.getGraph(), g.getBottoms()
    with contextlib.redirect_stdout(io.StringIO()):
        merge_batchnorm(m, G, B, T)
        rels = create_relation(G, B, T)
        torch.cuda.synchronize()
        cle.cross_layer_equalization(G, rels, T, Save_state=False, Treshhold=2e-7, launch=False)
    r = cle.LAST_RUN
    print(json.dumps({"model": a.model, "rep": rep, "iterations": r["iterations"],
                      "iterations_launched": r["iterations_launched"], "device_ms": r["device_ms"],
                      "launches_per_iteration": r["launches_per_iteration"],
                      "bytes_per_iteration": r["bytes_per_iteration"]}), flush=True)
