"""Bias-correction chain A/B in one process (diagnostics library): the BC stage
time of run_dfq (per-channel sym INT8, fused BC) and the pipeline total, median
of ``--reps`` warm runs per configuration, interleaved; every configuration
also checked against the reference fixture once.

  python scripts/bc_ab.py [--reps 7] [--configs coop,launches,grid16,...]
"""
import argparse
import contextlib
import io
import json
import logging
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ["DFQ_LIB"] = "diag"

SWITCHES = ("DFQ_BC_CHAIN", "DFQ_BC_GRID", "DFQ_BC_COOPLAUNCH")
CONFIGS = {
    "launches": {},                                                  # the product: one launch per op
    "coop": {"DFQ_BC_CHAIN": "coop"},                                # one launch of 64 co-resident blocks
    "cooplaunch": {"DFQ_BC_CHAIN": "coop", "DFQ_BC_COOPLAUNCH": "1"},   # the same via hipLaunchCooperativeKernel
    "grid16": {"DFQ_BC_CHAIN": "coop", "DFQ_BC_GRID": "16"},
    "grid32": {"DFQ_BC_CHAIN": "coop", "DFQ_BC_GRID": "32"},
    "grid128": {"DFQ_BC_CHAIN": "coop", "DFQ_BC_GRID": "128"},
    "grid256": {"DFQ_BC_CHAIN": "coop", "DFQ_BC_GRID": "256"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--models", default="mobilenetv2,resnet50")
    a = ap.parse_args()
    import torch
    import torch.nn as nn
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.pipeline import run_dfq
    from data_free_quantization_amd.utils.tracer import build_graph
    from tests.parity import pipeline_mismatches
    logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
    dev = torch.device("cuda:0")
    cfgs = a.configs.split(",")
    models = a.models.split(",")

    def use(tag):
        for k in SWITCHES:
            os.environ.pop(k, None)
        os.environ.update(CONFIGS[tag])

    res = {(t, m): [] for t in cfgs for m in models}
    tot = {(t, m): [] for t in cfgs for m in models}
    info = {}
    for t in cfgs:   # parity + warm-up
        use(t)
        for m in models:
            with contextlib.redirect_stdout(io.StringIO()):
                r = pipeline_mismatches(m, 8, dev)
            info[(t, m)] = {"mismatches": r["mismatches"]}
    for rep in range(a.reps):
        for t in cfgs:
            use(t)
            for m in models:
                model = zoo.build(m, seed=0, relu=True).to(dev)
                g = build_graph(model, "positional")
                tm = {}
                with contextlib.redirect_stdout(io.StringIO()):
                    run_dfq(model, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel",
                            symmetric=True, bc_mode="fused", timings=tm)
                torch.cuda.synchronize(dev)
                res[(t, m)].append(tm["bc"] * 1e3)
                tot[(t, m)].append(sum(tm.values()) * 1e3)
    for t in cfgs:
        for m in models:
            v, w = res[(t, m)], tot[(t, m)]
            print(json.dumps({"config": t, "model": m, "bc_ms_median": round(statistics.median(v), 3),
                              "bc_ms_min": round(min(v), 3), "total_ms_median": round(statistics.median(w), 3),
                              **info[(t, m)]}), flush=True)


if __name__ == "__main__":
    main()
