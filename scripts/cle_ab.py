"""CLE loop schedules A/B in one process (diagnostics library): the CLE stage
time of run_dfq (per-channel sym INT8, fused BC) on MobileNetV2 and ResNet-50,
median of ``--reps`` warm runs per configuration, interleaved; every
configuration also checked against the reference fixture once.

  python scripts/cle_ab.py [--reps 7] [--configs grouped,tiles_fin,...]
"""
import argparse
import contextlib
import io
import json
import logging
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ["DFQ_LIB"] = "diag"

SWITCHES = ("DFQ_CLE_UNFUSED_FIN", "DFQ_CLE_GROUPS", "DFQ_CLE_GROUP_GRID", "DFQ_CLE_ORDERED", "DFQ_CLE_GSYNC_NOFENCE",
            "DFQ_CLE_NO_DW_PAIRS", "DFQ_CLE_FORK", "DFQ_CLE_NO_SELF_RANGES", "DFQ_CLE_GRAPH",
            "DFQ_CLE_BATCH", "DFQ_CLE_APPLY_OCC4",
            "DFQ_CLE_POS_ROWS")
CONFIGS = {
    "tiles_fin": {},                                       # the product (eager batches of 4)
    "no_dw_pairs": {"DFQ_CLE_NO_DW_PAIRS": "1"},           # round-2 steps: one launch per relation
    "fork": {"DFQ_CLE_FORK": "1"},                         # next ranges on a concurrent graph branch
    "no_self_ranges": {"DFQ_CLE_NO_SELF_RANGES": "1"},     # every next range from a range task
    "apply_occ4": {"DFQ_CLE_APPLY_OCC4": "1"},              # rescale kernel capped at 128 VGPRs (4 waves / SIMD)
    "pos_rows16": {"DFQ_CLE_POS_ROWS": "16"},               # 3x3 rescale tiles of 16 rows (round 2)
    "graph": {"DFQ_CLE_GRAPH": "1"},                       # each batch replayed as a (cached) HIP graph
    "batch8": {"DFQ_CLE_BATCH": "8"},
    "batch2": {"DFQ_CLE_BATCH": "2"},
    "tiles_fin_ordered": {"DFQ_CLE_ORDERED": "1"},
    "grouped": {"DFQ_CLE_GROUPS": "1"},
    "grouped_ordered": {"DFQ_CLE_GROUPS": "1", "DFQ_CLE_ORDERED": "1"},
    "grouped_512": {"DFQ_CLE_GROUPS": "1", "DFQ_CLE_GROUP_GRID": "512"},
    "grouped_nofence": {"DFQ_CLE_GROUPS": "1", "DFQ_CLE_GSYNC_NOFENCE": "1"},   # timing only: stale results
    "grouped_nofence_1024": {"DFQ_CLE_GROUPS": "1", "DFQ_CLE_GSYNC_NOFENCE": "1", "DFQ_CLE_GROUP_GRID": "1024"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--models", default="mobilenetv2,resnet50")
    a = ap.parse_args()
    import torch
    import torch.nn as nn
    from data_free_quantization_amd import zoo, Cross_layer_equal as cle
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
    host = {(t, m): [] for t in cfgs for m in models}
    info = {}
    for t in cfgs:   # parity + warm-up
        use(t)
        for m in models:
            with contextlib.redirect_stdout(io.StringIO()):
                r = pipeline_mismatches(m, 8, dev)
            info[(t, m)] = {"mismatches": r["mismatches"], "launches": cle.LAST_RUN.get("launches_per_iteration"),
                            "iterations": r["cle_iterations"]}
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
                res[(t, m)].append(tm["cle"] * 1e3)
                host[(t, m)].append(cle.LAST_RUN.get("host_ms", {}))
    for t in cfgs:
        for m in models:
            v = res[(t, m)]
            print(json.dumps({"config": t, "model": m, "cle_ms_median": round(statistics.median(v), 3),
                              "cle_ms_min": round(min(v), 3), **info[(t, m)],
                              "host_ms_median": {k: round(statistics.median(h[k] for h in host[(t, m)]), 3)
                                                 for k in (host[(t, m)][0] if host[(t, m)] else {})}}), flush=True)


if __name__ == "__main__":
    main()
