"""CLE loop schedules A/B in one process (diagnostics library): the CLE stage
time of run_dfq (per-channel sym INT8, fused BC) and its end-to-end time (no
sync between stages) on MobileNetV2 and ResNet-50,
median of ``--reps`` warm runs per configuration, interleaved; every
configuration also checked against the reference fixture once.

  python scripts/cle_ab.py [--reps 7] [--configs tiles_fin,unfused_steps,...]
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

SWITCHES = ("DFQ_CLE_FUSED", "DFQ_CLE_TILE_GRID", "DFQ_CLE_STEP_GRID", "DFQ_CLE_LAG", "DFQ_CLE_BAND", "DFQ_CLE_STOP",
            "DFQ_CLE_W1_ROWS", "DFQ_CLE_DW_ROWS", "DFQ_CLE_TILES_FIRST",
            "CLE_AB_BLOCKING")
CONFIGS = {
    "tiles_fin": {},                                # the product (lagged schedule where the plan allows it)
    "unfused_steps": {"DFQ_CLE_FUSED": "0"},        # per-step range launches
    "tile_grid_1024": {"DFQ_CLE_TILE_GRID": "1024"},
    "step_grid_1024": {"DFQ_CLE_STEP_GRID": "1024"},
    "step_grid_4096": {"DFQ_CLE_STEP_GRID": "4096"},
    "no_lag": {"DFQ_CLE_LAG": "0"},                 # round 4's schedule: tiles / ranges / stop rule in a launch of their own
    "stop_arrival": {"DFQ_CLE_STOP": "arrival"},    # lagged, the stop rule at the last tile arrival (band of 3)
    "band1": {"DFQ_CLE_BAND": "1"},                 # the tiles' band start (lagged schedule)
    "band2": {"DFQ_CLE_BAND": "2"},
    "blocking": {"CLE_AB_BLOCKING": "1"},           # run_dfq's CLE blocking (no caller gate beside the loop)
    # round 6: rows per W1 / depthwise-pair rescale task (x one row per wave)
    "w1x1": {"DFQ_CLE_W1_ROWS": "1"},               # round 5: one row per wave in every W1 task
    "w1x2": {"DFQ_CLE_W1_ROWS": "2"},
    "w1x4": {"DFQ_CLE_W1_ROWS": "4"},
    "w1x8": {"DFQ_CLE_W1_ROWS": "8"},
    "dwx2": {"DFQ_CLE_DW_ROWS": "2"},
    "w1x4_dwx2": {"DFQ_CLE_W1_ROWS": "4", "DFQ_CLE_DW_ROWS": "2"},
    "tiles_first": {"DFQ_CLE_TILES_FIRST": "1"},   # metric tiles before the rescale tasks (the product)
    "tiles_last": {"DFQ_CLE_TILES_FIRST": "0"},    # round 6 before: tiles after the rescale tasks
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

    import data_free_quantization_amd.pipeline as pipeline_mod
    cle_call = cle.cross_layer_equalization

    def blocking_cle(*args, **kw):
        kw["launch"] = False
        return cle_call(*args, **kw)

    def use(tag):
        for k in SWITCHES:
            os.environ.pop(k, None)
        os.environ.update(CONFIGS[tag])
        pipeline_mod.cle.cross_layer_equalization = blocking_cle if os.environ.get("CLE_AB_BLOCKING") else cle_call

    res = {(t, m): [] for t in cfgs for m in models}
    e2e = {(t, m): [] for t in cfgs for m in models}
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
                # end to end as main_dfq runs it: no sync between the stages
                model = zoo.build(m, seed=0, relu=True).to(dev)
                g = build_graph(model, "positional")
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                with contextlib.redirect_stdout(io.StringIO()):
                    run_dfq(model, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel",
                            symmetric=True, bc_mode="fused")
                torch.cuda.synchronize(dev)
                e2e[(t, m)].append((time.perf_counter() - t0) * 1e3)
    for t in cfgs:
        for m in models:
            v = res[(t, m)]
            print(json.dumps({"config": t, "model": m, "cle_ms_median": round(statistics.median(v), 3),
                              "cle_ms_min": round(min(v), 3),
                              "e2e_ms_median": round(statistics.median(e2e[(t, m)]), 3),
                              "e2e_ms_min": round(min(e2e[(t, m)]), 3), **info[(t, m)],
                              "host_ms_median": {k: round(statistics.median(h[k] for h in host[(t, m)]), 3)
                                                 for k in (host[(t, m)][0] if host[(t, m)] else {})}}), flush=True)


if __name__ == "__main__":
    main()
