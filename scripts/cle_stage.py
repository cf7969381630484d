"""CLE stage timing in one process (GPU): bench.pipeline_timing's stage-synced CLE
stage and end-to-end time, and bench.cle_roofline's device loop, for the models
given; ``--reps`` alternations.  Prints one JSON line per model and rep.

  python scripts/cle_stage.py [--models mobilenetv2 resnet50] [--reps 3]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--models", nargs="+", default=["mobilenetv2", "resnet50"])
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda:0")
for rep in range(a.reps):
    for m in a.models:
        p = bench.pipeline_timing(dev, m)
        r = bench.cle_roofline(dev, m)
        print(json.dumps({"rep": rep, "model": m, "cle_ms": p["cle"], "total_ms": p["total"],
                          "end_to_end_ms": p["end_to_end"], "cle_host_ms": p.get("cle_host_ms"),
                          "loop_device_ms": r["loop_device_ms"], "us_per_iteration": r["device_us_per_iteration"],
                          "frac": r["frac"]}), flush=True)
