"""CLE stage A/B across product-library builds with other compile-time CLE
constants (the position-parallel 3x3 tile rows and the POS kernel's wave cap),
side by side, one child process per library and round, alternated.
  build here:      python scripts/cle_lib_ab.py build
  run on the GPU:  python scripts/cle_lib_ab.py run [rounds]"""
import json
import os
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
OUT = ROOT / "data_free_quantization_amd" / "ab"
LIBS = {   # tag: defines (round-6 A/Bs: profiles/r06/cle_lib_ab_*.jsonl)
    "product": [],
    "inner_sum_generic": ["-DDFQ_INNER_SUM_FAST=0"],
}
ALL = {
    "inner_sum_generic": ["-DDFQ_INNER_SUM_FAST=0"],
    "rows2_w3": ["-DDFQ_CLE_POS_ROWS=2", "-DDFQ_CLE_POS_WAVES=3"],
    "rows1_w4": ["-DDFQ_CLE_POS_ROWS=1", "-DDFQ_CLE_POS_WAVES=4"],
    "rows2_w1": ["-DDFQ_CLE_POS_ROWS=2"],
}
if os.environ.get("CLE_LIB_AB"):   # e.g. CLE_LIB_AB=rows2_w3,rows1_w4
    LIBS = {"product": [], **{k: ALL[k] for k in os.environ["CLE_LIB_AB"].split(",")}}

CODE = r"""
import contextlib, io, json, logging, sys, time, torch
import torch.nn as nn
sys.path.insert(0, {root!r})
from pathlib import Path
from data_free_quantization_amd import _lib
p = {path!r}
if p:
    _lib.LIB_PATH = Path(p)
from data_free_quantization_amd import zoo
from data_free_quantization_amd.pipeline import run_dfq
from data_free_quantization_amd.utils.tracer import build_graph
from tests.parity import pipeline_mismatches
logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
dev = torch.device("cuda:0")
out = {{}}
for m in ("deeplab", "resnet50", "mobilenetv2"):
    with contextlib.redirect_stdout(io.StringIO()):
        r = pipeline_mismatches(m, 8, dev)
    if m == "deeplab":   # parity only (run_dfq's fused BC reproduces the reference's cat crash there)
        out[m] = {{"mismatches": r["mismatches"], "cle_ms": [0.0]}}
        continue
    cle = []
    for _ in range({reps}):
        model = zoo.build(m, seed=0, relu=True).to(dev)
        g = build_graph(model, "positional")
        tm = {{}}
        with contextlib.redirect_stdout(io.StringIO()):
            run_dfq(model, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel",
                    symmetric=True, bc_mode="fused", timings=tm)
        torch.cuda.synchronize(dev)
        cle.append(tm["cle"] * 1e3)
    out[m] = {{"mismatches": r["mismatches"], "cle_ms": sorted(cle)}}
print("RESULT " + json.dumps(out))
"""


def build():
    from data_free_quantization_amd import build as B
    OUT.mkdir(exist_ok=True)
    for tag, defs in LIBS.items():
        if defs:
            B._build_one(OUT / f"libdfq_cle_{tag}.so", B.SOURCES, defs, True, False)


def run(rounds):
    res = {tag: {} for tag in LIBS}
    for r in range(rounds):
        for tag, defs in LIBS.items():
            path = str(OUT / f"libdfq_cle_{tag}.so") if defs else ""
            p = subprocess.run([sys.executable, "-c", CODE.format(root=str(ROOT), path=path, reps=5)], cwd=ROOT,
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(json.dumps({"lib": tag, "error": p.stderr[-2000:]}), flush=True)
                sys.exit(1)
            d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1][7:])
            for m, v in d.items():
                e = res[tag].setdefault(m, {"mismatches": 0, "cle_ms": []})
                e["mismatches"] += v["mismatches"]
                e["cle_ms"] += v["cle_ms"]
            print(json.dumps({"round": r, "lib": tag, **{m: round(statistics.median(v["cle_ms"]), 3) for m, v in d.items()}}),
                  flush=True)
    for tag, d in res.items():
        print(json.dumps({"lib": tag, **{m: {"cle_ms_median": round(statistics.median(v["cle_ms"]), 3),
                                              "cle_ms_min": round(min(v["cle_ms"]), 3), "mismatches": v["mismatches"]}
                                          for m, v in d.items()}}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 3)
