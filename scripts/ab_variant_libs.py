"""Product-library builds with another default sweep variant, side by side
(build here: `python scripts/ab_variant_libs.py build 9 10`; run on the GPU:
`python scripts/ab_variant_libs.py run 6 9 10`): single-model latency rows and
the bench list's step, one child process per library."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
OUT = ROOT / "data_free_quantization_amd" / "ab"

CODE = """
import json, sys, torch
sys.path.insert(0, {root!r})
from data_free_quantization_amd import _lib
from pathlib import Path
p = {path!r}
if p:
    _lib.LIB_PATH = Path(p)
import bench
dev = torch.device('cuda:0'); s = torch.cuda.current_stream(dev)
r = bench.single_model_latency(dev, s)
items, _, per_copy, copies = bench.build_batch('mobilenetv2', dev)
from data_free_quantization_amd.sweep import SweepPlan
plan = SweepPlan(items)
ms = bench.time_plan(plan, s, dev, 20, 3)
r['bench_list_ms'] = round(ms, 4); r['bench_frac'] = round(plan.stats['algo_bytes'] / ms / 1e6 / 8000, 4)
print(json.dumps(r))
"""


def build(variants):
    from data_free_quantization_amd import build as B
    OUT.mkdir(exist_ok=True)
    for v in variants:
        B._build_one(OUT / f"libdfq_v{v}.so", B.SOURCES, [f"-DDFQ_DEFAULT_VARIANT={v}"], True, False)


def run(variants):
    for v in variants:
        path = "" if v == "6" else str(OUT / f"libdfq_v{v}.so")
        r = subprocess.run([sys.executable, "-c", CODE.format(root=str(ROOT), path=path)], capture_output=True,
                           text=True, timeout=300, cwd=ROOT)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        d = json.loads(line[-1]) if line else {"error": r.stderr[-400:]}
        print(json.dumps({"variant": v, **d}), flush=True)


if __name__ == "__main__":
    (build if sys.argv[1] == "build" else run)(sys.argv[2:])
