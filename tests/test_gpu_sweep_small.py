"""Small sweep lists (one round of resident blocks even at 1,536-element tasks: a
single MobileNetV2) get variant 10; larger lists keep variant 6.  The product
library picks the variant on its own and matches the C oracle; the diagnostics
library's variant-10 result equals a forced variant 6 bit for bit (fresh processes)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, os.environ["DFQ_ROOT"])
import torch
import bench
from data_free_quantization_amd.sweep import SweepPlan
from tests.parity import sweep_mismatches
dev = torch.device("cuda:0")
diag = os.environ.get("DFQ_LIB") == "diag"
CASES = [("mobilenetv2", 1, 8, True, True, False), ("mobilenetv2", 1, 4, False, False, True),
         ("mobilenetv2", 1, 8, True, False, False), ("mobilenetv2", 2, 8, True, True, False),
         ("resnet50", 1, 8, True, True, False), ("deeplab", 1, 8, True, True, False)]
out = []
for model, copies, bits, sym, esum, pack in CASES:
    res = {}
    for v in (("", "6") if diag else ("",)):
        os.environ["DFQ_SWEEP_VARIANT"] = v
        items, shapes, _, _ = bench.build_batch(model, dev, copies=copies, bits=bits, channel=True, sym=sym,
                                                esum=esum, seed=91, pack=pack)
        plan = SweepPlan(items)
        plan.execute()
        torch.cuda.synchronize()
        res[v] = (items, plan.stats["variant"], plan.stats["grid_blocks"])
        plan.destroy()
    items = res[""][0]
    diff = 0
    if diag:
        for x, y in zip(items, res["6"][0]):
            for f in ("dst", "codes", "scale", "zero", "esum"):
                tx, ty = getattr(x, f), getattr(y, f)
                if tx is not None:
                    diff += int((tx.view(torch.uint8) != ty.view(torch.uint8)).sum())
    mm = sweep_mismatches(items[:len(shapes)])
    out.append({"case": [model, copies, bits, sym, esum, pack], "variant": res[""][1], "grid_blocks": res[""][2],
                "diff_vs_v6": diff, "oracle_mismatches": mm["mismatches"], "tensors": mm["tensors"]})
print("RESULT " + json.dumps(out))
"""

EXPECTED = {("mobilenetv2", 1): 10, ("mobilenetv2", 2): 6, ("resnet50", 1): 6, ("deeplab", 1): 6}


@pytest.mark.parametrize("lib", ["product", "diag"])
def test_small_list_variant(lib):
    env = dict(os.environ, DFQ_ROOT=ROOT, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.pop("DFQ_SWEEP_VARIANT", None)
    if lib == "diag":
        env["DFQ_LIB"] = "diag"
    else:
        env.pop("DFQ_LIB", None)
    r = subprocess.run([sys.executable, "-c", _SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1][7:])
    print(json.dumps(res))
    for x in res:
        assert x["variant"] == EXPECTED[tuple(x["case"][:2])], x
        assert x["diff_vs_v6"] == 0 and x["oracle_mismatches"] == 0 and x["tensors"] > 0, x
