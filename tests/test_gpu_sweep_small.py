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


def test_small_list_falls_back_when_the_small_tasks_cannot_hold_it():
    """A small list holding a tensor whose KH*KW (40 x 40 = 1,600) exceeds the small
    tasks' 1,536 elements: the 1,536 table cannot be built, so the plan keeps the
    2,048-element tasks (variant 6), and the result matches the oracle."""
    import numpy as np
    import torch
    from oracle import oracle as O
    from data_free_quantization_amd.sweep import SweepPlan, allocate, khw_of
    rng = np.random.default_rng(3)
    shapes = [(2, 1, 40, 40), (16, 8, 3, 3), (5, 7)]
    items, xs = [], []
    for shp in shapes:
        x = rng.normal(0, 1, shp).astype(np.float32)
        t = torch.from_numpy(x).to("cuda:0")
        xs.append(x)
        items.append(allocate(t, bits=8, per_channel=True, symmetric=True, khw=khw_of(t), want_esum=True))
    plan = SweepPlan(items)
    assert plan.stats["variant"] == 6, plan.stats
    plan.execute()
    torch.cuda.synchronize()
    for x, it in zip(xs, items):
        o = O.quantize(x, 8, 3, rows=x.shape[0], khw=it.khw, want_esum=True)
        assert np.array_equal(it.dst.cpu().numpy(), o["dq"]), x.shape
        assert np.array_equal(it.codes.cpu().numpy().view(o["codes"].dtype), o["codes"]), x.shape
        assert np.array_equal(it.esum.cpu().numpy(), o["esum"]), x.shape
    plan.destroy()
