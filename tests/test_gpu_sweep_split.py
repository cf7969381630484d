"""Sweep variant 16 (compute_task_split: whole-row tasks in two row batches, the
first quantized and stored while the second's loads land, LDS-DMA issued through
inline asm so only the explicit counted waits order the LDS reads) equals variant 6
bit for bit on every output field, and the C oracle, over the three bench families
and the INT4 / asymmetric / no-E forms (diagnostics library, fresh process)."""
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
out = []
CASES = [("mobilenetv2", 8, True, True, True, False), ("resnet50", 8, True, True, True, False),
         ("deeplab", 8, True, True, True, False), ("resnet50", 4, True, False, False, True),
         ("mobilenetv2", 8, True, False, False, False), ("mobilenetv2", 8, True, True, False, False)]
for model, bits, ch, sym, esum, pack in CASES:
    res = {}
    for v in ("6", "16"):
        os.environ["DFQ_SWEEP_VARIANT"] = v
        items, shapes, _, copies = bench.build_batch(model, dev, copies=2, bits=bits, channel=ch, sym=sym, esum=esum,
                                                     seed=77, pack=pack)
        plan = SweepPlan(items)
        plan.execute()
        torch.cuda.synchronize()
        res[v] = (items, plan.stats["variant"])
        plan.destroy()
    a, b = res["6"][0], res["16"][0]
    diff = 0
    for x, y in zip(a, b):
        for f in ("dst", "codes", "scale", "zero", "esum"):
            tx, ty = getattr(x, f), getattr(y, f)
            if tx is not None:
                diff += int((tx.view(torch.uint8) != ty.view(torch.uint8)).sum())
    mm = sweep_mismatches(b[:len(shapes)])
    out.append({"case": [model, bits, sym, esum, pack], "variants": [res["6"][1], res["16"][1]], "diff_vs_v6": diff,
                "oracle_mismatches": mm["mismatches"], "tensors": mm["tensors"]})
print("RESULT " + json.dumps(out))
"""


def test_split_variant_bit_identical():
    env = dict(os.environ, DFQ_ROOT=ROOT, DFQ_LIB="diag", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", _SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1][7:])
    print(json.dumps(res))
    for x in res:
        assert x["variants"] == [6, 16], x
        assert x["diff_vs_v6"] == 0 and x["oracle_mismatches"] == 0 and x["tensors"] > 0, x
