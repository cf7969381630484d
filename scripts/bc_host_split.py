"""Where the bias-correction stage's time goes (MobileNetV2 / ResNet-50, warm,
fused BC): the Python walk that records the chain vs the dfq_bc_chain calls
(_BcChain.flush, each followed by a device sync here), for the live walk and for
the compiled walk's replay (bias_correction._TEMPLATES): its structure
signature, the replay's host part (tables + the dfq_bc_chain call that enqueues
the launches) and the device tail after it.  (Timing only: the syncs inside the
stage add to its total.)"""
import contextlib
import io
import json
import logging
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("DFQ_LIB", "diag")
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
from data_free_quantization_amd import zoo, bias_correction as BC  # noqa: E402
from data_free_quantization_amd import pipeline  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
acc = {}
orig_flush = BC._BcChain.flush
orig_bc = pipeline.bias_correction


def flush(self, stream):
    t0 = time.perf_counter()
    try:
        return orig_flush(self, stream)
    finally:
        torch.cuda.synchronize()
        acc["flush"] = acc.get("flush", 0.0) + time.perf_counter() - t0


def bc(*a, **k):
    t0 = time.perf_counter()
    try:
        return orig_bc(*a, **k)
    finally:
        torch.cuda.synchronize()
        acc["stage"] = acc.get("stage", 0.0) + time.perf_counter() - t0


orig_replay = BC._WalkTemplate.replay
orig_structure = BC._structure


def replay(self, *a, **k):
    t0 = time.perf_counter()
    out = orig_replay(self, *a, **k)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    acc["replay_host"] = acc.get("replay_host", 0.0) + t1 - t0
    acc["replay_device_tail"] = acc.get("replay_device_tail", 0.0) + time.perf_counter() - t1
    return out


def structure(*a, **k):
    t0 = time.perf_counter()
    try:
        return orig_structure(*a, **k)
    finally:
        acc["structure"] = acc.get("structure", 0.0) + time.perf_counter() - t0


BC._BcChain.flush = flush
BC._WalkTemplate.replay = replay
BC._structure = structure
pipeline.bias_correction = bc
for model in (sys.argv[1:] or ["mobilenetv2", "resnet50"]):
    for mode in ("live", "replay"):   # live: the walk recorded each time; replay: the compiled walk
        res = []
        for rep in range(6):
            acc.clear()
            if mode == "live":
                BC._TEMPLATES.clear()
            m = zoo.build(model, seed=0, relu=True).cuda()
            g = build_graph(m, "positional")
            with contextlib.redirect_stdout(io.StringIO()):
                pipeline.run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel",
                                 symmetric=True, bc_mode="fused", timings={})
            if rep:
                res.append((acc["stage"] * 1e3, acc.get("flush", 0.0) * 1e3, acc.get("structure", 0.0) * 1e3,
                            acc.get("replay_host", 0.0) * 1e3, acc.get("replay_device_tail", 0.0) * 1e3))
        res.sort()
        st, fl, sg, rh, rd = res[len(res) // 2]
        print(json.dumps({"model": model, "mode": mode, "stage_ms": round(st, 3), "flush_ms": round(fl, 3),
                          "walk_ms": round(st - fl, 3), "structure_ms": round(sg, 3),
                          "replay_host_ms": round(rh, 3), "replay_device_tail_ms": round(rd, 3)}), flush=True)
