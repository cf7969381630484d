"""Which earlier bench leg lowers the in-bench ResNet-50 x22 figure (diagnostic,
GPU)?  One process: the R50 secondary config timed fresh, then after each of the
bench's earlier legs in turn -- the headline MobileNetV2 x155 list kept alive (as
bench.py keeps it for the parity check), the pipeline legs, the same-mix probe --
each time on newly allocated R50 tensors.  Prints one JSON line."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402

dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)


def r50():
    items, _, _, _ = bench.build_batch("resnet50", dev, bits=8, channel=True, sym=True, esum=True, seed=99)
    plan = SweepPlan(items)
    ms = bench.time_plan(plan, s, dev, 20, 3)
    f = round(plan.stats["algo_bytes"] / ms / 1e6 / bench.HBM_PEAK_GBS, 4)
    plan.destroy()
    del items, plan
    torch.cuda.empty_cache()
    return f


out = {"fresh": r50()}
head, _, per_copy, copies = bench.build_batch("mobilenetv2", dev)   # the headline list, kept alive
hp = SweepPlan(head)
bench.time_plan(hp, s, dev, 5, 2)
out["headline_alive"] = r50()
out["pipeline_timing"] = (bench.pipeline_timing(dev, "mobilenetv2"), bench.pipeline_timing(dev, "resnet50"))[0]["total"]
out["after_pipeline"] = r50()
bench.same_mix_probe(per_copy * copies, dev, s)
out["after_probe"] = r50()
hp.destroy()
del head, hp
torch.cuda.empty_cache()
out["headline_freed"] = r50()
print(json.dumps(out), flush=True)
