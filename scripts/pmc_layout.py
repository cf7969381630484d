"""PMC probe of the placement sensitivity: three output layouts of the bench list
(scripts/ab_chunks.py: separate / fields / interC64) timed with HIP events, then
ONE more dispatch of each in that order at the end -- under rocprofv3 --pmc, the
last three sweep_main_kernel dispatches are those three."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import ab_chunks as A  # noqa: E402
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    items, shapes, per_copy, copies = bench.build_batch("mobilenetv2", dev)
    v, inar = A.carve([(i, 4 * it.src.numel(), A.A) for i, it in enumerate(items)], 0, dev)
    srcs = []
    for i, it in enumerate(items):
        t = v[i].view(torch.float32).view(it.src.shape)
        t.copy_(it.src)
        srcs.append(t)
    hows = ["separate", "fields", "interC64"]
    plans, keep = {}, []
    for h in hows:
        p, k = A.build(items, srcs, h, dev)
        plans[h] = p
        keep.append(k)
    res = {h: round(bench.time_plan(plans[h], stream, dev, 10, 2), 4) for h in hows}
    print(json.dumps(res), flush=True)
    for h in hows:
        plans[h].execute(stream)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
