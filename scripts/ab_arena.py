"""A/B on one box: the bench's layer list swept from separate torch allocations
(round-1 layout) vs from distributed.ShardedSweep's arenas (one per field) at
tensor alignments given on the command line (distributed.ALIGN).  Same weights; interleaved runs; device ms per
step (HIP events)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from data_free_quantization_amd import distributed as D  # noqa: E402
from data_free_quantization_amd.sweep import SweepPlan  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    items, shapes, per_copy, copies = bench.build_batch("mobilenetv2", dev)
    plans = {"separate": SweepPlan(items)}
    it0 = items[0]
    print(json.dumps({"separate_ptrs_item0": [hex(t.data_ptr()) for t in (it0.src, it0.dst, it0.codes, it0.scale,
                                                                            it0.zero, it0.esum)],
                      "separate_ptrs_item1": [hex(t.data_ptr()) for t in (items[1].src, items[1].dst,
                                                                            items[1].codes, items[1].esum)],
                      "separate_ptrs_item100": [hex(t.data_ptr()) for t in (items[100].src, items[100].dst,
                                                                              items[100].codes, items[100].esum)]}))
    keep = []
    for cfg in (sys.argv[1:] or ["4096:256"]):
        align, small = (int(x) for x in cfg.split(":"))
        D.ALIGN, D.SMALL_ALIGN = align, small
        specs = D.uniform_specs(shapes * copies, bits=8, per_channel=True, symmetric=True, want_esum=True,
                                clip=(-15.0, 15.0))
        sw = D.ShardedSweep(specs, device=dev)
        for i, it in enumerate(items):
            sw.weight(i).copy_(it.src)
        sw.run(stream)
        plans[f"sharded_a{align}_s{small}"] = sw._plan
        keep.append(sw)
    res = {k: [] for k in plans}
    for rep in range(3):
        for k, p in plans.items():
            res[k].append(round(bench.time_plan(p, stream, dev, 20, 3), 4))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
