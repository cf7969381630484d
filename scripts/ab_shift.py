"""Placement robustness on one box: the bench list in (a) round-1 separate torch
allocations (per layer: src, dst, codes, scale, zero, E) and (b) ShardedSweep's
per-field arenas, each instantiated several times behind a different-size
"shift" allocation so the physical placement moves.  Device ms per step."""
import gc
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
    shapes = bench.model_shapes("mobilenetv2")
    per_copy = sum(int(torch.Size(s).numel()) for s in shapes)
    copies = -(-(2 << 30) // (4 * per_copy))
    res = {"separate": [], "arenas": [], "arenas_shuffled": []}
    for j, shift_mb in enumerate([0, 37, 260, 1029, 3001]):
        for how in ("separate", "arenas", "arenas_shuffled"):
            D.SHUFFLE_FIELDS = how == "arenas_shuffled"
            shift = torch.empty((shift_mb << 20) + 4096 * (j + 1), dtype=torch.uint8, device=dev)
            if how == "separate":
                items, _, _, _ = bench.build_batch("mobilenetv2", dev, copies=copies)
                plan = SweepPlan(items)
                keep = items
            else:
                specs = D.uniform_specs(shapes * copies, bits=8, per_channel=True, symmetric=True, want_esum=True,
                                        clip=(-15.0, 15.0))
                sw = D.ShardedSweep(specs, device=dev)
                gen = torch.Generator(device=dev).manual_seed(1234)
                for i, s in enumerate(specs):
                    std = (2.0 / (s.shape[2] * s.shape[3] * s.shape[0])) ** 0.5 if len(s.shape) == 4 else 0.01
                    sw.weight(i).normal_(0.0, std, generator=gen)
                sw.run(stream)
                plan, keep = sw._plan, sw
            res[how].append(round(min(bench.time_plan(plan, stream, dev, 10, 2) for _ in range(2)), 4))
            plan.destroy()
            del plan, keep, shift
            gc.collect()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
