"""Robustness of output placement: several independent instantiations (fresh
allocations) of each layout on one box, device ms per step of the bench list.
  separate      torch allocation per tensor (round 1)
  fields        one arena per output field (4 KB aligned tensors)
  fieldsC<M>    per field, arenas of at most M MB (whole tensors per chunk)
  interC<M>     per-layer interleaved fields (dq, codes, E, scale, zero), chunks of M MB
  <layout>+shuf the same with DFQ_SWEEP_SHUFFLE=1 (workgroup quads in random order)
Inputs: one packed 4 KB arena (measured neutral)."""
import os
os.environ.setdefault("DFQ_LIB", "diag")   # A/B variants, switches and probes: libdfq_diag.so
import gc
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from data_free_quantization_amd.sweep import SweepItem, SweepPlan  # noqa: E402

A = 4096
F = [("dst", lambda it: 4 * it.src.numel(), torch.float32, A),
     ("codes", lambda it: it.src.numel(), torch.int8, A),
     ("esum", lambda it: 4 * it.esum.numel(), torch.float32, A),
     ("scale", lambda it: 4 * it.scale.numel(), torch.float32, 256),
     ("zero", lambda it: 4 * it.zero.numel(), torch.float32, 256)]


def up(n, a):
    return -(-n // a) * a


def carve(entries, chunk, dev):
    """entries: [(key, nbytes, align)] -> {key: uint8 view}, chunks <= chunk bytes."""
    out, plan, bufs, off = {}, [], [], 0
    for k, n, a in entries:
        o = up(off, a)
        if chunk and o + n > chunk and off > 0:
            bufs.append(off)
            o, off = 0, 0
        plan.append((k, len(bufs), o, n))
        off = o + n
    bufs.append(off)
    arenas = [torch.empty(max(b, 256), dtype=torch.uint8, device=dev) for b in bufs]
    for k, b, o, n in plan:
        out[k] = arenas[b][o:o + n]
    return out, arenas


def build(items, srcs, how, dev):
    import os
    keep = []
    if how.endswith("+shuf"):
        os.environ["DFQ_SWEEP_SHUFFLE"] = "1"
        how = how[:-5]
    else:
        os.environ.pop("DFQ_SWEEP_SHUFFLE", None)
    if how == "separate":
        outs = {(i, f): getattr(it, f) for i, it in enumerate(items) for f, *_ in F}
    else:
        outs = {}
        if how.startswith("fields"):
            chunk = int(how[7:]) << 20 if len(how) > 6 else 0
            for f, nb, dt, a in F:
                v, ar = carve([((i, f), nb(it), a) for i, it in enumerate(items)], chunk, dev)
                keep += ar
                outs.update({k: t.view(dt) for k, t in v.items()})
        else:
            chunk = int(how[6:]) << 20
            v, ar = carve([((i, f), nb(it), a) for i, it in enumerate(items) for f, nb, dt, a in F], chunk, dev)
            keep += ar
            dts = {f: dt for f, _, dt, _ in F}
            outs = {k: t.view(dts[k[1]]) for k, t in v.items()}
    plan = SweepPlan([SweepItem(src=srcs[i], dst=outs[(i, "dst")].view(it.src.shape),
                                codes=outs[(i, "codes")].view(it.src.shape), scale=outs[(i, "scale")],
                                zero=outs[(i, "zero")], esum=outs[(i, "esum")], bits=8, per_channel=True,
                                symmetric=True, khw=it.khw, clip=(-15.0, 15.0), rows=it.rows)
                      for i, it in enumerate(items)])
    return plan, keep


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    items, shapes, per_copy, copies = bench.build_batch("mobilenetv2", dev)
    v, inar = carve([(i, 4 * it.src.numel(), A) for i, it in enumerate(items)], 0, dev)
    srcs = []
    for i, it in enumerate(items):
        t = v[i].view(torch.float32).view(it.src.shape)
        t.copy_(it.src)
        srcs.append(t)
    hows = sys.argv[1:] or ["separate", "fields", "interC64", "separate+shuf", "fields+shuf", "interC64+shuf"]
    res = {h: [] for h in hows}
    for inst in range(3):
        for h in hows:
            plan, keep = build(items, srcs, h, dev)
            res[h].append(round(min(bench.time_plan(plan, stream, dev, 15, 3) for _ in range(2)), 4))
            plan.destroy()
            del plan, keep
            gc.collect()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()    # next instantiation gets fresh hipMallocs
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
