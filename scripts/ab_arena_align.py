"""Which property of the output placement slows the sweep's stores?  Same
weights and plan shape; only addresses differ.  Variants:
  <src>_<out>  src in {sep: one torch allocation per weight, arena: one packed
  input arena (4 KB)}, out in {sep: torch allocations per tensor (round 1),
  fields: one arena per output field (4 KB aligned tensors), onebuf<G>: one
  buffer with the field regions G MB apart}."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from data_free_quantization_amd.sweep import SweepItem, SweepPlan  # noqa: E402

A = 4096


def up(n, a=A):
    return -(-n // a) * a


def field_offsets(items, nbytes_of):
    offs, off = [], 0
    for it in items:
        offs.append(off)
        off += up(nbytes_of(it))
    return offs, off


FIELDS = [("dq", lambda it: 4 * it.src.numel(), torch.float32),
          ("codes", lambda it: it.src.numel(), torch.int8),
          ("esum", lambda it: 4 * it.esum.numel(), torch.float32),
          ("scale", lambda it: 4 * it.scale.numel(), torch.float32),
          ("zero", lambda it: 4 * it.zero.numel(), torch.float32)]


def out_views(items, how, dev, keep):
    per = {}
    if how == "fields":
        for name, nb, dt in FIELDS:
            offs, tot = field_offsets(items, nb)
            buf = torch.empty(tot, dtype=torch.uint8, device=dev)
            keep.append(buf)
            per[name] = [buf[o:o + nb(it)].view(dt) for o, it in zip(offs, items)]
    elif how.startswith("onebuf"):
        gap = int(how[6:]) << 20
        layout, base = [], 0
        for name, nb, dt in FIELDS:
            offs, tot = field_offsets(items, nb)
            layout.append((name, nb, dt, base, offs))
            base = up(base + tot, gap) if gap else up(base + tot)
        buf = torch.empty(base, dtype=torch.uint8, device=dev)
        keep.append(buf)
        for name, nb, dt, b0, offs in layout:
            per[name] = [buf[b0 + o:b0 + o + nb(it)].view(dt) for o, it in zip(offs, items)]
    return per


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    items, shapes, per_copy, copies = bench.build_batch("mobilenetv2", dev)
    keep = []
    offs, tot = field_offsets(items, lambda it: 4 * it.src.numel())
    inbuf = torch.empty(tot, dtype=torch.uint8, device=dev)
    src_arena = []
    for o, it in zip(offs, items):
        v = inbuf[o:o + 4 * it.src.numel()].view(torch.float32).view(it.src.shape)
        v.copy_(it.src)
        src_arena.append(v)
    plans = {"sep_sep": SweepPlan(items)}
    variants = sys.argv[1:] or ["arena_sep", "sep_fields", "arena_fields", "arena_onebuf0", "arena_onebuf1024",
                                "sep_onebuf0"]
    for v in variants:
        src_how, out_how = v.split("_", 1)
        if out_how == "sep":
            outs = {n: [getattr(it, "dst" if n == "dq" else n) for it in items] for n, _, _ in FIELDS}
        else:
            outs = out_views(items, out_how, dev, keep)
        srcs = src_arena if src_how == "arena" else [it.src for it in items]
        plans[v] = SweepPlan([SweepItem(src=srcs[i], dst=outs["dq"][i].view(it.src.shape),
                                        codes=outs["codes"][i].view(it.src.shape), scale=outs["scale"][i],
                                        zero=outs["zero"][i], esum=outs["esum"][i], bits=8, per_channel=True,
                                        symmetric=True, khw=it.khw, clip=(-15.0, 15.0), rows=it.rows)
                              for i, it in enumerate(items)])
    res = {k: [] for k in plans}
    for rep in range(3):
        for k, p in plans.items():
            res[k].append(round(bench.time_plan(p, stream, dev, 20, 3), 4))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
