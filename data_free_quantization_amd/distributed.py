"""Multi-GPU DFQ sweep: shard a model's layer list across ranks.

Layers are independent for quantize / clip / bias-correction error sums, so each
rank sweeps only its share (longest-processing-time greedy over layer bytes) with
no communication, then one packed ``all_gather_into_tensor`` (RCCL over xGMI on
MI355X; gloo in the CPU tests) leaves every rank -- or only rank 0 -- with all
layers' outputs.  One process per GPU (torchrun); ``bench.py --gpus N`` uses the
communication-free form (independent weight sets per rank, weak scaling).

The per-rank compute is a callable so the partition/pack/gather logic can be
tested on CPU with the oracle; the product passes ``gpu_sweep``.
"""
from __future__ import annotations

import heapq
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist


def partition(sizes: Sequence[int], world: int) -> List[List[int]]:
    """LPT greedy: biggest layer first onto the least-loaded rank.  Returns
    per-rank lists of layer indices (each list in ascending layer order);
    deterministic for ties (lower rank wins)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    heap = [(0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda k: (-sizes[k], k)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + int(sizes[i]), r))
    return [sorted(x) for x in out]


@dataclass
class LayerOut:
    """Outputs of one layer's sweep (all on the layer's device)."""
    dq: torch.Tensor
    codes: torch.Tensor
    scale: torch.Tensor
    zero: torch.Tensor
    esum: Optional[torch.Tensor] = None


def _layout(spec: Dict) -> List[tuple]:
    """(field, shape, dtype, nbytes) of one layer's outputs, padded to 16 B."""
    fields = []
    for name in ("dq", "codes", "scale", "zero", "esum"):
        shp, dt = spec.get(name, (None, None))
        if shp is None:
            continue
        nb = int(torch.Size(shp).numel()) * torch.empty(0, dtype=dt).element_size()
        fields.append((name, tuple(shp), dt, (nb + 15) // 16 * 16))
    return fields


def output_spec(weight: torch.Tensor, per_channel: bool, bits: int, symmetric: bool, khw: int,
                want_esum: bool, pack_int4: bool = False) -> Dict:
    rows = weight.shape[0] if per_channel else 1
    cdt = (torch.int8 if symmetric else torch.uint8) if bits <= 8 else torch.int16
    cshape = ((weight.numel() + 1) // 2,) if pack_int4 else tuple(weight.shape)
    spec = {"dq": (tuple(weight.shape), torch.float32), "codes": (cshape, torch.uint8 if pack_int4 else cdt),
            "scale": ((rows,), torch.float32), "zero": ((rows,), torch.float32)}
    if want_esum:
        spec["esum"] = ((weight.numel() // khw,), torch.float32)
    return spec


def _pack(outs: List[LayerOut], specs: List[Dict], device, cap: int = 0) -> torch.Tensor:
    """All fields of all layers, each at a 16-B aligned offset, in ONE byte buffer
    of max(cap, 16) bytes, written by a single concatenation kernel.  Padding and
    the tail are never read (``_unpack`` reads each field's own bytes), so they are
    left uninitialised."""
    parts = []
    total = 0
    for o, s in zip(outs, specs):
        for name, shp, dt, nb in _layout(s):
            raw = getattr(o, name).contiguous().view(-1).view(torch.uint8)
            parts.append(raw)
            if nb > raw.numel():
                parts.append(torch.empty(nb - raw.numel(), dtype=torch.uint8, device=device))
            total += nb
    buf = torch.empty(max(cap, total, 16), dtype=torch.uint8, device=device)
    if parts:
        torch.cat(parts, out=buf[:total])
    return buf


def _unpack(buf: torch.Tensor, specs: List[Dict]) -> List[LayerOut]:
    """Views into ``buf`` (no copies): the gathered layers alias the receive buffer."""
    outs, off = [], 0
    for s in specs:
        vals = {}
        for name, shp, dt, nb in _layout(s):
            n = int(torch.Size(shp).numel()) * torch.empty(0, dtype=dt).element_size()
            vals[name] = buf[off:off + n].view(dt).view(shp)
            off += nb
        outs.append(LayerOut(**vals))
    return outs


def sharded_sweep(weights: Sequence[torch.Tensor], compute: Callable[[List[int]], List[LayerOut]],
                  specs: Sequence[Dict], gather: str = "all", group=None) -> Dict[int, LayerOut]:
    """Sweep ``weights`` (replicated on every rank) with each rank computing only
    its LPT share via ``compute(indices) -> [LayerOut]``, then gather.

    gather="all": every rank returns all layers; "rank0": only rank 0 does;
    "none": each rank returns its own share (outputs stay sharded)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    sizes = [w.numel() for w in weights]
    parts = partition(sizes, world)
    mine = parts[rank]
    local = compute(mine)
    result = {i: o for i, o in zip(mine, local)}
    if world == 1 or gather == "none":
        return result
    dev = weights[0].device
    sizes_b = [sum(nb for i in p for (_, _, _, nb) in _layout(specs[i])) for p in parts]
    cap = max(max(sizes_b), 16)
    send = _pack(local, [specs[i] for i in mine], dev, cap)
    recv = torch.empty(cap * world, dtype=torch.uint8, device=dev)
    if gather == "rank0" and dist.get_backend(group) == "gloo":
        gl = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
        dist.gather(send, gl, dst=0, group=group)
        if rank != 0:
            return result
        recv = torch.cat(gl)
    else:
        if dist.get_backend(group) == "gloo":      # gloo: list form (CPU or CUDA tensors)
            dist.all_gather(list(recv.view(world, cap).unbind(0)), send, group=group)
        else:                                     # RCCL: one packed all-gather over xGMI
            dist.all_gather_into_tensor(recv, send, group=group)
        if gather == "rank0" and rank != 0:
            return result
    for r, p in enumerate(parts):
        if not p or r == rank:
            continue
        outs = _unpack(recv[r * cap:(r + 1) * cap], [specs[i] for i in p])
        result.update({i: o for i, o in zip(p, outs)})
    return result


def max_over_ranks(value: float, device=None, group=None) -> float:
    """Max of a per-rank float over the group (bench.py's step time); identity
    when torch.distributed is not initialised."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def gpu_sweep(weights: Sequence[torch.Tensor], bits=8, per_channel=True, symmetric=True, want_esum=True,
              clip=None, reuse: bool = False, pack_int4: bool = False) -> Callable[[List[int]], List[LayerOut]]:
    """The product compute for ``sharded_sweep``: one grouped HIP sweep over the
    rank's layers (SweepPlan).  ``reuse``: keep the plan and its output buffers
    for the next call with the same layers (repeated passes overwrite them)."""
    from .sweep import SweepPlan, allocate, khw_of
    cache: Dict[tuple, tuple] = {}

    def run(indices: List[int]) -> List[LayerOut]:
        key = tuple(indices)
        if reuse and key in cache:
            plan, items = cache[key]
        else:
            items = [allocate(weights[i], bits=bits, per_channel=per_channel, symmetric=symmetric,
                              khw=khw_of(weights[i]), want_esum=want_esum, clip=clip, pack_int4=pack_int4)
                     for i in indices]
            plan = SweepPlan(items) if items else None
            if reuse:
                cache[key] = (plan, items)
        if plan is not None:
            plan.execute()
            if not reuse:
                plan.destroy()
        return [LayerOut(it.dst, it.codes, it.scale, it.zero, it.esum) for it in items]

    return run
