"""Multi-GPU DFQ sweep: the model's layer list sharded across ranks.

The reference has no multi-GPU DFQ code (its whole DFQ path is CPU,
``/root/reference/main_dfq.py:145``; its only collective is SyncBN,
``modeling/segmentation/sync_batchnorm/batchnorm.py:102,105``, unused on the DFQ
path).  north_star asks for the layer-sharded sweep with a trivial RCCL
broadcast/gather, so this module is designed for that and nothing else.

Layers are independent for quantize / clip / bias-correction error sums.  Each
rank sweeps its longest-processing-time share of the layer list with ONE grouped
launch.  Memory is laid out for the collective (``ShardLayout``): every rank's
share is one contiguous *slab* of the input arena (fp32 weights) and of each
output field's arena (dq, codes, scale, zero, E), slabs in rank order at a fixed
stride, so

* the sweep writes its outputs straight into the slabs that are sent (no pack);
* ``scatter()``   -- rank 0 holds every weight; one send per rank of that rank's
  slab (grouped send/recv; ``broadcast()`` sends the whole arena instead);
* ``gather("root")`` -- per rank one grouped receive of its slabs, straight into
  rank 0's arenas (only rank 0 allocates full arenas);
* ``gather("all")``  -- one in-place ``all_gather_into_tensor`` per field.

One process per GPU (torchrun), RCCL over xGMI (backend "nccl").  The gloo backend
is supported for the CPU tests and for rehearsing N ranks on one GPU; it stages
device tensors through host memory (gloo has no device send/recv), which only a
rehearsal ever pays.

The per-rank compute is injectable (``compute=``) so the CPU tests can run the
layout and collectives with the oracle as the checker; the product compute is the
HIP sweep (``SweepPlan`` over arena views).
"""
from __future__ import annotations

import heapq
import math
import random
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

FIELDS = ("dq", "codes", "scale", "zero", "esum")
# Arena layout (measured on MI355X, scripts/ab_arena*.py, profiles/r02/ab_arena.md):
# the sweep's store streams lose 7-22 % when its output fields (dq, codes, E) share
# ONE allocation -- per-layer interleaved at any alignment from 256 B to 16 KB, or
# as field regions back to back, 2 MB / 32 MB / 1 GB aligned, or staggered -- and
# when a field's tensors are packed at 256 B or 64 KB.  One allocation per field,
# tensors at 4 KB, matches separate per-tensor allocations (1.09 ms vs 1.16-1.33
# per step on the bench list).  So each output field has its own arena.
#
# ARENA_ORDER.  Even then, placement decides: over five physical placements on one
# box (scripts/ab_shift.py) per-field arenas ran 1.08 or 1.31 ms (bimodal) while
# round-1 per-tensor torch allocations stayed at 1.09-1.14.  The sweep writes a
# task's dq, codes and E at the same time; in arenas that share the layer order
# those streams sit at a FIXED distance from each other for the whole launch, which
# a given placement either tolerates or turns into a systematic conflict.  So each
# field's arena holds the layers in its own seeded order: the distance between a
# task's streams varies from layer to layer, as it does between separate
# allocations, and no placement can line them all up.
ALIGN = 4096                       # dq / codes / E / weight tensors inside their arena
SMALL_ALIGN = 256                  # scale / zero
SHUFFLE_FIELDS = True              # ARENA_ORDER: per-field seeded layer order


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
    """Outputs of one layer's sweep (views into an output arena)."""
    dq: torch.Tensor
    codes: Optional[torch.Tensor]
    scale: torch.Tensor
    zero: torch.Tensor
    esum: Optional[torch.Tensor] = None


@dataclass(frozen=True)
class LayerSpec:
    """How one fp32 tensor is quantized (the SweepItem options, minus pointers)."""
    shape: tuple
    bits: int = 8
    per_channel: bool = True
    symmetric: bool = True
    want_codes: bool = True
    want_esum: bool = False
    clip: Optional[tuple] = None
    pack_int4: bool = False

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))

    @property
    def khw(self) -> int:
        """Spatial size KH*KW of a KCRS conv weight (1 for Linear / vectors)."""
        return int(math.prod(self.shape[2:])) if len(self.shape) >= 3 else 1

    @property
    def rows(self) -> int:
        return int(self.shape[0]) if (self.per_channel and len(self.shape) > 0) else 1

    def outputs(self) -> Dict[str, tuple]:
        """field -> (shape, dtype) of the sweep outputs of this tensor."""
        out = {"dq": (tuple(self.shape), torch.float32)}
        if self.want_codes:
            if self.pack_int4:
                out["codes"] = (((self.numel + 1) // 2,), torch.uint8)
            else:
                out["codes"] = (tuple(self.shape), code_dtype(self.bits, self.symmetric))
        out["scale"] = ((self.rows,), torch.float32)
        out["zero"] = ((self.rows,), torch.float32)
        if self.want_esum:
            out["esum"] = ((self.numel // self.khw,), torch.float32)
        return out


def code_dtype(bits: int, symmetric: bool) -> torch.dtype:
    if bits <= 8:
        return torch.int8 if symmetric else torch.uint8
    return torch.int16


def _nbytes(shape, dtype) -> int:
    return int(math.prod(shape)) * torch.empty(0, dtype=dtype).element_size()


def _up(n: int, a: int) -> int:
    return -(-n // a) * a


class ShardLayout:
    """Where every layer's input and outputs live.  Rank r owns ``parts[r]``.
    There is one arena for the fp32 inputs and one per output field (dq, codes,
    scale, zero, E); in each, rank r's tensors form slab r (back to back, each
    at a 4 KB aligned offset -- 256 B for scale / zero).  Slabs sit at a fixed
    stride ``cap[f]`` (the largest rank's slab, 4 KB aligned), so an arena is
    ``world`` equal slots -- the shape all_gather_into_tensor wants -- and
    ``used[f][r]`` is what a point-to-point transfer of that slab moves."""

    def __init__(self, specs: Sequence[LayerSpec], world: int):
        self.specs = list(specs)
        self.world = world
        # LPT over the bytes a layer moves (read 4 B + its outputs)
        outs = [s.outputs() for s in self.specs]
        work = [4 * s.numel + sum(_nbytes(*v) for v in o.values()) for s, o in zip(self.specs, outs)]
        self.parts = partition(work, world)
        n = len(self.specs)
        self.owner = [0] * n
        self.off: List[Dict[str, int]] = [dict() for _ in range(n)]   # field ("w" = input) -> byte offset
        self.fields = ["w"] + [f for f in FIELDS if any(f in o for o in outs)]
        self.used = {f: [0] * world for f in self.fields}
        for r, p in enumerate(self.parts):
            for i in p:
                self.owner[i] = r
            for j, f in enumerate(self.fields):
                # each field's arena holds the rank's layers in its own seeded order
                # (see ARENA_ORDER above); the order is a pure function of (layout,
                # field), identical on every rank
                order = list(p)
                if SHUFFLE_FIELDS and j > 0:
                    random.Random(0x5EED + 7919 * j + r).shuffle(order)
                cur = 0
                for i in order:
                    sz = (self.specs[i].shape, torch.float32) if f == "w" else outs[i].get(f)
                    if sz is None:
                        continue
                    self.off[i][f] = cur
                    cur += _up(_nbytes(*sz), SMALL_ALIGN if f in ("scale", "zero") else ALIGN)
                self.used[f][r] = cur
        self.cap = {f: _up(max(max(self.used[f]), 1), ALIGN) for f in self.fields}

    def nbytes(self, i: int, f: str) -> int:
        if f == "w":
            return 4 * self.specs[i].numel
        return _nbytes(*self.specs[i].outputs()[f])


def _backend(group=None) -> Optional[str]:
    return dist.get_backend(group) if dist.is_initialized() else None


class ShardedSweep:
    """The layer-sharded DFQ sweep of one layer list over the process group.

    ``sources``: the fp32 input tensors, replicated on every rank (main_dfq's
    case: every rank holds the model); the input arena is then not used.
    Without ``sources`` the weights live in the input arena: rank 0 holds all of
    them (``replicate=False``) or every rank does (``replicate=True``); fill them
    with ``weight(i).copy_(...)`` and distribute with ``scatter()`` /
    ``broadcast()``.  The output arenas are full-size on rank 0 (and on every
    rank with ``replicate=True``, needed for ``gather("all")``), one slab
    elsewhere.

    ``run()`` sweeps this rank's share into its output slabs (one HIP launch, or
    two when a per-tensor range is needed); ``gather()`` collects the slabs.
    """

    def __init__(self, specs: Sequence[LayerSpec], *, sources: Optional[Sequence[torch.Tensor]] = None,
                 replicate: bool = False, device=None, group=None,
                 compute: Optional[Callable[["ShardedSweep", List[int]], None]] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.layout = ShardLayout(specs, self.world)
        self.specs = self.layout.specs
        self.sources = list(sources) if sources is not None else None
        if self.sources is not None:
            if len(self.sources) != len(self.specs):
                raise ValueError("one source tensor per layer spec")
            for t, s in zip(self.sources, self.specs):
                if tuple(t.shape) != tuple(s.shape):
                    raise ValueError(f"source shape {tuple(t.shape)} != spec shape {s.shape}")
            device = self.sources[0].device if self.sources else device
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.full = replicate or self.rank == 0
        self.replicate = replicate
        L = self.layout
        slots = self.world if self.full else 1
        self.arenas: Dict[str, torch.Tensor] = {}
        for f in L.fields:
            if f == "w" and self.sources is not None:
                continue
            self.arenas[f] = torch.empty(slots * L.cap[f], dtype=torch.uint8, device=self.device)
        self.mine = L.parts[self.rank]
        self._compute = compute
        self._plan = None

    @property
    def in_arena(self) -> Optional[torch.Tensor]:
        return self.arenas.get("w")

    # ---- views -------------------------------------------------------------------
    def _slot(self, f: str, r: int) -> torch.Tensor:
        arena, cap = self.arenas[f], self.layout.cap[f]
        if arena.numel() == cap * self.world:
            return arena[r * cap:(r + 1) * cap]
        if r != self.rank:
            raise KeyError(f"rank {self.rank} does not hold slab {r}")
        return arena[:cap]

    def _view(self, i: int, f: str, shape, dtype) -> torch.Tensor:
        off = self.layout.off[i][f]
        slab = self._slot(f, self.layout.owner[i])
        return slab[off:off + self.layout.nbytes(i, f)].view(dtype).view(shape)

    def holds(self, i: int) -> bool:
        return self.full or self.layout.owner[i] == self.rank

    def weight(self, i: int) -> torch.Tensor:
        """Layer i's fp32 input (a view into the input arena, or the source)."""
        if self.sources is not None:
            return self.sources[i]
        return self._view(i, "w", self.specs[i].shape, torch.float32)

    def outputs(self, i: int) -> LayerOut:
        vals = {f: None for f in FIELDS}
        for f, (shp, dt) in self.specs[i].outputs().items():
            vals[f] = self._view(i, f, shp, dt)
        return LayerOut(**vals)

    # ---- compute -----------------------------------------------------------------
    def _gpu_plan(self):
        from .sweep import SweepItem, SweepPlan
        items = []
        for i in self.mine:
            s, o = self.specs[i], self.outputs(i)
            items.append(SweepItem(src=self.weight(i), dst=o.dq, codes=o.codes, scale=o.scale, zero=o.zero,
                                   esum=o.esum, bits=s.bits, per_channel=s.per_channel, symmetric=s.symmetric,
                                   khw=s.khw, clip=s.clip, rows=s.rows, pack_int4=s.pack_int4))
        return SweepPlan(items) if items else None

    def run(self, stream: Optional[torch.cuda.Stream] = None):
        """Sweep this rank's share into its output slab (asynchronous on ``stream``)."""
        if self._compute is not None:
            self._compute(self, self.mine)
            return
        if self._plan is None:
            self._plan = self._gpu_plan()
        if self._plan is not None:
            self._plan.execute(stream)
            self._run_stream = stream

    def _await_run(self):
        """Collectives are ordered against the current stream only: make it wait for
        a sweep that run() enqueued on another stream before sending its outputs."""
        s = getattr(self, "_run_stream", None)
        if s is not None and self.device.type == "cuda":
            cur = torch.cuda.current_stream(self.device)
            if s != cur:
                cur.wait_stream(s)

    @property
    def plan_stats(self) -> Optional[Dict]:
        if self._plan is None and self._compute is None:
            self._plan = self._gpu_plan()
        return self._plan.stats if self._plan is not None else None

    # ---- collectives -------------------------------------------------------------
    def _staged(self) -> bool:
        """gloo has no device-side send/recv: stage device tensors through the host."""
        return _backend(self.group) == "gloo" and self.device.type == "cuda"

    def _p2p(self, sends, recvs):
        """Grouped point-to-point: ``sends``/``recvs`` = [(tensor, peer)]."""
        if not sends and not recvs:
            return
        if self._staged():
            hrecv = [(torch.empty(t.shape, dtype=t.dtype), t, p) for t, p in recvs]
            for t, p in sends:
                dist.send(t.cpu(), p, group=self.group)
            for h, t, p in hrecv:
                dist.recv(h, p, group=self.group)
                t.copy_(h)
            return
        ops = [dist.P2POp(dist.isend, t, p, self.group) for t, p in sends]
        ops += [dist.P2POp(dist.irecv, t, p, self.group) for t, p in recvs]
        for w in dist.batch_isend_irecv(ops):
            w.wait()

    def _out_fields(self):
        return [f for f in self.layout.fields if f != "w"]

    def scatter(self):
        """Rank 0 -> every rank: its slab of the input arena (one transfer per rank)."""
        if self.sources is not None:
            raise RuntimeError("scatter() needs the input arena (no sources=)")
        if self.world == 1:
            return
        used = self.layout.used["w"]
        if self.rank == 0:
            self._p2p([(self._slot("w", r)[:used[r]], r) for r in range(1, self.world) if used[r]], [])
        elif used[self.rank]:
            self._p2p([], [(self._slot("w", self.rank)[:used[self.rank]], 0)])

    def broadcast(self):
        """Rank 0 -> every rank: the whole input arena (needs ``replicate=True``)."""
        if self.sources is not None or not self.replicate:
            raise RuntimeError("broadcast() needs a replicated input arena")
        if not dist.is_initialized():
            return
        a = self.arenas["w"]
        if self._staged():
            h = a.cpu()
            dist.broadcast(h, 0, group=self.group)
            a.copy_(h)
        else:
            dist.broadcast(a, 0, group=self.group)

    def gather(self, to: str = "root"):
        """Collect every rank's output slabs: ``to="root"`` into rank 0's arenas
        (one grouped receive per rank and field, exact sizes); ``to="all"`` into
        every rank's arenas (one in-place all_gather_into_tensor per field; needs
        ``replicate=True``).  Runs the collective even at world size 1 so the RCCL
        path is exercised."""
        if not dist.is_initialized():
            return
        self._await_run()
        L = self.layout
        if to == "all":
            if not self.replicate:
                raise RuntimeError('gather("all") needs replicate=True (full output arenas on every rank)')
            for f in self._out_fields():
                arena, own = self.arenas[f], self._slot(f, self.rank)
                if _backend(self.group) == "gloo":
                    # gloo: list form on host tensors (CPU tests, one-GPU rehearsal)
                    host = arena.cpu() if self.device.type == "cuda" else arena
                    dist.all_gather(list(host.view(self.world, L.cap[f]).unbind(0)), own.cpu().clone(),
                                    group=self.group)
                    if host is not arena:
                        arena.copy_(host)
                else:
                    dist.all_gather_into_tensor(arena, own, group=self.group)
        elif to == "root":
            if self.world == 1:
                return
            if self.rank == 0:
                self._p2p([], [(self._slot(f, r)[:L.used[f][r]], r) for r in range(1, self.world)
                               for f in self._out_fields() if L.used[f][r]])
            else:
                self._p2p([(self._slot(f, self.rank)[:L.used[f][self.rank]], 0) for f in self._out_fields()
                           if L.used[f][self.rank]], [])
        else:
            raise ValueError('to must be "root" or "all"')

    def result(self) -> Dict[int, LayerOut]:
        """Every layer whose outputs this rank holds (after ``gather``: all on rank 0)."""
        return {i: self.outputs(i) for i in range(len(self.specs)) if self.holds(i)}

    def destroy(self):
        if self._plan is not None:
            self._plan.destroy()
            self._plan = None


def uniform_specs(shapes: Sequence[tuple], **cfg) -> List[LayerSpec]:
    return [LayerSpec(shape=tuple(s), **cfg) for s in shapes]


def max_over_ranks(value: float, device=None, group=None) -> float:
    """Max of a per-rank float over the group (bench.py's step time); identity
    when torch.distributed is not initialised."""
    if not dist.is_initialized():
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def init_from_env(backend: Optional[str] = None):
    """torchrun's RANK / WORLD_SIZE / LOCAL_RANK -> (world, rank, device); one
    process per GPU over RCCL ("nccl"), or gloo (CPU / one-GPU rehearsal:
    ranks share the visible cards round-robin).  Identity at WORLD_SIZE=1."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1:
        dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        return world, rank, dev
    backend = backend or os.environ.get("DFQ_DIST_BACKEND", "nccl")
    if torch.cuda.is_available():
        local = local % torch.cuda.device_count() if backend == "gloo" else local
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return world, rank, dev
