"""Benchmark: the per-channel INT8 DFQ weight sweep on MI355X.

One STEP = one pass of the fused DFQ sweep (per-channel symmetric INT8
quantize-dequantize + integer codes + clip_weight + bias-correction error sums
E[o,i]) over ONE layer list: ``--copies`` MobileNetV2 weight sets back to back
(BASELINE.json configs[1]; synthetic random-init weights of the reference's
shapes, already resident in HBM).  The list defeats the 256 MB Infinity Cache
(SURVEY.md 8d), so the number is an HBM number.

At N GPUs the SAME list is LPT-sharded over the ranks by algorithmic bytes
(distributed.ShardLayout): each rank materialises only its own
layers and the timed step is its sweep with the outputs left sharded (strong
scaling); ``value`` is the whole list's weight bytes over the max-over-ranks
step.  Beside it: ``sharded_gathers`` (the same list in the sharded sweep's slab
arenas: sweep, sweep + gather to rank 0, sweep + in-place all-gather),
``weak_scaling`` (every rank its own whole list) and BASELINE configs[4]
(``configs4_sharded``: ONE ResNet-50 INT4 + clip list of >= 2 GiB held by rank 0,
scattered, swept and gathered, with its oracle parity counts).

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N     (one process per GPU, RCCL)

``python bench.py --gpus N`` with N > 1 and no torchrun environment starts
torchrun as a CHILD process (``--nproc-per-node N``, 127.0.0.1) before anything
touches the GPU, passes rank 0's JSON line through and exits with torchrun's
exit status.  Every rank checks that the process group has exactly N ranks.

Rank 0 prints ONE JSON line (contract in the task statement); ``roofline``
times the sweep kernel with HIP events on the stream it is launched on;
``cpu_baseline`` times the reference's torch CPU ops as restated in
oracle/torch_port.py (all host threads; the 1-thread C oracle beside it) on a
bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "weight-GB/s quantized (per-ch INT8 DFQ sweep) + top-1 delta, MobileNetV2"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--model", default="mobilenetv2", choices=["mobilenetv2", "resnet50", "deeplab"])
    p.add_argument("--copies", type=int, default=0, help="weight sets in the layer list (0: enough for >= 2 GiB)")
    p.add_argument("--bits", type=int, default=8)
    p.add_argument("--granularity", default="channel", choices=["channel", "tensor"])
    p.add_argument("--asym", action="store_true", help="asymmetric (reference default) instead of symmetric")
    p.add_argument("--no-esum", action="store_true", help="skip the bias-correction error sums")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (0 = skip)")
    p.add_argument("--no-pipeline", action="store_true", help="skip the one-off full-DFQ pipeline timing")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the other BASELINE configs (ResNet-50, DeepLab, INT4, per-tensor; sharded single model)")
    p.add_argument("--layout", default="tensor", choices=["tensor", "arena"],
                   help="N=1 tensor placement: one allocation per tensor, or the sharded path's per-field arenas")
    p.add_argument("--no-parity", action="store_true",
                   help="skip the parity checks of the timed outputs (vs the C oracle) and of the MobileNetV2 "
                        "pipeline (vs the reference fixture)")
    p.add_argument("--prewarm-ms", type=float, default=600.0,
                   help="time-based pre-warm (ms of sweep steps) before the counted warm-up: a fresh lease starts "
                        "at idle clocks (0 = none)")
    p.add_argument("--traffic-json", default=str(ROOT / "profiles" / "traffic_r06.json"),
                   help="the committed rocprofv3 summary of this bench command (scripts/profile.sh + "
                        "scripts/summarize_profile.py): PMC traffic and the kernel's rocprof average")
    p.add_argument("--no-sharded", action="store_true",
                   help="N > 1: skip configs4_sharded (the ResNet-50 INT4 list sharded from rank 0)")
    p.add_argument("--probe-ranks", action="store_true",
                   help="launcher check: every rank joins the process group, checks the world size and "
                        "rank 0 prints the ranks it saw (no sweep; runs on the CPU with gloo)")
    return p.parse_args(argv)


def launch_command(n: int, argv, port: int):
    """torchrun command line for ``--gpus n`` started from a plain ``python bench.py``."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"), *argv]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """Run the N-rank bench as a child torchrun (one process per GPU) and return its
    exit status.  The parent touches no GPU API (no torch.cuda call at all): it
    only waits.  Rank 0's JSON line reaches our stdout directly (inherited)."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run(launch_command(n, argv, _free_port()), env=env)
    return r.returncode


def check_world(args, world: int):
    """Every rank: the process group must have exactly ``--gpus`` ranks."""
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {world} rank(s) "
                         f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')})")


def model_shapes(name):
    from data_free_quantization_amd import zoo
    return [tuple(m.weight.shape) for m in zoo.target_layers(zoo.MODELS[name]())]


def synth_weight(s, dev, gen):
    """conv ~ N(0, sqrt(2/(k*k*O))), linear ~ N(0, 0.01)."""
    std = (2.0 / (s[2] * s[3] * s[0])) ** 0.5 if len(s) == 4 else 0.01
    return torch.randn(s, device=dev, generator=gen) * std


def build_batch(model, dev, copies=0, bits=8, channel=True, sym=True, esum=True, seed=1234, pack=False):
    """Synthetic weight sets of the model's target-layer shapes, generated on the
    GPU; ``copies`` = 0 picks enough for >= 2 GiB of fp32 weights (past the
    256 MB Infinity Cache)."""
    from data_free_quantization_amd.sweep import allocate, khw_of
    shapes = model_shapes(model)
    per_copy = sum(int(torch.Size(s).numel()) for s in shapes)
    copies = copies or max(1, -(-(2 << 30) // (4 * per_copy)))
    gen = torch.Generator(device=dev).manual_seed(seed + int(os.environ.get("RANK", "0")))
    items = []
    for c in range(copies):
        for s in shapes:
            w = synth_weight(s, dev, gen)
            items.append(allocate(w, bits=bits, per_channel=channel, symmetric=sym, khw=khw_of(w), want_esum=esum,
                                  clip=(-15.0, 15.0), pack_int4=pack))
    return items, shapes, per_copy, copies


class Telemetry:
    """GPU clocks, power and throttle state read in-process through the amdsmi
    Python module (sysfs / driver queries, no HIP call), for the device this
    process runs on (matched by PCI bus id).  Every read is best effort: a box
    where amdsmi is missing or refuses a query reports None for that field."""

    def __init__(self, dev):
        self.handle, self.error = None, None
        try:
            import amdsmi
            self.smi = amdsmi
            amdsmi.amdsmi_init()
            p = torch.cuda.get_device_properties(dev)
            want = (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
            for h in amdsmi.amdsmi_get_processor_handles():
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)          # "dddd:bb:dd.f"
                dom, bus, rest = bdf.split(":")
                if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                    self.handle = h
                    break
            if self.handle is None:
                self.error = f"no amdsmi handle with PCI id {want}"
        except Exception as e:   # amdsmi absent or not permitted on this box
            self.error = f"{type(e).__name__}: {e}"

    def sample(self, tag):
        out = {"tag": tag, "t": round(time.perf_counter(), 4)}
        if self.handle is None:
            out["error"] = self.error
            return out
        smi = self.smi
        try:
            m = smi.amdsmi_get_gpu_metrics_info(self.handle)
            for k in ("current_gfxclk", "current_uclk", "current_socclk", "average_gfxclk_frequency",
                      "average_uclk_frequency", "average_socket_power", "current_socket_power",
                      "average_umc_activity", "average_gfx_activity", "temperature_hotspot", "temperature_mem",
                      "throttle_status", "indep_throttle_status", "gfxclk_lock_status"):
                v = m.get(k)
                if v is not None and v != "N/A":
                    out[k] = v
            g = m.get("current_gfxclks")
            if isinstance(g, list):
                g = [x for x in g if isinstance(x, int) and x < 0xFFFF]
                if g:
                    out["gfxclk_per_xcd"] = g
        except Exception as e:
            out["metrics_error"] = f"{type(e).__name__}: {e}"
        for name, ct in (("sclk", "GFX"), ("mclk", "MEM"), ("fclk", "DF"), ("socclk", "SOC")):
            try:
                c = smi.amdsmi_get_clock_info(self.handle, getattr(smi.AmdSmiClkType, ct))
                out[name] = {"clk": c["clk"], "min": c["min_clk"], "max": c["max_clk"],
                             "deep_sleep": c["clk_deep_sleep"]}
            except Exception:
                pass
        return out


def steps_with_events(run, stream, n):
    """Run ``run`` n times with a HIP event pair around each call on ``stream``;
    returns the per-step device milliseconds (after one synchronize)."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in evs:
        a.record(stream)
        run()
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


def prewarm(run, stream, dev, ms_target):
    """Time-based pre-warm before the counted warm-up: sweep steps until
    ``ms_target`` milliseconds of wall time have passed, in batches of 8 with a
    HIP event pair per step.  A fresh lease starts with the GPU at idle clocks;
    the per-step series shows the ramp (first / last steps, and the mean of each
    tenth of the run)."""
    series = []
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms_target or not series:
        series += steps_with_events(run, stream, 8)
    wall = (time.perf_counter() - t0) * 1e3
    k = max(1, len(series) // 10)
    return {"ms_target": ms_target, "wall_ms": round(wall, 1), "steps": len(series),
            "first_steps_ms": [round(x, 4) for x in series[:8]],
            "last_steps_ms": [round(x, 4) for x in series[-8:]],
            "tenths_mean_ms": [round(sum(series[i:i + k]) / len(series[i:i + k]), 4)
                               for i in range(0, len(series), k)][:10]}


def time_plan(plan, stream, dev, steps, warmup, prewarm_ms=100.0):
    """Device ms per execute() of ``plan`` (all its launches; HIP events on its stream),
    after ``prewarm_ms`` of wall time of executes (the GPU idles between legs) and
    ``warmup`` more."""
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < prewarm_ms:
        for _ in range(4):
            plan.execute(stream)
        torch.cuda.synchronize(dev)
    for _ in range(warmup):
        plan.execute(stream)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        plan.execute(stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / steps


SECONDARY = [
    # (name, model, bits, channel, sym, esum) -- BASELINE.json configs[2..4]
    ("resnet50 per-ch sym INT8 + clip + BC error sums", "resnet50", 8, True, True, True),
    ("deeplab per-ch sym INT8 + clip + BC error sums", "deeplab", 8, True, True, True),
    ("resnet50 per-ch asym INT4 + clip", "resnet50", 4, True, False, False),
    ("resnet50 per-ch asym INT4 + clip, packed int4 codes", "resnet50", 4, True, False, False, True),
    ("mobilenetv2 per-tensor asym INT8 (quantize_targ_layer) + clip", "mobilenetv2", 8, False, False, False),
]


def secondary_configs(dev, stream, steps=20):
    """The other BASELINE configs on this GPU (>= 2 GiB batches): algorithmic
    GB/s of the sweep kernel and weight-GB/s, so the >= 60 % roofline target is
    checked on ResNet-50 as well as MobileNetV2."""
    from data_free_quantization_amd.sweep import SweepPlan
    out = []
    for name, model, bits, ch, sym, es, *pack in SECONDARY:
        items, _, per_copy, copies = build_batch(model, dev, bits=bits, channel=ch, sym=sym, esum=es, seed=99,
                                                 pack=bool(pack and pack[0]))
        plan = SweepPlan(items)
        ms = time_plan(plan, stream, dev, steps, 3)
        st = plan.stats
        out.append({"config": name, "copies": copies, "algo_GBs": round(st["algo_bytes"] / ms / 1e6, 1),
                    "frac": round(st["algo_bytes"] / ms / 1e6 / HBM_PEAK_GBS, 4),
                    "weight_GBs": round(4 * per_copy * copies / ms / 1e6, 1),
                    "step_ms": round(ms, 4), "launches": st["launches"], "reduce_tasks": st["n_tasks_reduce"]})
        plan.destroy()
        del items, plan
        torch.cuda.empty_cache()
    return out


def fold_quant_pair(dev, stream, steps=20):
    """main_dfq's merge_batchnorm #2 + quantize_targ_layer pair (main_dfq.py:211-214)
    in the reference's per-tensor mode, MobileNetV2 x155 (per-tensor asym INT8 +
    clip): the second fold's BatchNorms are the identity the first fold left, so it
    reads each weight (factor exactly 1: nothing rewritten) and leaves the
    weight's (min, max) on the device; the quantize sweep then runs in ONE pass
    (DFQ_DEVICE_RANGE) instead of reduce + quantize.  Algorithmic bytes: the
    fold's read (4 B/element) + the sweep's 9 B/element (+ scale, zero)."""
    import ctypes as C
    import numpy as np
    from data_free_quantization_amd import _lib
    from data_free_quantization_amd.sweep import SweepPlan
    from data_free_quantization_amd.utils.layer_transform import _BN_DESC
    L = _lib.load()
    items, _, per_copy, copies = build_batch("mobilenetv2", dev, bits=8, channel=False, sym=False, esum=False,
                                             seed=99)
    n = len(items)
    rows = np.array([it.src.shape[0] for it in items], dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(rows)[:-1]]).astype(np.uint64)
    tot = int(rows.sum())
    ones = torch.ones(2 * tot, device=dev)           # bn weight, bn var
    zeros = torch.zeros(3 * tot, device=dev)         # bn bias, bn mean, conv bias
    rbuf = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    tab = np.zeros(n, dtype=_BN_DESC)
    p1, p0 = np.uint64(ones.data_ptr()), np.uint64(zeros.data_ptr())
    t4 = np.uint64(4 * tot)
    ptr = tab["ptr"]
    ptr[:, 0] = [it.src.data_ptr() for it in items]
    ptr[:, 1] = p0 + 2 * t4 + 4 * off                # conv bias
    ptr[:, 2] = p1 + 4 * off                         # bn weight
    ptr[:, 3] = p0 + 4 * off                         # bn bias
    ptr[:, 4] = p0 + t4 + 4 * off                    # bn mean
    ptr[:, 5] = p1 + t4 + 4 * off                    # bn var
    tab["rows"] = rows
    tab["row_len"] = [it.src.numel() // it.src.shape[0] for it in items]
    tab["range_enc"] = np.uint64(rbuf.data_ptr()) + 8 * np.arange(n, dtype=np.uint64)
    descs = tab.ctypes.data_as(C.POINTER(_lib.BnFoldDesc))
    ws = torch.empty(max(int(L.dfq_bn_fold_ws_bytes(descs, n)), 256), dtype=torch.uint8, device=dev)
    sp = C.c_void_p(stream.cuda_stream)

    def fold():
        _lib.check(L.dfq_bn_fold_batch(descs, n, ws.data_ptr(), ws.numel(), sp), "dfq_bn_fold_batch")

    two_pass = SweepPlan(items)                      # the range from a reduce pass
    for j, it in enumerate(items):
        it.range_enc = rbuf[2 * j:2 * j + 2]
    one_pass = SweepPlan(items)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / steps

    def pair():
        fold()
        one_pass.execute(stream)

    def old_pair():
        fold()
        two_pass.execute(stream)

    ms_pair, ms_fold = timed(pair), timed(fold)
    ms_old = timed(old_pair)
    elems = per_copy * copies
    algo = 4 * elems + one_pass.stats["algo_bytes"]
    out = {"config": "mobilenetv2 bn2 fold + per-tensor asym INT8 + clip (main_dfq order, fold ranges -> "
                     "one-pass sweep)", "copies": copies,
           "algo_GBs": round(algo / ms_pair / 1e6, 1), "frac": round(algo / ms_pair / 1e6 / HBM_PEAK_GBS, 4),
           "weight_GBs": round(4 * elems / ms_pair / 1e6, 1), "step_ms": round(ms_pair, 4),
           "fold_ms": round(ms_fold, 4), "sweep_launches": one_pass.stats["launches"],
           "with_reduce_pass_ms": round(ms_old, 4)}
    two_pass.destroy()
    one_pass.destroy()
    del items, ws, ones, zeros
    torch.cuda.empty_cache()
    return out


def time_plan_graph(plan, dev, per_graph=50, replays=8):
    """Device ms per execute() with the host out of the loop: ``per_graph``
    executes captured in one HIP graph (stream capture), replayed back to back.
    A Python execute() costs several microseconds of host time, more than a
    single small model's kernel, so the back-to-back event timing of time_plan is
    host-paced for one weight set; this is the kernel-to-kernel rate."""
    cs = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(g, stream=cs):
        for _ in range(per_graph):
            plan.execute(cs)
    g.replay()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream(dev)
    e0.record(cur)
    for _ in range(replays):
        g.replay()
    e1.record(cur)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / (replays * per_graph)


def single_model_latency(dev, stream, reps=200):
    """ONE weight set per model (cache-resident: MobileNetV2
    45 MB algorithmic), per-channel sym INT8 + codes + clip + BC sums; device
    microseconds per execute() and the algorithmic GB/s that implies: ``us`` from
    back-to-back Python execute() calls (host-paced at this size), ``graph_us``
    from the same executes replayed as one HIP graph (kernel to kernel)."""
    from data_free_quantization_amd.sweep import SweepPlan
    out = {}
    for model in ("mobilenetv2", "resnet50", "deeplab"):
        items, _, _, _ = build_batch(model, dev, copies=1, seed=5)
        plan = SweepPlan(items)
        ms = time_plan(plan, stream, dev, reps, 20)
        try:
            gms = time_plan_graph(plan, dev)
        except Exception as e:   # capture unsupported: report the host-paced number only
            gms = None
            print(f"# graph timing unavailable: {e}", file=sys.stderr)
        out[model] = {"us": round(ms * 1e3, 2), "algo_GBs": round(plan.stats["algo_bytes"] / ms / 1e6, 1),
                      "graph_us": None if gms is None else round(gms * 1e3, 2),
                      "graph_algo_GBs": None if gms is None else round(plan.stats["algo_bytes"] / gms / 1e6, 1),
                      "launches": plan.stats["launches"]}
        plan.destroy()
    # BASELINE.md's GPU target rows as defined there (per-channel W8 + codes + clip;
    # E only where the row says "+ BC"), time at 60 % of 8 TB/s
    rows = []
    for name, model, es, target_us in (("MobileNetV2 per-channel W8", "mobilenetv2", False, 6.5),
                                       ("ResNet-50 per-channel W8 + BC", "resnet50", True, 47.8),
                                       ("DeepLab per-channel W8", "deeplab", False, 10.8)):
        items, _, _, _ = build_batch(model, dev, copies=1, seed=5, esum=es)
        plan = SweepPlan(items)
        ms = time_plan(plan, stream, dev, reps, 20)
        try:
            gms = time_plan_graph(plan, dev)
        except Exception:
            gms = None
        rows.append({"row": name, "us": round(ms * 1e3, 2), "target_us": target_us,
                     "graph_us": None if gms is None else round(gms * 1e3, 2),
                     "algo_MB": round(plan.stats["algo_bytes"] / 1e6, 1),
                     "algo_GBs": round(plan.stats["algo_bytes"] / ms / 1e6, 1)})
        plan.destroy()
    out["baseline_md_rows"] = rows
    return out


def _timed_steps(fn, dev, reps, warmup=3):
    """Wall seconds per call of ``fn`` (collectives inside), barrier-bracketed and
    max over ranks."""
    import torch.distributed as dist
    from data_free_quantization_amd.distributed import max_over_ranks
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    return max_over_ranks(time.perf_counter() - t0, dev) / reps


def _std_of(shp):
    """Synthetic init scale: conv ~ N(0, sqrt(2/(k*k*O))), linear ~ N(0, 0.01)."""
    return (2.0 / (shp[2] * shp[3] * shp[0])) ** 0.5 if len(shp) == 4 else 0.01


def make_list(specs, mine, dev, seed):
    """Per-tensor allocations (input, then its outputs, in the order eager code
    makes them) of the layers ``mine`` of the list ``specs``.  Every layer's
    synthetic weight is drawn from ONE generator in list order -- a layer this rank
    does not hold is drawn into a scratch buffer and dropped -- so layer i holds the
    same values whatever the world size and no broadcast is needed.  (The sweep
    over per-field arenas is placement-bound: 1.08 or 1.31-1.37 ms per step box to
    box, 1.36 against 1.11 for per-tensor allocations on one box in five
    interleaved process pairs; profiles/r02/ab_layout.jsonl, ab_arena.md.)"""
    from data_free_quantization_amd.sweep import allocate
    gen = torch.Generator(device=dev).manual_seed(seed)
    keep = set(mine)
    scratch = None
    if len(keep) < len(specs):
        scratch = torch.empty(max(s.numel for i, s in enumerate(specs) if i not in keep), device=dev)
    items = []
    for i, s in enumerate(specs):
        if i in keep:
            w = torch.empty(s.shape, device=dev).normal_(0.0, _std_of(s.shape), generator=gen)
            items.append(allocate(w, bits=s.bits, per_channel=s.per_channel, symmetric=s.symmetric, khw=s.khw,
                                  want_esum=s.want_esum, clip=s.clip, pack_int4=s.pack_int4))
        else:
            scratch[:s.numel].view(s.shape).normal_(0.0, _std_of(s.shape), generator=gen)
    del scratch
    return items


def _plan_of(items):
    from data_free_quantization_amd.sweep import SweepPlan
    return SweepPlan(items)


def sharded_gathers(specs, dev, stream, reps=10):
    """Beside the headline (the one list LPT-sharded, outputs left sharded): the same
    list in the sharded sweep's per-field slab arenas (distributed.ShardedSweep,
    the layout its collectives move), timed per pass of the whole list (wall,
    barrier-bracketed, max over ranks): ``sweep_ms`` (outputs sharded),
    ``sweep_gather_root_ms`` (+ one grouped receive per rank of its output slabs
    into rank 0's arenas) and ``sweep_allgather_ms`` (+ one in-place
    all_gather_into_tensor per output field: every rank ends holding every output).
    Each rank fills only its own layers' inputs (same generator order as the
    headline)."""
    import torch.distributed as dist
    from data_free_quantization_amd import distributed as D
    sw = D.ShardedSweep(specs, replicate=True, device=dev)
    gen = torch.Generator(device=dev).manual_seed(1234)
    mine = set(sw.mine)
    for i, s in enumerate(specs):   # the headline's values (one generator in list order)
        if i in mine:
            sw.weight(i).normal_(0.0, _std_of(s.shape), generator=gen)
        else:
            torch.empty(s.shape, device=dev).normal_(0.0, _std_of(s.shape), generator=gen)
    torch.cuda.synchronize(dev)
    wbytes = 4 * sum(s.numel for s in specs)
    out = {"rccl_ranks": sw.world, "backend": dist.get_backend() if dist.is_initialized() else None,
           "layers_per_rank": [len(p) for p in sw.layout.parts],
           "output_bytes_per_rank": [sum(sw.layout.used[f][r] for f in sw.layout.fields if f != "w")
                                     for r in range(sw.world)]}

    def step_root():
        sw.run(stream)
        sw.gather("root")

    def step_all():
        sw.run(stream)
        sw.gather("all")

    for name, fn in (("sweep", lambda: sw.run(stream)), ("sweep_gather_root", step_root),
                     ("sweep_allgather", step_all)):
        t = _timed_steps(fn, dev, reps)
        out[f"{name}_ms"] = round(t * 1e3, 4)
        out[f"{name}_weight_GBs"] = round(wbytes / t / 1e9, 1)
    out["note"] = ("the headline's list in per-field slab arenas; host-timed, barrier-bracketed, max over ranks; "
                   "weight_GBs = the whole list's fp32 weight bytes per pass")
    sw.destroy()
    del sw
    torch.cuda.empty_cache()
    return out


def weak_scaling(specs, weights, dev, stream, rank, world, steps, warmup):
    """Secondary: every rank sweeps its OWN whole list (rank-seeded synthetic
    weights, per-tensor allocations), no collective; weight-GB/s = all ranks'
    weight bytes over the max-over-ranks step (the round-5 headline)."""
    import torch.distributed as dist
    from data_free_quantization_amd import distributed as D
    items = make_list(specs, range(len(specs)), dev, 1234 + 7919 * rank)
    plan = _plan_of(items)
    for _ in range(max(warmup, 1)):
        plan.execute(stream)
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        plan.execute(stream)
    torch.cuda.synchronize(dev)
    dist.barrier()
    t = D.max_over_ranks(time.perf_counter() - t0, dev) / steps
    plan.destroy()
    del plan, items
    torch.cuda.empty_cache()
    return {"ms_per_step": round(t * 1e3, 4), "value": round(4 * weights * world / t / 1e9, 2),
            "unit": "GB/s", "lists": world,
            "note": "every rank its own whole list, no collective; value = all ranks' weight bytes / max step"}


def configs4_sharded(dev, stream, reps=10, parity=True):
    """BASELINE configs[4] at N > 1: ONE >= 2 GiB layer list of ResNet-50 weight
    sets (per-channel asym INT4 + clip [-15, 15], packed int4 codes: the
    SECONDARY config of that name), held by rank 0 and LPT-sharded over the ranks
    (distributed.ShardedSweep; scatter once before timing).  Timed (wall,
    barrier-bracketed, max over ranks), ms per pass of the WHOLE list:

    * ``sweep``: every rank sweeps its share, outputs left sharded (strong scaling);
    * ``sweep_gather_root``: + one grouped receive per rank of its output slabs
      into rank 0's arenas (rank 0 ends holding every output);
    * ``scatter_sweep_gather_root``: rank 0 -> ranks input slabs, sweep, gather
      (rank 0 holds the list end to end);
    * ``sweep_allgather``: + one in-place all_gather_into_tensor per field.

    Parity (checker leg): after a gather to rank 0, the first, middle and last
    weight sets' outputs vs the C oracle on the same inputs (every field)."""
    import torch.distributed as dist
    from data_free_quantization_amd import distributed as D
    from data_free_quantization_amd.sweep import SweepItem
    shapes = model_shapes("resnet50")
    per_copy = sum(int(torch.Size(s).numel()) for s in shapes)
    copies = max(1, -(-(2 << 30) // (4 * per_copy)))
    specs = D.uniform_specs(shapes * copies, bits=4, per_channel=True, symmetric=False, want_esum=False,
                            clip=(-15.0, 15.0), pack_int4=True)
    sw = D.ShardedSweep(specs, replicate=True, device=dev)
    if sw.rank == 0:
        gen = torch.Generator(device=dev).manual_seed(4321)
        for i, s in enumerate(specs):
            sw.weight(i).copy_(synth_weight(s.shape, dev, gen))
    sw.scatter()
    torch.cuda.synchronize(dev)
    wbytes = 4 * per_copy * copies
    out = {"config": "resnet50 per-ch asym INT4 + clip, packed int4 codes; one layer list on rank 0, "
                     "LPT-sharded over the ranks", "copies": copies, "layers": len(specs),
           "rccl_ranks": sw.world, "backend": dist.get_backend() if dist.is_initialized() else None,
           "layers_per_rank": [len(p) for p in sw.layout.parts],
           "weight_bytes_per_rank": [sum(4 * specs[i].numel for i in p) for p in sw.layout.parts]}

    def step_root():
        sw.run(stream)
        sw.gather("root")

    def step_e2e():
        sw.scatter()
        sw.run(stream)
        sw.gather("root")

    def step_all():
        sw.run(stream)
        sw.gather("all")

    for name, fn in (("sweep", lambda: sw.run(stream)), ("sweep_gather_root", step_root),
                     ("scatter_sweep_gather_root", step_e2e), ("sweep_allgather", step_all)):
        t = _timed_steps(fn, dev, reps)
        out[f"{name}_ms"] = round(t * 1e3, 4)
        out[f"{name}_weight_GBs"] = round(wbytes / t / 1e9, 1)
    if sw.plan_stats is not None:
        out["rank_plan"] = {"algo_bytes": sw.plan_stats["algo_bytes"], "launches": sw.plan_stats["launches"]}
    if parity:
        sw.run(stream)
        sw.gather("root")
        torch.cuda.synchronize(dev)
        if sw.rank == 0:
            from tests.parity import sweep_mismatches
            sets = sorted({0, copies // 2, copies - 1})
            items = []
            for c in sets:
                for i in range(c * len(shapes), (c + 1) * len(shapes)):
                    s, o = specs[i], sw.outputs(i)
                    items.append(SweepItem(src=sw.weight(i), dst=o.dq, codes=o.codes, scale=o.scale, zero=o.zero,
                                           esum=o.esum, bits=s.bits, per_channel=s.per_channel,
                                           symmetric=s.symmetric, khw=s.khw, clip=s.clip, rows=s.rows,
                                           pack_int4=s.pack_int4))
            t0 = time.perf_counter()
            par = sweep_mismatches(items)
            par["weight_sets"] = sets
            par["owners"] = sorted({sw.layout.owner[c * len(shapes) + j] for c in sets for j in range(len(shapes))})
            par["seconds"] = round(time.perf_counter() - t0, 2)
            out["parity"] = par
        if dist.is_initialized():
            dist.barrier()
    out["note"] = ("host-timed, barrier-bracketed, max over ranks; weight_GBs = the whole list's fp32 weight "
                   "bytes per pass; gather/scatter = one grouped send/recv per rank of exactly its slabs, "
                   "all-gather = one in-place all_gather_into_tensor per output field")
    sw.destroy()
    del sw
    torch.cuda.empty_cache()
    return out


def sharded_single_model(dev, stream, reps=20):
    """BASELINE configs[4]: ONE ResNet-50 weight set (INT4 per-channel asym +
    clip, packed codes), its layer list LPT-sharded over the ranks; ms per pass
    with outputs left sharded, gathered to rank 0, and all-gathered."""
    from data_free_quantization_amd import distributed as D
    specs = D.uniform_specs(model_shapes("resnet50"), bits=4, per_channel=True, symmetric=False, want_esum=False,
                            clip=(-15.0, 15.0), pack_int4=True)
    sw = D.ShardedSweep(specs, replicate=True, device=dev)
    gen = torch.Generator(device=dev).manual_seed(7)
    if sw.rank == 0:
        for i, s in enumerate(specs):
            sw.weight(i).copy_(synth_weight(s.shape, dev, gen))
    sw.broadcast()
    res = {}
    for name, fn in (("none", lambda: sw.run(stream)),
                     ("root", lambda: (sw.run(stream), sw.gather("root"))),
                     ("all", lambda: (sw.run(stream), sw.gather("all")))):
        res[f"ms_gather_{name}"] = round(_timed_steps(fn, dev, reps) * 1e3, 4)
    sw.destroy()
    res["weights"] = sum(s.numel for s in specs)
    res["note"] = "host-timed per pass; single-model sizes are latency bound (one 102 MB weight set)"
    return res


def cpu_baseline(args, shapes, seconds):
    """The reference's CPU arithmetic on the GPU box's host cores, on a bounded
    sample of the same workload (one whole weight set of the model), BASELINE.md
    section 2's protocol: best of 5 passes with all of this process's host threads and
    best of 5 (3 when a pass is long) on 1 thread.

    * value: oracle/torch_port.py -- a PORT of the reference's own torch CPU op
      sequence (UniformQuantize.forward per output channel, clip_weight's clamp,
      the BC error sums; the per-channel composition SURVEY.md 8a row a3 defines),
      ``cores`` intra-op threads;
    * per_tensor_*: quantize_targ_layer's per-tensor sweep (the reference's own
      mode), same protocol;
    * oracle_c_1thread_GBs: the scalar C restatement (oracle/dfq_oracle.c)."""
    import numpy as np
    from oracle import oracle as O
    from oracle import torch_port as TP
    rng = np.random.default_rng(0)
    ws = []
    for s in shapes:
        std = (2.0 / (s[2] * s[3] * s[0])) ** 0.5 if len(s) == 4 else 0.01
        ws.append(rng.normal(0, std, s).astype(np.float32))
    tw = [torch.from_numpy(w) for w in ws]
    elems = sum(w.size for w in ws)
    sym = not args.asym

    def best_of(fn, reps, budget):
        """Best single-pass seconds over up to ``reps`` passes within ``budget`` s."""
        best, t_all = None, time.perf_counter()
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
            if time.perf_counter() - t_all > budget:
                break
        return best

    def port_pass():
        for w in tw:
            TP.per_channel_sweep(w, args.bits, sym, clip=(-15.0, 15.0), want_esum=not args.no_esum)

    def per_tensor_pass():
        for w in tw:
            TP.per_tensor_sweep(w, args.bits, False)

    mode = (O.CHANNEL_ASYM if args.asym else O.CHANNEL_SYM) if args.granularity == "channel" else \
        (O.TENSOR_ASYM if args.asym else O.TENSOR_SYM)

    def c_pass():
        for w in ws:
            rows = w.shape[0] if mode >= 2 else 1
            khw = w.shape[2] * w.shape[3] if w.ndim == 4 else 1
            O.quantize(w, args.bits, mode, rows=rows, khw=khw, flags=O.F_CLIP, clip=(-15.0, 15.0),
                       want_esum=not args.no_esum)

    threads = torch.get_num_threads()
    gbs = lambda t: round(4.0 * elems / t / 1e9, 4)    # noqa: E731
    t_port = best_of(port_pass, 5, seconds * 0.4)
    t_tensor = best_of(per_tensor_pass, 5, seconds * 0.05)
    torch.set_num_threads(1)
    try:
        t_port1 = best_of(port_pass, 5, seconds * 0.4)
        t_tensor1 = best_of(per_tensor_pass, 5, seconds * 0.05)
    finally:
        torch.set_num_threads(threads)
    t_c = best_of(c_pass, 3, seconds * 0.1)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    return {"value": gbs(t_port), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{args.model} x1 weight set ({len(ws)} layers, {elems} weights), best of 5 passes: a port "
                      f"of the reference's torch CPU ops (oracle/torch_port.py: quantize() per output channel + "
                      f"clamp + BC error sums) on {threads} intra-op threads (this process's host-CPU share: "
                      f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}, os.cpu_count()={os.cpu_count()}, "
                      f"affinity {affinity})",
            "threads_note": (f"cores = torch's intra-op threads = OMP_NUM_THREADS ({os.environ.get('OMP_NUM_THREADS')}), "
                             f"the CPU share the GPU box gives this process; os.cpu_count() ({os.cpu_count()}) counts "
                             "the whole host, and that many threads on this share would oversubscribe it.  The "
                             "per-channel port equals its 1-thread rate because the reference's per-row quantize() "
                             "calls (one Python call per output channel, tiny rows) bound it, not arithmetic; the "
                             "per-tensor mode below shows the thread scaling"),
            "value_1thread": gbs(t_port1),
            "per_tensor_GBs": gbs(t_tensor), "per_tensor_1thread_GBs": gbs(t_tensor1),
            "per_tensor_sample": "quantize_targ_layer's arithmetic (one range per tensor), best of 5",
            "oracle_c_1thread_GBs": gbs(t_c)}


def cpu_baseline_transforms(dev, seconds):
    """The reference's CLE loop and bias-correction error reduction as torch CPU
    ops (oracle/torch_port.py: Cross_layer_equal.py:11-116, bias_correction.py:
    111-144,231), on MobileNetV2 after the first BN fold (seed 0, the pipeline
    fixture's model), with this process's host threads.  CLE: whole iterations
    until ~``seconds`` are spent (the reference's per-channel Python loop makes
    one iteration take seconds), each iteration's diff checked against the
    reference's own (tests/golden/pipeline_mobilenetv2.npz); the full loop is
    that per-iteration time x the reference's iteration count.  BC: best of 3
    passes of _quantize_error + spatial sum over every target weight."""
    import numpy as np
    import torch.nn as nn
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.utils.layer_transform import merge_batchnorm
    from data_free_quantization_amd.utils.relation import create_relation
    from data_free_quantization_amd.utils.tracer import build_graph
    from oracle import torch_port as TP
    from tests.helpers import pipeline
    targ = (nn.Conv2d, nn.Linear)
    m = zoo.build("mobilenetv2", seed=0, relu=True).to(dev)
    g = build_graph(m, "positional")
    G, B = g.getGraph(), g.getBottoms()
    merge_batchnorm(m, G, B, targ)
    rels = create_relation(G, B, targ)
    tk = [k for k in G if type(G[k]) in targ]
    weights = {k: G[k].weight.detach().cpu().clone() for k in tk}
    biases = {k: (G[k].bias.detach().cpu().clone() if G[k].bias is not None else None) for k in tk}
    bn = {r.bn_idx: (G[r.bn_idx].fake_weight.detach().cpu().clone(), G[r.bn_idx].fake_bias.detach().cpu().clone())
          for r in rels}
    relations = [r.get_idxs() for r in rels]
    ref_diffs = [float(x) for x in pipeline("mobilenetv2")["cle_diffs"]]
    times, diffs = [], []
    t_all = time.perf_counter()
    while time.perf_counter() - t_all < seconds and len(diffs) < len(ref_diffs):
        t0 = time.perf_counter()
        diffs.append(TP.cle_iteration(weights, biases, bn, relations))
        times.append(time.perf_counter() - t0)
    per_it = float(np.median(times))
    bc = []
    for _ in range(3):
        t0 = time.perf_counter()
        for k in tk:
            TP.quantize_error_spatial(weights[k], 8, False)
        bc.append(time.perf_counter() - t0)
    elems = sum(w.numel() for w in weights.values())
    return {"threads": torch.get_num_threads(), "kind": "port",
            "cle_s_per_iteration": round(per_it, 4), "cle_iterations_timed": len(times),
            "cle_iterations_reference": len(ref_diffs),
            "cle_loop_s_est": round(per_it * len(ref_diffs), 2),
            "cle_diffs_max_rel_dev_vs_reference": float(max(abs(a - b) / abs(b) for a, b in zip(diffs, ref_diffs))),
            "cle_diffs_note": "the port runs torch.sqrt through this host's MKL path; the fixtures were made with "
                              "MKL_CBWR=AVX2 (IEEE sqrt), so the two agree to ~1 ulp per step (DESIGN.md 3.3)",
            "bc_error_reduction_ms": round(min(bc) * 1e3, 3),
            "bc_error_reduction_GBs": round(4 * elems / min(bc) / 1e9, 3),
            "sample": f"MobileNetV2 after BN fold ({len(relations)} relations, {len(tk)} target layers, {elems} "
                      f"weights): {len(times)} whole CLE iterations of the reference's op sequence "
                      f"(per-channel Python loop; full loop = median iteration x {len(ref_diffs)} iterations); "
                      f"BC: _quantize_error + spatial sum over every target weight, best of 3"}


def parity_of_timed(items, mine, layers_per_copy, copies, dev):
    """Checker leg (test infrastructure, like cpu_baseline): the timed plan's
    outputs on this rank's layers (``items`` are the list's layers ``mine``) of the
    list's first, middle and last weight sets vs the C oracle
    (oracle/dfq_oracle.c) run on the same input tensors -- dq, codes, scale, zero
    and the bias-correction sums E, element by element (tests/parity.py)."""
    from tests.parity import sweep_mismatches
    torch.cuda.synchronize(dev)
    sets = sorted({0, copies // 2, copies - 1}) if copies else []
    sample = [it for it, i in zip(items, mine) if i // layers_per_copy in sets]
    t0 = time.perf_counter()
    out = sweep_mismatches(sample)
    out["weight_sets"] = sets
    out["seconds"] = round(time.perf_counter() - t0, 2)
    return out


def pipeline_parity(dev):
    """The whole main_dfq stage order on MobileNetV2 (reference-mode bias
    correction, per-tensor INT8, the fixture's configuration) vs the reference's
    own run: mismatch counts per stage (tests/parity.py, tests/golden)."""
    import contextlib
    import io
    import logging
    from tests.parity import pipeline_mismatches
    logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
    with contextlib.redirect_stdout(io.StringIO()):
        out = pipeline_mismatches("mobilenetv2", 8, dev)
    return out


def pipeline_timing(dev, model="mobilenetv2"):
    """One-off: the full main_dfq stage order on one model (per-channel sym INT8,
    fused BC) on the GPU; milliseconds per stage of the fastest of three warm runs
    (host-bound stages: a busy host core shows up as noise)."""
    import torch.nn as nn
    from data_free_quantization_amd import zoo, Cross_layer_equal as cle
    from data_free_quantization_amd.pipeline import run_dfq
    from data_free_quantization_amd.utils.tracer import build_graph
    import contextlib
    import io
    import logging
    logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
    best = None
    for rep in range(4):   # rep 0 warms up
        m = zoo.build(model, seed=0, relu=True).to(dev)
        g = build_graph(m, "positional")
        t = {}
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):   # the reference's progress prints
            run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel",
                    symmetric=True, bc_mode="fused", timings=t)
        torch.cuda.synchronize(dev)
        total = time.perf_counter() - t0
        if rep > 0 and (best is None or total < best[0]):
            best = (total, t, cle.LAST_RUN.get("iterations"), cle.LAST_RUN.get("host_ms"))
    total, t, iters, cle_host = best
    out = {k: round(v * 1e3, 3) for k, v in t.items()}
    out["total"] = round(total * 1e3, 3)
    out["cle_iterations"] = iters
    out["cle_host_ms"] = {k: round(v, 3) for k, v in (cle_host or {}).items()}   # create / launch / join
    # the same stage order as main_dfq runs it: no device sync between the stages,
    # so the host work of absorption / fold / quantize / BC overlaps the CLE loop
    # (launched asynchronously); one sync at the end
    e2e = None
    for rep in range(4):   # rep 0 warms up
        m = zoo.build(model, seed=0, relu=True).to(dev)
        g = build_graph(m, "positional")
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel",
                    symmetric=True, bc_mode="fused")
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        if rep > 0 and (e2e is None or dt < e2e):
            e2e = dt
    out["end_to_end"] = round(e2e * 1e3, 3)
    out["cle_launched"] = bool(cle.LAST_RUN.get("launched"))
    return out


def cle_roofline(dev, model="mobilenetv2", reps=4, traffic_json=None):
    """The CLE loop (Cross_layer_equal.py:63-116, the reference's dominant cost)
    against the HBM roofline: one blocking device run per rep on a fresh model
    after the first BN fold (the main_dfq order), with the loop's device time from
    one HIP event pair on its stream (Cross_layer_equal.DEVICE_TIMING).
    ``algo_bytes_per_iteration`` (dfq_cle_plan_stats): rescales 8 B per weight
    element and per-channel vector entry, metric tiles 12 B per target element,
    weight-reading range tasks 4 B per element.  Per iteration =
    device time / iteration groups launched (the iterations run + the one queued
    no-op group).  Fastest rep.  ``traffic``: HBM bytes per iteration from the
    committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the same loop
    (scripts/cle_pmc.sh), when present."""
    import torch.nn as nn
    from data_free_quantization_amd import zoo, Cross_layer_equal as cle
    from data_free_quantization_amd.utils.layer_transform import merge_batchnorm
    from data_free_quantization_amd.utils.relation import create_relation
    from data_free_quantization_amd.utils.tracer import build_graph
    import contextlib
    import io
    T = (nn.Conv2d, nn.Linear)
    best = None
    cle.DEVICE_TIMING = True
    try:
        for rep in range(reps + 1):   # rep 0 warms up
            m = zoo.build(model, seed=0, relu=True).to(dev)
            g = build_graph(m, "positional")
            G, B = g.getGraph(), g.getBottoms()
            with contextlib.redirect_stdout(io.StringIO()):
                merge_batchnorm(m, G, B, T)
                rels = create_relation(G, B, T)
                torch.cuda.synchronize(dev)
                cle.cross_layer_equalization(G, rels, T, Save_state=False, Treshhold=2e-7, launch=False)
            r = dict(cle.LAST_RUN)
            if rep > 0 and r.get("device_ms") and (best is None or r["device_ms"] < best["device_ms"]):
                best = r
    finally:
        cle.DEVICE_TIMING = False
    if best is None:
        return None
    groups = max(best["iterations_launched"], 1)
    per_it_s = best["device_ms"] / 1e3 / groups
    by = best["bytes_per_iteration"]
    achieved = by["total"] / per_it_s / 1e9
    out = {"model": model, "bound": "hbm", "kernel": "cle_loop_step_kernel", "iterations": best["iterations"],
           "iteration_groups_launched": groups, "launches_per_iteration": best["launches_per_iteration"],
           "loop_device_ms": round(best["device_ms"], 4), "device_us_per_iteration": round(per_it_s * 1e6, 3),
           "algo_bytes_per_iteration": by, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
           "note": "latency-bound: each iteration is dependent launches of a few microseconds over ~100 MB"}
    tj = Path(traffic_json) if traffic_json else None
    if tj is not None and tj.exists():
        try:
            tr = json.loads(tj.read_text())
            out["traffic"] = tr.get("hbm_bytes_per_iteration")
            out["traffic_source"] = str(tj.relative_to(ROOT)) if tj.is_relative_to(ROOT) else str(tj)
        except Exception:
            pass
    return out


def pipeline_cold(model="mobilenetv2"):
    """The first run of the stage order in a FRESH process (child process,
    scripts/cold_pipeline.py: dfq_preload as main_dfq does, then a cold and a warm
    run), ms per stage; None if the child fails."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, str(ROOT / "scripts" / "cold_pipeline.py"), model, "--preload"],
                           capture_output=True, text=True, timeout=300)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        return json.loads(line)
    except Exception:
        return None


def same_mix_probe(n, dev, stream, reps=10):
    """Achievable-ceiling probes with the sweep's 1x1-layer traffic mix (read 4 B,
    write 4 + 1 + 4 B per element) and no arithmetic: a grid-stride VGPR stream,
    and the sweep's own memory pattern (2048-element wave tasks through LDS-DMA,
    non-temporal stores).  Returns (stream GB/s, LDS-DMA GB/s)."""
    import ctypes as C
    from data_free_quantization_amd import _lib
    n = n // 2048 * 2048
    x = torch.randn(n, device=dev)
    y = torch.empty_like(x)
    cds = torch.empty(n, dtype=torch.uint8, device=dev)
    e = torch.empty_like(x)
    L = _lib.load_diag()   # the probes live in the diagnostics library (include/dfq_diag.h)
    s = C.c_void_p(stream.cuda_stream)

    def best_of(fn):
        best = None
        for _ in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / reps
            best = ms if best is None else min(best, ms)
        return best

    stream_ms = min(best_of(lambda b=b: _lib.check(L.dfq_probe_stream(_lib.ptr(x), _lib.ptr(y),
                                                                      C.c_void_p(cds.data_ptr()), _lib.ptr(e), n,
                                                                      b, s), "dfq_probe_stream"))
                    for b in (2048, 8192, -4096))
    lds_ms = best_of(lambda: _lib.check(L.dfq_probe_lds(_lib.ptr(x), _lib.ptr(y), C.c_void_p(cds.data_ptr()),
                                                        _lib.ptr(e), n, 0, 16384, s), "dfq_probe_lds"))
    del x, y, cds, e
    return round(13 * n / (stream_ms / 1e3) / 1e9, 1), round(13 * n / (lds_ms / 1e3) / 1e9, 1)


def probe_ranks(args):
    """--probe-ranks: join the process group, check the world size, gather every
    rank's (rank, world, local rank, pid) to rank 0, which prints one JSON line.
    No GPU work (gloo on the CPU), so the launcher is testable without a GPU."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    check_world(args, world)
    if world > 1:
        dist.init_process_group(os.environ.get("DFQ_DIST_BACKEND", "gloo"))
        check_world(args, dist.get_world_size())
        me = torch.tensor([dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", "0")),
                           os.getpid()], dtype=torch.int64)
        allv = [torch.zeros_like(me) for _ in range(world)]
        dist.all_gather(allv, me)
        rows = [v.tolist() for v in allv]
        backend = dist.get_backend()
        dist.destroy_process_group()
    else:
        rows, backend = [[0, 1, 0, os.getpid()]], None
    if rows[0][0] == 0 and int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps({"probe_ranks": rows, "n_gpus": world, "backend": backend}), flush=True)


def _side_leg(fn):
    """A secondary measurement after the timed step: its exception (on this rank)
    becomes {"error": ...} in the JSON line instead of ending the run before rank 0
    prints the headline."""
    try:
        return fn()
    except Exception as e:   # noqa: BLE001 -- reported, the headline stands
        try:
            torch.cuda.synchronize()
        except Exception:   # noqa: BLE001 -- the device error itself is what gets reported
            pass
        return {"error": f"{type(e).__name__}: {e}"[:500]}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: torchrun as a child, started before any GPU call here
        return launch_ranks(args.gpus, argv)
    check_world(args, int(os.environ.get("WORLD_SIZE", "1")))
    if args.probe_ranks:
        return probe_ranks(args)
    from data_free_quantization_amd import distributed as D
    world, rank, dev = D.init_from_env()
    if world > 1:
        import torch.distributed as dist
        check_world(args, dist.get_world_size())
    telemetry = Telemetry(dev)
    tele_start = telemetry.sample("process_start")
    shapes = model_shapes(args.model)
    per_copy = sum(int(torch.Size(s).numel()) for s in shapes)
    copies = args.copies or max(1, -(-(2 << 30) // (4 * per_copy)))   # >= 2 GiB of fp32 weights per rank
    specs = D.uniform_specs(shapes * copies, bits=args.bits, per_channel=args.granularity == "channel",
                            symmetric=not args.asym, want_esum=not args.no_esum, clip=(-15.0, 15.0))
    stream = torch.cuda.current_stream(dev)
    sw = plan = None
    # The headline: ONE layer list of ``copies`` weight sets (the N = 1 workload),
    # LPT-sharded over the ranks (distributed.ShardLayout, the partition the
    # sharded sweep and its gathers use).  Each rank materialises only its own
    # layers -- every layer's synthetic weight comes from one generator in list
    # order, so a layer holds the same values at every N and no broadcast is
    # needed -- and the timed step is its sweep with the outputs
    # left sharded (strong scaling).  The gathers are timed beside it
    # (sharded_gathers); N independent lists are the secondary weak_scaling key.
    layout = D.ShardLayout(specs, world)
    mine = layout.parts[rank]
    if args.layout == "arena" and world == 1:
        # diagnostics: the sharded path's per-field slab arenas at one rank
        gen = torch.Generator(device=dev).manual_seed(1234)
        sw = D.ShardedSweep(specs, replicate=True, device=dev)
        for i, s in enumerate(specs):
            sw.weight(i).normal_(0.0, _std_of(s.shape), generator=gen)
        st = sw.plan_stats
        run = lambda: sw.run(stream)   # noqa: E731
        items = None
    else:
        items = make_list(specs, mine, dev, 1234)
        plan = _plan_of(items)
        st = plan.stats
        run = lambda: plan.execute(stream)   # noqa: E731
    tele = [telemetry.sample("before_prewarm")]
    warm = prewarm(run, stream, dev, args.prewarm_ms) if args.prewarm_ms > 0 else None
    tele.append(telemetry.sample("after_prewarm"))
    warm_steps = steps_with_events(run, stream, args.warmup) if args.warmup > 0 else []
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    tele.append(telemetry.sample("before_timed"))
    step_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for a, b in step_ev:
        a.record(stream)
        run()
        b.record(stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    tele.append(telemetry.sample("after_timed"))
    step_ms = [a.elapsed_time(b) for a, b in step_ev]
    dev_ms = ev0.elapsed_time(ev1)          # device time of this rank's K launches on this stream
    t_step = D.max_over_ranks(wall, dev) / args.steps
    weight_bytes = 4 * per_copy * copies     # the one layer list, swept once per step (sharded at N > 1)
    value = weight_bytes / t_step / 1e9
    launch_ms = dev_ms / args.steps          # device time of one execute() (st["launches"] kernels)
    achieved = st["algo_bytes"] / (launch_ms / 1e3) / 1e9
    rank_launch_ms, rank_algo = [launch_ms], [st["algo_bytes"]]
    if world > 1:   # every rank's own kernel time and bytes (rank 0 reports its roofline)
        lt = torch.zeros(2, world, dtype=torch.float64, device=dev)
        lt[0, rank], lt[1, rank] = launch_ms, float(st["algo_bytes"])
        dist.all_reduce(lt)
        rank_launch_ms = [round(float(x), 4) for x in lt[0].tolist()]
        rank_algo = [int(x) for x in lt[1].tolist()]
    # parity of what was just timed: this rank's layers of the list's first, middle
    # and last weight sets vs the C oracle on the same input tensors (every field)
    timed_parity = None
    if items is not None and not args.no_parity:
        timed_parity = parity_of_timed(items, mine, len(shapes), copies, dev)
        if world > 1:   # every rank checked its own share: the job's total, and who held them
            tot = torch.zeros(2 + world, dtype=torch.int64, device=dev)
            tot[0], tot[1] = timed_parity["mismatches"], timed_parity["tensors"]
            tot[2 + rank] = 1 if timed_parity["tensors"] else 0
            dist.all_reduce(tot)
            timed_parity["all_ranks"] = {"mismatches": int(tot[0]), "tensors": int(tot[1])}
            timed_parity["mismatches"] = int(tot[0])
            timed_parity["tensors"] = int(tot[1])
            timed_parity["owners"] = [r for r in range(world) if int(tot[2 + r])]
        else:
            timed_parity["owners"] = [0]
    for obj in (sw, plan):
        if obj is not None:
            obj.destroy()
    del sw, plan, run, items
    torch.cuda.empty_cache()
    gathers = weak = None
    if world > 1:   # the side legs after the timed step: a failure is reported in the line, not fatal
        gloo = dist.get_backend() == "gloo"   # a one-GPU rehearsal stages every transfer through the host
        gathers = _side_leg(lambda: sharded_gathers(specs, dev, stream, reps=2 if gloo else 10))
        weak = _side_leg(lambda: weak_scaling(specs, per_copy * copies, dev, stream, rank, world, args.steps,
                                              args.warmup))
    sharded4 = None
    if world > 1 and not args.no_sharded:
        gloo = dist.get_backend() == "gloo"   # a one-GPU rehearsal stages every transfer through the host
        sharded4 = _side_leg(lambda: configs4_sharded(dev, stream, reps=2 if gloo else 10, parity=not args.no_parity))
    traffic, prof = None, None
    tj = Path(args.traffic_json)
    if tj.exists():
        try:
            tr = json.loads(tj.read_text())
            traffic = tr.get("hbm_bytes_per_launch")
            avg_ms = tr["rocprof_avg_ns"] / 1e6
            prof = {"source": str(tj.relative_to(ROOT)) if tj.is_relative_to(ROOT) else str(tj),
                    "rocprof_kernel_avg_ms": round(avg_ms, 4),
                    "frac_at_rocprof_avg": round(tr["algo_bytes_per_launch"] / (avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                                                 4),
                    "same_process_hip_event_ms": tr.get("same_process_hip_event_ms"),
                    "note": "rocprofv3 --kernel-trace --stats of `python bench.py` (same command, committed "
                            "build) on the lease box named in the summary; HIP-event frac above is this run's box"}
            if tr.get("algo_bytes_per_launch") != st["algo_bytes"]:
                prof["warning"] = "the profiled workload's algorithmic bytes differ from this run's"
        except Exception:
            traffic, prof = None, None
    sharded = sharded_single_model(dev, stream) if world > 1 and not args.no_secondary else None
    res = None
    if rank == 0:
        # the pipeline legs first: measured after the secondary / single-model legs
        # (HIP-graph captures, many plans) the same process ran the CLE loop 2.4x
        # slower (profiles/r03/validate_as vs r03at: MobileNetV2 end to end 10.4 vs
        # 5.3 ms), a state a main_dfq run never starts from
        # every leg below is a side measurement: an exception becomes {"error": ...}
        # in its key (_side_leg) and the headline above still prints
        pipe = None if args.no_pipeline else _side_leg(
            lambda: {m: pipeline_timing(dev, m) for m in ("mobilenetv2", "resnet50")})
        cle_roof = None if args.no_pipeline else _side_leg(lambda: {
            m: cle_roofline(dev, m, traffic_json=ROOT / "profiles" / "r06" / f"cle_traffic_{m}.json")
            for m in ("mobilenetv2", "resnet50")})
        second = None if args.no_secondary else _side_leg(
            lambda: secondary_configs(dev, stream) + [fold_quant_pair(dev, stream)])
        single = None if args.no_secondary else _side_leg(lambda: single_model_latency(dev, stream))
        # the same-mix probe last: a ResNet-50 x22 list allocated into the blocks its
        # ~7 GB of probe buffers left ran 0.699 of peak against 0.770 before it in the
        # same process (scripts/r50_state.py; DESIGN.md 3.1 "ResNet-50 in the bench")
        probe = _side_leg(lambda: same_mix_probe(per_copy * copies, dev, stream))
        probe_stream, probe_lds = probe if isinstance(probe, tuple) else (probe, probe)
        torch.cuda.empty_cache()
        cpu = _side_leg(lambda: cpu_baseline(args, shapes, args.cpu_seconds)) \
            if args.cpu_seconds > 0 and world == 1 else None
        if isinstance(cpu, dict) and "error" not in cpu:
            cpu["transforms"] = _side_leg(lambda: cpu_baseline_transforms(dev, args.cpu_seconds))
        parity = None
        if not args.no_parity:
            pp = _side_leg(lambda: pipeline_parity(dev))
            parity = {"timed_sweep": timed_parity, "pipeline_mobilenetv2": pp}
            if sharded4 is not None and "parity" in sharded4:
                parity["configs4_sharded"] = sharded4["parity"]
            parity["mismatches"] = pp.get("mismatches", "error") if "error" not in pp else "error"
            if isinstance(parity["mismatches"], int):
                parity["mismatches"] += (timed_parity["mismatches"] if timed_parity else 0) + \
                    (sharded4["parity"]["mismatches"] if sharded4 is not None and "parity" in sharded4 else 0)
        if pipe is not None and "error" not in pipe:   # the same run again after the other legs (see above)
            pipe["mobilenetv2"]["end_to_end_after_other_legs"] = _side_leg(
                lambda: pipeline_timing(dev, "mobilenetv2")["end_to_end"])
            pipe["cold_process_mobilenetv2"] = _side_leg(lambda: pipeline_cold("mobilenetv2"))
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "rccl_ranks": world,
            "backend": dist.get_backend() if world > 1 else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "codes": f"{args.bits}-bit grid indices stored as "
                     f"{'int16' if args.bits > 8 else ('uint8' if args.asym else 'int8')}",
            "data": "synthetic random-init weights of the reference shapes (no checkpoints offline)",
            "box": socket.gethostname(),
            "config": {
                "workload": f"{args.model} x{copies} weight sets in one layer list: {args.granularity} "
                            f"{'asym' if args.asym else 'sym'} INT{args.bits} quantize-dequantize + codes + "
                            f"clip[-15,15]" + ("" if args.no_esum else " + bias-correction error sums"),
                "weight_shapes": f"{args.model} target layers (SURVEY.md 8, synthetic init)",
                "copies": copies,
                "layers": len(specs),
                "layers_per_copy": len(shapes),
                "weights_per_copy": per_copy,
                "parallelism": (f"layer-sharded x{world}: one process per GPU; the one list's {len(specs)} layers "
                                "LPT-sharded over the ranks by algorithmic bytes, each rank materialises and sweeps "
                                "its share (per-tensor allocations), outputs left sharded in the timed step "
                                "(strong scaling); the gathers to rank 0 / to every rank in sharded_gathers, "
                                "N independent lists in weak_scaling")
                if world > 1 else "1 rank: the whole layer list on one GPU (per-tensor allocations, no exchange)",
                "layers_per_rank": [len(p) for p in layout.parts],
                "algo_bytes_per_rank": rank_algo,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic if world == 1 else None,
                "algo_bytes_per_launch": st["algo_bytes"],
                "launch_ms": round(launch_ms, 4),
                "launches": st["launches"],
                "kernel": "sweep_main_kernel",
                "tasks": st["n_tasks_main"],
                "grid_blocks": st["grid_blocks"],
                "variant": st["variant"],
                "rank": 0,
                "launch_ms_per_rank": rank_launch_ms,
                # the whole job: every rank's algorithmic bytes over the slowest rank's launch
                "job_achieved": round(sum(rank_algo) / (max(rank_launch_ms) / 1e3) / 1e9, 1),
                "job_frac_of_n_gpus": round(sum(rank_algo) / (max(rank_launch_ms) / 1e3) / 1e9
                                            / (HBM_PEAK_GBS * world), 4),
                "traffic_source": ("PMC FETCH_SIZE (x2, the gfx950 correction) + WRITE_SIZE per launch from "
                                   f"{prof['source']}: separate rocprofv3 --pmc passes over this bench command, "
                                   "not measured in this run") if prof else None,
                "profile": prof,
            },
            "timing": {
                "prewarm": warm,
                "warmup_step_ms": [round(x, 4) for x in warm_steps],
                "step_ms": [round(x, 4) for x in step_ms],
                "step_ms_min": round(min(step_ms), 4),
                "step_ms_median": round(sorted(step_ms)[len(step_ms) // 2], 4),
                "step_ms_max": round(max(step_ms), 4),
                "note": "HIP events around each execute() on the launch stream (device ms); prewarm = the "
                        "time-based sweep steps run before the counted warm-up (a fresh lease starts at idle "
                        "clocks), not part of the timed steps",
                "telemetry": [tele_start] + tele + [telemetry.sample("end_of_bench")],
            },
            "memory_pattern_probe": {
                "lds_dma_GBs": probe_lds, "vgpr_stream_GBs": probe_stream,
                "note": "the sweep's read 4 B / write 9 B per element pattern without arithmetic, on this box after "
                        "the timed steps.  NOT a ceiling: box to box it lands 5.2-6.5 TB/s, sometimes below the "
                        "sweep itself, so it only shows how far arithmetic and row logic cost on this box"},
            "parity": parity,
            "sharded_gathers": gathers,
            "weak_scaling": weak,
            "configs4_sharded": sharded4,
            "cpu_baseline": cpu,
            "secondary_configs": second,
            "single_model_latency": single,
            "sharded_single_model": sharded,
            "pipeline_ms": pipe,
            "cle_roofline": cle_roof,
            "top1_delta": None,
            "notes": "top-1 needs ImageNet-val + the pretrained checkpoint (absent offline); weight outputs are "
                     "bit-exact with the reference CPU path (tests/test_gpu_pipeline.py)",
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return res


if __name__ == "__main__":
    rc = main()
    sys.exit(rc if isinstance(rc, int) else 0)
