"""Drop-in for the reference's ``Cross_layer_equal.py`` (Cross_layer_equal.py:1-116).

``_layer_equalization`` runs one relation as HIP kernels (channel-parallel
ranges + rescale, bit-exact with the reference's sequential channel loop);
``cross_layer_equalization`` runs the reference's loop and stop rule on the
device (``dfq_cle_plan``); the metric is exact (fp32 torch.mean in ATen's order,
then numpy's pairwise float64 sum), so the iteration count and every weight match
the reference.
"""
from __future__ import annotations

import atexit
from collections.abc import MutableMapping
import ctypes as C
import os
import sys
import time
import warnings

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .utils.relation import Relation

class _LastRun(MutableMapping):
    """LAST_RUN: a dict whose reads first wait for a launched (asynchronous) loop."""

    def __init__(self):
        self._d = {}

    def __getitem__(self, k):
        wait()
        return self._d[k]

    def __setitem__(self, k, v):
        self._d[k] = v

    def __delitem__(self, k):
        del self._d[k]

    def __iter__(self):
        wait()
        return iter(self._d)

    def __len__(self):
        wait()
        return len(self._d)

    def clear(self):
        self._d.clear()

    def update(self, *a, **k):
        self._d.update(*a, **k)

    def __repr__(self):
        wait()
        return repr(self._d)


#: statistics of the last cross_layer_equalization call (extension, for tests/bench)
LAST_RUN = _LastRun()

#: Default of ``cross_layer_equalization(..., launch=None)``.  False (the
#: reference's contract): the call blocks until the loop is done and raises its
#: errors.  True: the device loop runs asynchronously (dfq_cle_plan_launch): the
#: call returns once the loop is under way, and whatever the caller enqueues on the
#: device's CURRENT stream afterwards waits for it in the device (work on any other
#: stream is not ordered behind it) -- the next stages' host work overlaps the
#: loop.  ``wait()`` (or reading LAST_RUN) joins it and raises its error.
#: run_dfq and main_dfq opt in (launch=True) and call wait() at their end.
ASYNC = False
_PENDING = None   # (plan, workspace, host times) of the launched loop
_ABANDONED = []   # (plan, workspace) of launched loops join gave up on: their worker may still use both


def _layer_equalization(W1, W2, B1, Batnorm_weight=None, Batnorm_bias=None, s_min_max=(1e-8, 1e8), signed=False,
                        eps=0, S_acc=None):
    """Equalize the output channels of W1 with the input channels of W2, in place.
    Returns (W1, W2, B1, S).  ``S_acc`` (extension): a [C] device tensor the scales
    are multiplied into (``None``: not accumulated)."""
    _lib.require_device(W1, W2, B1, Batnorm_weight, Batnorm_bias)
    c1 = W1.shape[0]
    o2, i2 = W2.shape[0], W2.shape[1]
    S = torch.empty(c1, dtype=torch.float32, device=W1.device)
    L = _lib.load()
    ws_bytes = L.dfq_cle_ws_bytes(c1)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=W1.device)
    rc = L.dfq_cle_relation(
        _lib.ptr(W1), _lib.ptr(W2), _lib.ptr(B1), _lib.ptr(Batnorm_weight), _lib.ptr(Batnorm_bias), c1,
        W1.numel() // c1, o2, i2, W2.numel() // (o2 * i2), float(s_min_max[0]), float(s_min_max[1]),
        int(bool(signed)), float(eps), _lib.ptr(S), _lib.ptr(S_acc), 0, C.c_void_p(ws.data_ptr()), ws_bytes,
        _lib.stream_of(W1))
    _lib.check(rc, "dfq_cle_relation")
    return W1, W2, B1, S


class _DiffPlan:
    """mean|W - W_old| per target layer, snapshot kept on the device."""

    def __init__(self, weights):
        self.weights = weights
        self.snaps = [torch.empty_like(w) for w in weights]
        n = len(weights)
        L = _lib.load()
        wp = (C.c_void_p * max(n, 1))(*[w.data_ptr() for w in weights])
        sp = (C.c_void_p * max(n, 1))(*[s.data_ptr() for s in self.snaps])
        ns = (C.c_int64 * max(n, 1))(*[w.numel() for w in weights])
        self._plan = C.c_void_p()
        _lib.check(L.dfq_diff_plan_create(wp, sp, ns, n, C.byref(self._plan)), "dfq_diff_plan_create")
        self._out = (C.c_double * max(n, 1))()
        self._dev = weights[0].device if weights else None

    def snapshot(self):
        _lib.check(_lib.load().dfq_diff_plan_snapshot(self._plan, _lib.stream_of(self.weights[0])),
                   "dfq_diff_plan_snapshot")

    def diffs(self):
        _lib.check(_lib.load().dfq_diff_plan_execute(self._plan, self._out, _lib.stream_of(self.weights[0])),
                   "dfq_diff_plan_execute")
        return [float(self._out[i]) for i in range(len(self.weights))]

    def close(self):
        if self._plan is not None:
            _lib.load().dfq_diff_plan_destroy(self._plan)
            self._plan = None


#: iteration cap of the device loop (the reference's loop has none; a run that
#: reaches it warns).  A LAUNCHED run (launch=True) is also bounded in time: it
#: stops enqueueing iterations after 60 s and fails at join, well before the
#: caller's stream gate traps at 120 s (dfq_cle.hip, kCleGateSeconds /
#: kCleLaunchDeadlineUs); a blocking run has no time bound.
MAX_ITERS = int(os.environ.get("DFQ_CLE_MAX_ITERS", "100000"))
#: measurement: blocking device runs record the loop's device time (one HIP event
#: pair on its stream; LAST_RUN["device_ms"]); bench.py's cle_roofline sets it
DEVICE_TIMING = False
_TIMING = bool(os.environ.get("DFQ_CLE_TIMING"))   # host-side split of create (stderr)


def cross_layer_equalization(graph, relations, Target_list, s_min_max=[1e-8, 1e8], Treshhold=2e-7, Count=20,
                             signed=False, eps=0, Save_state=True, *, launch=None):
    """Iterate the relations until the summed mean weight change is <= Treshhold
    or it stayed within 1e-9 for ``Count`` iterations (Cross_layer_equal.py:81-115).

    The loop runs on the device (``dfq_cle_plan``): relations grouped into
    independent chains, the metric (fp32 torch.mean order + numpy's pairwise sum)
    and the stop rule evaluated by the GPU.  ``DFQ_CLE_MODE=host`` keeps the
    relation-by-relation host loop (one C call per relation, metric read back
    every iteration) for comparison.

    ``launch`` (extension, keyword-only; None: module ``ASYNC``, False by
    default): True returns as soon as the loop is under way; only the device's
    current stream is ordered behind it, and its errors surface at ``wait()``."""
    print("Cross layer equalization")
    _lib.weights_changed()
    if Save_state:
        warnings.warn("Save_state plots (ourplots.save_layer) are visualization, not part of the weight path; "
                      "skipped")
    wait()   # a launched loop before this one (one at a time)
    with torch.no_grad():
        if os.environ.get("DFQ_CLE_MODE", "device") == "host":
            _cle_host_loop(graph, relations, Target_list, s_min_max, Treshhold, Count, signed, eps)
        else:
            _cle_device_loop(graph, relations, Target_list, s_min_max, Treshhold, Count, signed, eps,
                             ASYNC if launch is None else bool(launch))


_CLE_REL = np.dtype([("w1", "<u8"), ("w2", "<u8"), ("b1", "<u8"), ("bn_w", "<u8"), ("bn_b", "<u8"), ("s_acc", "<u8"),
                     ("c1", "<i8"), ("len1", "<i8"), ("o2", "<i8"), ("i2", "<i8"), ("khw2", "<i8"),
                     ("s_acc_init", "<i4"), ("reserved", "<i4")])
assert _CLE_REL.itemsize == C.sizeof(_lib.CleRel)


def _state(m, name):
    """A module's registered buffer ``name`` without Module.__getattr__ (any other
    object, or a plain attribute: getattr)."""
    b = getattr(m, "_buffers", None)
    if b is not None and name in b:
        return b[name]
    return getattr(m, name, None)


def _tensor_info(t, memo):
    """(data_ptr, shape, numel) of a weight, checked like _lib.require_device once
    per tensor (every relation weight is also a target, and a relation's W2 is the
    next one's W1): the per-tensor property calls were a good part of plan
    creation's host time."""
    k = id(t)
    r = memo.get(k)
    if r is None:
        r = memo[k] = (_checked_ptr(t), t.shape, t.numel())
    return r


def _checked_ptr(t):
    """data_ptr of a tensor the loop reads or writes, checked like _lib.require_device."""
    if not (t.is_cuda and t.dtype is _F32 and t.is_contiguous()):
        _lib.require_device(t)   # raises the reference-style error
    return t.data_ptr()


_F32 = torch.float32


class _DescTemplate:
    """What the relation descriptors of one graph STRUCTURE need besides addresses:
    the target keys, each relation's (first, bn) keys and the target indices of its
    W1 / W2, the shape columns of the table, and the targets' sizes.  Keyed by
    (target keys, relation key triples) and checked against the live targets'
    shapes, so a fresh model of a seen architecture describes its relations by
    gathering addresses only (MobileNetV2 on a GPU box: 193 us of Python per plan
    before; scripts/cle_create_split.py)."""
    __slots__ = ("shapes", "first", "bn", "idx1", "idx2", "tab", "tn", "nt", "c1", "s_off", "s_total")

    def __init__(self, tkeys, rk, targets, shapes):
        pos = {k: i for i, k in enumerate(tkeys)}
        self.shapes = shapes
        self.first = [f for f, _, _ in rk]
        self.bn = [b for _, _, b in rk]
        self.idx1 = np.array([pos[f] for f, _, _ in rk], dtype=np.int64)
        self.idx2 = np.array([pos[s] for _, s, _ in rk], dtype=np.int64)
        n = len(rk)
        self.tab = np.zeros(max(n, 1), dtype=_CLE_REL)
        numel = [t.numel() for t in targets]
        for j, (i1, i2) in enumerate(zip(self.idx1, self.idx2)):
            s1, s2 = shapes[i1], shapes[i2]
            self.tab[j] = (0, 0, 0, 0, 0, 0, s1[0], numel[i1] // s1[0], s2[0], s2[1], numel[i2] // (s2[0] * s2[1]),
                           1, 0)
        self.nt = len(targets)
        self.tn = (C.c_int64 * max(self.nt, 1))(*numel)
        self.c1 = [int(shapes[i][0]) for i in self.idx1]
        self.s_off = np.concatenate([[0], np.cumsum(self.c1)[:-1]]).astype(np.uint64) if n else np.zeros(0, np.uint64)
        self.s_total = int(sum(self.c1))


_DESC_CACHE: "dict" = {}


def _describe_fast(graph, relations, tl):
    """The descriptor table through a cached _DescTemplate; None when this call
    needs the general path (a relation layer outside the targets, a missing bias
    the loop must create, a Relation.S already set, a non-Relation object)."""
    tkeys = tuple(k for k, v in graph.items() if type(v) in tl)
    try:
        rk = tuple((r.layer_first, r.layer_second, r.bn_idx) for r in relations)
    except AttributeError:
        return None
    if not all(type(r) is Relation and r._S is None and r._S_lazy is None for r in relations):
        return None
    targets = [graph[k]._parameters["weight"] for k in tkeys]
    shapes = [t.shape for t in targets]
    key = (tkeys, rk)
    tpl = _DESC_CACHE.get(key)
    if tpl is None or tpl.shapes != shapes:
        try:
            tpl = _DescTemplate(tkeys, rk, targets, shapes)
        except KeyError:   # a relation layer that is not a target
            return None
        if len(_DESC_CACHE) >= 8:
            _DESC_CACHE.pop(next(iter(_DESC_CACHE)))
        _DESC_CACHE[key] = tpl
    tptr = np.array([_checked_ptr(t) for t in targets], dtype=np.uint64)
    bias = [graph[f]._parameters.get("bias") for f in tpl.first]
    if any(b is None for b in bias):
        return None
    bw, bb = [], []
    for k in tpl.bn:
        m = graph[k]
        bw.append(_state(m, "fake_weight"))
        bb.append(_state(m, "fake_bias"))
    tab = tpl.tab.copy()
    n = len(rk)
    if n:
        tab["w1"] = tptr[tpl.idx1]
        tab["w2"] = tptr[tpl.idx2]
        tab["b1"] = [_checked_ptr(b) for b in bias]
        tab["bn_w"] = [0 if t is None else _checked_ptr(t) for t in bw]
        tab["bn_b"] = [0 if t is None else _checked_ptr(t) for t in bb]
        # every Relation.S new: one allocation, handed out as lazy slices
        flat = torch.empty(tpl.s_total, dtype=torch.float32, device=targets[0].device)
        tab["s_acc"] = np.uint64(flat.data_ptr()) + np.uint64(4) * tpl.s_off
        for r, o, c in zip(relations, tpl.s_off.tolist(), tpl.c1):
            r._S_lazy = (flat, o, o + c)
    return targets, tab, tptr, tpl


def _create_plan(graph, relations, Target_list, s_min_max, signed, eps):
    """dfq_cle_plan_create over the relations' tensors; returns (plan, workspace,
    device).  The workspace (W_prev snapshots, torch's caching allocator) must
    outlive the plan."""
    # module state straight from the parameter / buffer dicts (Module.__getattr__
    # per access was a good part of this host time)
    tc = [time.perf_counter()] if _TIMING else None
    tl = tuple(Target_list)
    fast = _describe_fast(graph, relations, tl)
    if fast is not None:
        targets, tab, tptr, tpl = fast
        n = len(relations)
        if tc:
            tc.append(time.perf_counter())
        descs = tab.ctypes.data_as(C.POINTER(_lib.CleRel))
        nt = tpl.nt
        tp = (C.c_void_p * max(nt, 1))(*tptr.tolist())
        tn = tpl.tn
        return _plan_from_table(descs, n, tp, tn, nt, targets, tab, s_min_max, signed, eps, tc)
    targets = [v._parameters["weight"] for v in graph.values() if type(v) in tl]
    memo = {}
    tinfo = [_tensor_info(t, memo) for t in targets]
    n = len(relations)
    rows = []
    fresh = []   # relations whose S the loop creates: views of one allocation, carved below
    for rel in relations:
        first, second, bn_idx = rel.layer_first, rel.layer_second, rel.bn_idx
        l1, l2 = graph[first], graph[second]
        p1 = l1._parameters
        if p1.get("bias") is None:   # :93-94
            l1.bias = nn.Parameter(torch.zeros(p1["weight"].size(0), dtype=torch.float32, device=p1["weight"].device),
                                   requires_grad=False)
        bn = graph[bn_idx]
        W1 = p1["weight"]
        bnw, bnb = _state(bn, "fake_weight"), _state(bn, "fake_bias")
        w1p, s1, n1 = _tensor_info(W1, memo)
        w2p, s2, n2 = _tensor_info(l2._parameters["weight"], memo)
        init = not rel._has_S() if isinstance(rel, Relation) else rel.S is None
        if init:
            fresh.append((len(rows), rel, s1[0]))
        rows.append([w1p, w2p, _checked_ptr(p1["bias"]), 0 if bnw is None else _checked_ptr(bnw),
                     0 if bnb is None else _checked_ptr(bnb), 0 if init else rel.S.data_ptr(), s1[0],
                     n1 // s1[0], s2[0], s2[1], n2 // (s2[0] * s2[1]), 1 if init else 0, 0])
    if fresh:   # one allocation for every new Relation.S (a torch.empty per relation cost ~7 us each),
        # handed out as lazy slices (Relation.S: the view is made on first read)
        flat = torch.empty(sum(c for _, _, c in fresh), dtype=torch.float32, device=targets[0].device)
        base, off = flat.data_ptr(), 0
        for j, rel, c in fresh:
            if isinstance(rel, Relation):
                rel._set_S_lazy(flat, off, off + c)
            else:
                rel.S = flat[off:off + c]
            rows[j][5] = base + 4 * off
            off += c
    rows = [tuple(r) for r in rows]
    if tc:
        tc.append(time.perf_counter())
    # the descriptor table as a numpy record array (layout of _lib.CleRel), one row per
    # relation from plain tuples instead of ctypes field by field
    tab = np.array(rows if rows else [(0,) * 13], dtype=_CLE_REL)
    descs = tab.ctypes.data_as(C.POINTER(_lib.CleRel))
    nt = len(targets)
    tp = (C.c_void_p * max(nt, 1))(*[i[0] for i in tinfo])
    tn = (C.c_int64 * max(nt, 1))(*[i[2] for i in tinfo])
    return _plan_from_table(descs, n, tp, tn, nt, targets, tab, s_min_max, signed, eps, tc)


def _plan_from_table(descs, n, tp, tn, nt, targets, tab, s_min_max, signed, eps, tc):
    """The workspace and the dfq_cle_plan_create call (``tab`` backs ``descs``)."""
    L = _lib.load()
    dev = targets[0].device if targets else torch.device("cuda", torch.cuda.current_device())
    # W_prev snapshots from torch's caching allocator (no hipMalloc / hipFree per call)
    ws_bytes = int(L.dfq_cle_plan_ws_bytes(tn, nt))
    if ws_bytes < 0:
        raise RuntimeError("dfq_cle_plan_ws_bytes: invalid target sizes")
    ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=dev)
    if tc:
        tc.append(time.perf_counter())
    plan = C.c_void_p()
    _lib.check(L.dfq_cle_plan_create(descs, n, tp, tn, nt, float(s_min_max[0]), float(s_min_max[1]),
                                     int(bool(signed)), float(eps), _lib.REF_THREADS, ws.data_ptr(), ws.numel(),
                                     C.byref(plan)),
               "dfq_cle_plan_create", RuntimeError)
    if tc:
        tc.append(time.perf_counter())
        print("DFQ_CLE_TIMING python create: relations %.1f us, tables + workspace %.1f us, plan_create %.1f us"
              % tuple((b - a) * 1e6 for a, b in zip(tc, tc[1:])), file=sys.stderr)
    return plan, ws, dev


def _plan_stats(plan):
    """dfq_cle_plan_stats: algorithmic HBM bytes of one iteration (rescale, metric,
    ranges), the last run's device milliseconds (DEVICE_TIMING runs; else None) and
    the iteration groups it enqueued."""
    b, ms, n = (C.c_int64 * 3)(), C.c_double(-1.0), C.c_int32(0)
    _lib.check(_lib.load().dfq_cle_plan_stats(plan, b, C.byref(ms), C.byref(n)), "dfq_cle_plan_stats")
    return {"bytes_per_iteration": {"rescale": b[0], "metric": b[1], "ranges": b[2], "total": b[0] + b[1] + b[2]},
            "device_ms": ms.value if ms.value >= 0 else None, "iterations_launched": n.value}


def _run_plan(plan, dev, Treshhold, Count):
    """dfq_cle_plan_run; returns (iterations, diffs, (chains, steps, launches per iteration), stats)."""
    L = _lib.load()
    iters = C.c_int32(0)
    hist = _hist_buffer()
    stream = _lib.raw_stream(dev)
    if DEVICE_TIMING:
        _lib.check(L.dfq_cle_plan_set_timing(plan, 1), "dfq_cle_plan_set_timing")
    _lib.check(L.dfq_cle_plan_run(plan, float(Treshhold), int(Count), MAX_ITERS, C.byref(iters), hist, stream),
               "dfq_cle_plan_run")
    chains, steps, launches = C.c_int32(0), C.c_int32(0), C.c_int32(0)
    L.dfq_cle_plan_info(plan, C.byref(chains), C.byref(steps), C.byref(launches))
    return (iters.value, [hist[i] for i in range(iters.value)], (chains.value, steps.value, launches.value),
            _plan_stats(plan))


def wait():
    """Wait for the launched CLE loop, if any: fills LAST_RUN and raises the loop's
    error (a HIP failure in the worker).  Called by every LAST_RUN read, by the
    next cross_layer_equalization, by run_dfq / main_dfq at their end and at exit."""
    global _PENDING
    pend = _PENDING
    if pend is None:
        return
    _PENDING = None
    plan, ws, host = pend
    L = _lib.load()
    iters = C.c_int32(0)
    hist = _hist_buffer()
    t0 = time.perf_counter()
    rc = L.dfq_cle_plan_join(plan, C.byref(iters), hist)
    if rc != _lib.DFQ_OK and "did not finish" in L.dfq_last_hip_error().decode():
        # the loop is still running (the caller's stream stays held behind its
        # gate): its plan and snapshot workspace must outlive it
        _ABANDONED.append((plan, ws))
        _lib.check(rc, "cross_layer_equalization (device loop)")
    try:
        _lib.check(rc, "cross_layer_equalization (device loop)")
        chains, steps, launches = C.c_int32(0), C.c_int32(0), C.c_int32(0)
        L.dfq_cle_plan_info(plan, C.byref(chains), C.byref(steps), C.byref(launches))
        stats = _plan_stats(plan)
    finally:
        L.dfq_cle_plan_destroy(plan)
        del ws
    n = iters.value
    if n >= MAX_ITERS:
        warnings.warn(f"cross_layer_equalization stopped at DFQ_CLE_MAX_ITERS={MAX_ITERS} iterations")
    LAST_RUN.clear()
    LAST_RUN.update(iterations=n, diffs=[hist[i] for i in range(n)], chains=chains.value, steps=steps.value,
                    launches_per_iteration=launches.value, mode="device", launched=True,
                    host_ms=dict(host, wait=(time.perf_counter() - t0) * 1e3), **stats)


def _at_exit():
    """A launched loop nobody joined: join it; its failure must not end the
    process with status 0 (the weights it was rescaling are not to be trusted)."""
    try:
        wait()
    except Exception as e:   # noqa: BLE001 -- the interpreter is going down
        import sys
        print(f"cross_layer_equalization (launched, never joined) failed: {e}", file=sys.stderr, flush=True)
        os._exit(1)


atexit.register(_at_exit)


def _cle_device_loop(graph, relations, Target_list, s_min_max, Treshhold, Count, signed, eps, launch):
    global _PENDING
    wait()   # one launched loop at a time
    t0 = time.perf_counter()
    plan, ws, dev = _create_plan(graph, relations, Target_list, s_min_max, signed, eps)
    t2 = time.perf_counter()
    if launch:
        L = _lib.load()
        stream = _lib.raw_stream(dev)
        t5 = time.perf_counter()
        rc = L.dfq_cle_plan_launch(plan, float(Treshhold), int(Count), MAX_ITERS, stream)
        if _TIMING:
            print("DFQ_CLE_TIMING python launch: stream %.1f us, plan_launch %.1f us"
                  % ((t5 - t2) * 1e6, (time.perf_counter() - t5) * 1e6), file=sys.stderr)
        if rc == _lib.DFQ_OK:
            _PENDING = (plan, ws, {"create": (t2 - t0) * 1e3, "launch": (time.perf_counter() - t2) * 1e3})
            LAST_RUN.clear()
            return
        if rc != _lib.DFQ_ERR_UNSUPPORTED:   # else: the device cannot wait on a value -- blocking run
            L.dfq_cle_plan_destroy(plan)
            _lib.check(rc, "dfq_cle_plan_launch")
    try:
        iters, diffs, (chains, steps, launches), stats = _run_plan(plan, dev, Treshhold, Count)
    finally:
        t3 = time.perf_counter()
        _lib.load().dfq_cle_plan_destroy(plan)
    t4 = time.perf_counter()
    if iters >= MAX_ITERS:
        warnings.warn(f"cross_layer_equalization stopped at DFQ_CLE_MAX_ITERS={MAX_ITERS} iterations")
    LAST_RUN.clear()
    LAST_RUN.update(iterations=iters, diffs=diffs, chains=chains, steps=steps, launches_per_iteration=launches,
                    mode="device", launched=False, host_ms={"create": (t2 - t0) * 1e3, "run": (t3 - t2) * 1e3,
                                            "destroy": (t4 - t3) * 1e3}, **stats)


_HIST = None


def _hist_buffer():
    """The iteration history buffer handed to dfq_cle_plan_run (MAX_ITERS + 1
    doubles), allocated once per process instead of once per call."""
    global _HIST
    if _HIST is None or len(_HIST) != MAX_ITERS + 1:
        _HIST = (C.c_double * (MAX_ITERS + 1))()
    return _HIST


def _cle_host_loop(graph, relations, Target_list, s_min_max, Treshhold, Count, signed, eps):
    targets = [graph[k] for k in graph if type(graph[k]) in Target_list]
    plan = _DiffPlan([t.weight.data for t in targets]) if targets else None
    diff = 1e8
    iter_count = 0
    history = []
    iters = 0
    try:
        if plan is not None:
            plan.snapshot()
        while diff > Treshhold and iter_count < Count:
            for rel in relations:
                first, second, bn_idx = rel.get_idxs()
                l1, l2 = graph[first], graph[second]
                if l1.bias is None:   # :93-94
                    l1.bias = nn.Parameter(torch.zeros(l1.weight.size(0), dtype=torch.float32,
                                                       device=l1.weight.device), requires_grad=False)
                bn = graph[bn_idx]
                first_time = rel.S is None
                if first_time:
                    rel.S = torch.empty(l1.weight.size(0), dtype=torch.float32, device=l1.weight.device)
                _cle_into(l1.weight.data, l2.weight.data, l1.bias.data, bn.fake_weight, bn.fake_bias,
                          s_min_max, signed, eps, rel.S, first_time)
            diff_list = plan.diffs() if plan is not None else []
            diff_tmp = np.sum(diff_list)
            history.append(float(diff_tmp))
            iters += 1
            if abs(diff - diff_tmp) > 1e-9:
                iter_count = 0
                diff = diff_tmp
            else:
                iter_count += 1
    finally:
        if plan is not None:
            plan.close()
    LAST_RUN.clear()
    LAST_RUN.update(iterations=iters, diffs=history, mode="host")


def _cle_into(W1, W2, B1, bnw, bnb, s_min_max, signed, eps, S_acc, first_time):
    c1 = W1.shape[0]
    o2, i2 = W2.shape[0], W2.shape[1]
    L = _lib.load()
    ws_bytes = L.dfq_cle_ws_bytes(c1)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=W1.device)
    rc = L.dfq_cle_relation(
        _lib.ptr(W1), _lib.ptr(W2), _lib.ptr(B1), _lib.ptr(bnw), _lib.ptr(bnb), c1, W1.numel() // c1, o2, i2,
        W2.numel() // (o2 * i2), float(s_min_max[0]), float(s_min_max[1]), int(bool(signed)), float(eps), None,
        _lib.ptr(S_acc), 1 if first_time else 0, C.c_void_p(ws.data_ptr()), ws_bytes, _lib.stream_of(W1))
    _lib.check(rc, "dfq_cle_relation")
