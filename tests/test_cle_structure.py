"""The CLE plan structure's index invariants, checked on the host (no GPU):
dfq_diag_cle_check_structure (libdfq_diag.so, dfq_cle.hip) builds exactly what
dfq_cle_plan_create builds -- chains, rescale / range tasks, metric chunks and
units, the lagged placement and the stop rule's offset -- and checks every index
the loop's kernels derive from it: task spans inside their relation's shapes,
range words and rollback saves inside their tables, each tensor's tiles and ranges
inside its window between two iterations' rescales, the stop rule after its
iteration's tiles and before the next iteration's (the round-5
illegal access of a development tree of the lagged schedule).

Relations come from the real host graph code (create_relation on the zoo models)
or from fuzzed layer chains; tensor addresses are stand-ins (one per module and
field, as the device tensors are distinct) -- the planner only compares them.
Every schedule switch of the diagnostics library is covered."""
import ctypes as C
import random

import numpy as np
import pytest
import torch.nn as nn

from data_free_quantization_amd import _lib, zoo
from data_free_quantization_amd.utils.relation import create_relation
from data_free_quantization_amd.utils.tracer import build_graph

TARG = (nn.Conv2d, nn.Linear)
SCHEDULES = {
    "product": {},
    "no_lag": {"DFQ_CLE_LAG": "0"},
    "unfused": {"DFQ_CLE_FUSED": "0"},
    "band0": {"DFQ_CLE_BAND": "0"},
    "band1": {"DFQ_CLE_BAND": "1"},
    "band2": {"DFQ_CLE_BAND": "2"},
    "stop_arrival": {"DFQ_CLE_STOP": "arrival"},
}
SWITCHES = ("DFQ_CLE_LAG", "DFQ_CLE_FUSED", "DFQ_CLE_BAND", "DFQ_CLE_STOP")


class _Addr:
    """Stand-in device addresses: one 4 KB-aligned address per (object, field)."""

    def __init__(self):
        self.map = {}

    def __call__(self, obj, field):
        k = (id(obj), field)
        if k not in self.map:
            self.map[k] = 0x7f0000000000 + 4096 * (len(self.map) + 1)
        return self.map[k]


def _check(rows, targets, target_n, threads=8):
    L = _lib.load_diag()
    n = len(rows)
    descs = (_lib.CleRel * max(n, 1))()
    for i, r in enumerate(rows):
        descs[i] = _lib.CleRel(*r)
    nt = len(targets)
    tp = (C.c_void_p * max(nt, 1))(*targets)
    tn = (C.c_int64 * max(nt, 1))(*target_n)
    info = (C.c_int64 * 8)()
    msg = C.create_string_buffer(512)
    rc = L.dfq_diag_cle_check_structure(descs, n, tp, tn, nt, threads, info, msg, 512)
    return rc, list(info), msg.value.decode()


def _model_rows(name):
    model = zoo.build(name, seed=0, relu=True)
    g = build_graph(model, "positional")
    graph, bottoms = g.getGraph(), g.getBottoms()
    rels = create_relation(graph, bottoms, TARG)
    A = _Addr()
    rows = []
    for r in rels:
        l1, l2, bn = graph[r.layer_first], graph[r.layer_second], graph[r.bn_idx]
        w1, w2 = l1.weight, l2.weight
        c1 = w1.shape[0]
        khw2 = w2.numel() // (w2.shape[0] * w2.shape[1])
        rows.append((A(l1, "w"), A(l2, "w"), A(l1, "b"), A(bn, "fw"), A(bn, "fb"), A(r, "S"), c1, w1.numel() // c1,
                     w2.shape[0], w2.shape[1], khw2, 1, 0))
    tmods = [m for m in graph.values() if type(m) in TARG]
    return rows, [A(m, "w") for m in tmods], [m.weight.numel() for m in tmods]


@pytest.fixture
def schedule_env(monkeypatch):
    def set_(env):
        for k in SWITCHES:
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
    return set_


@pytest.mark.parametrize("name", ["mobilenetv2", "resnet50", "deeplab", "resnet18"])
def test_zoo_plan_structures(name, schedule_env):
    rows, targets, tn = _model_rows(name)
    seen = {}
    for tag, env in SCHEDULES.items():
        schedule_env(env)
        for threads in (1, 8, 16):
            rc, info, msg = _check(rows, targets, tn, threads)
            assert rc == _lib.DFQ_OK, (name, tag, threads, msg)
        seen[tag] = info
    # the product schedule is what DESIGN.md states: MobileNetV2 lagged (3 launches
    # per iteration), ResNet-50 not (a tensor rescaled at both of its 2 steps)
    if name == "mobilenetv2":
        assert seen["product"][:3] == [3, 3, 1], seen["product"]
        assert seen["no_lag"][:3] == [3, 4, 0]
    if name == "resnet50":
        assert seen["product"][:3] == [2, 3, 0], seen["product"]


def _fuzz_rows(rng):
    """A random chain of conv layers (regular 1x1 / 3x3 or depthwise 3x3, random
    widths) with a random subset of consecutive pairs as relations -- chains of
    every length, depthwise pairs, tensors rescaled at two steps -- in graph order or
    shuffled (the planner keeps the order of relations touching a tensor)."""
    n_layers = rng.randint(2, 14)
    A = _Addr()
    layers = []
    ch = rng.choice([3, 8, 16, 32])
    for i in range(n_layers):
        kind = rng.choice(["pw", "pw", "k3", "dw"]) if i else rng.choice(["pw", "k3"])
        if kind == "dw":
            out, shape = ch, (ch, 1, 3, 3)
        else:
            out = rng.choice([8, 16, 24, 48, 96, 160])
            shape = (out, ch, 3, 3) if kind == "k3" else (out, ch, 1, 1)
        layers.append((object(), shape, kind))
        ch = out
    rels = []
    for i in range(n_layers - 1):
        if rng.random() < 0.75:
            (o1, s1, _), (o2, s2, _) = layers[i], layers[i + 1]
            c1 = s1[0]
            rels.append((A(o1, "w"), A(o2, "w"), A(o1, "b"), A(o1, "bnw"), A(o1, "bnb"), A(o1, "S"), c1,
                         int(np.prod(s1)) // c1, s2[0], s2[1], s2[2] * s2[3], 1, 0))
    if rels and rng.random() < 0.3:
        rng.shuffle(rels)
    return rels, [A(o, "w") for o, _, _ in layers], [int(np.prod(s)) for _, s, _ in layers]


@pytest.mark.parametrize("seed", range(60))
def test_fuzzed_plan_structures(seed, schedule_env):
    rng = random.Random(seed)
    rows, targets, tn = _fuzz_rows(rng)
    if not rows:
        return
    for tag, env in SCHEDULES.items():
        schedule_env(env)
        rc, info, msg = _check(rows, targets, tn, rng.choice([1, 8, 16]))
        assert rc == _lib.DFQ_OK, (seed, tag, msg, rows)
