"""dfq_bc_chain's one-launch path (diagnostics A/B DFQ_BC_CHAIN=coop: phases
split by grid barriers, expectations forwarded through LDS, propagates
recomputed from E) against the product's per-op launches, bit for bit, on
synthetic walks shaped like bias_correction.py:147-258's (expect -> apply ->
propagate into the next BN's fake_bias, 'add' branches accumulating, two
branches of one layer, depthwise and scalar broadcasts, before / after
snapshots).  The per-op path itself is pinned to the reference's fixtures in
test_gpu_transforms.py; the real walks of MobileNetV2 / ResNet-50 / DeepLab in
test_gpu_pipeline.py."""
import ctypes as C
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class Walk:
    """Device buffers + an op list, rebuilt identically from a seed."""

    def __init__(self, seed, layers=6, width=(24, 96), big_expect=False, alias=False, grouped=False, scratch=False):
        g = np.random.default_rng(seed)
        self.t = {}
        self.ops = []
        ch = [int(g.integers(*width)) for _ in range(layers + 1)]
        if grouped:   # depthwise layers: as many outputs as inputs
            for l in range(layers):
                if l % 3 == 2:
                    ch[l + 1] = ch[l]
        if big_expect:
            ch[1] = 9000   # larger than the LDS expectation slots: the whole chain takes the per-op path
        for l in range(layers + 1):
            self.vec(f"fw{l}", g.uniform(0.2, 2.0, ch[l]))
            self.vec(f"fb{l}", g.normal(0, 1, ch[l]))
        for l in range(layers):
            o, i = ch[l + 1], ch[l]
            dw = grouped and l % 3 == 2 and o == i
            i2 = 1 if dw else i
            self.vec(f"E{l}", g.normal(0, 0.01, o * i2))
            self.vec(f"bias{l}", g.normal(0, 0.1, o))
        self.layers, self.ch = layers, ch
        # before-snapshot copies
        for l in range(layers):
            self.vec(f"snap{l}", np.zeros(ch[l + 1]))
            self.op(3, 0, f"bias{l}", None, f"snap{l}", None, ch[l + 1])
        for l in range(layers):
            o, i = ch[l + 1], ch[l]
            i2 = self.t[f"E{l}"].numel() // o
            self.vec(f"ex{l}", np.zeros(i))
            relu = int(g.integers(0, 2))
            self.op(0, relu, f"fw{l}", f"fb{l}", f"ex{l}", None, i)
            if l >= 2 and ch[l - 2] == i and g.random() < 0.6:   # an 'add' branch: accumulate
                self.op(0, 1 | 2, f"fw{l - 2}", f"fb{l - 2}", f"ex{l}", None, i)
            f = i
            bcols = i2 if (i2 == f or f == 1) else f
            self.vec(f"vec{l}", np.zeros(o * bcols))
            self.op(1, int(scratch), f"E{l}", f"ex{l}", f"bias{l}", f"vec{l}", o, i2, f)
            if g.random() < 0.3 and i2 > 1:   # a second branch of the same layer: same bias, same row owners
                self.vec(f"exb{l}", np.zeros(1))
                self.op(0, 0, f"fw{l}", f"fb{l}", f"exb{l}", None, 1)
                self.vec(f"vecb{l}", np.zeros(o * i2))
                self.op(1, int(scratch), f"E{l}", f"exb{l}", f"bias{l}", f"vecb{l}", o, i2, 1)
                last = f"vecb{l}"
                numel = o * i2
            else:
                last, numel = f"vec{l}", o * bcols
            nxt = ch[l + 1]
            if numel % nxt == 0 and numel != nxt:
                self.op(2, 8, last, None, f"fb{l + 1}", None, numel, 0, nxt)
        if alias:   # an expectation written over its own fake_bias input
            self.op(0, 1, f"fw{layers}", f"fb{layers}", f"fb{layers}", None, ch[layers])
        for l in range(layers):
            self.vec(f"after{l}", np.zeros(ch[l + 1]))
            self.op(3, 0, f"bias{l}", None, f"after{l}", None, ch[l + 1])

    def vec(self, name, a):
        self.t[name] = torch.from_numpy(np.asarray(a, np.float32)).to(DEV)

    def op(self, kind, flag, a, b, out, out2, n, i2=0, f=0):
        self.ops.append((kind, flag, a, b, out, out2, n, i2, f))

    def run(self, L):
        arr = (L_BcOp() * len(self.ops))()
        p = lambda k: 0 if k is None else self.t[k].data_ptr()   # noqa: E731
        for j, (kind, flag, a, b, out, out2, n, i2, f) in enumerate(self.ops):
            arr[j].kind, arr[j].flag, arr[j].a, arr[j].b, arr[j].out, arr[j].out2 = kind, flag, p(a), p(b), p(out), p(out2)
            arr[j].n, arr[j].i2, arr[j].f = n, i2, f
        failed = C.c_int32(0)
        from data_free_quantization_amd import _lib
        rc = L.dfq_bc_chain(arr, len(self.ops), C.byref(failed), C.c_void_p(torch.cuda.current_stream().cuda_stream))
        _lib.check(rc, f"dfq_bc_chain (op {failed.value})")
        torch.cuda.synchronize()
        return {k: v.cpu().numpy().copy() for k, v in self.t.items()}


def L_BcOp():
    from data_free_quantization_amd import _lib
    return _lib.BcOp


def _same(a, b, skip=()):
    assert a.keys() == b.keys()
    for k in a:
        if not k.startswith(tuple(skip)):
            assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k


def _coop(walk_args, monkeypatch, grid=None):
    """The one-launch path (diagnostics library)."""
    from data_free_quantization_amd import _lib
    monkeypatch.setenv("DFQ_BC_CHAIN", "coop")
    if grid:
        monkeypatch.setenv("DFQ_BC_GRID", grid)
    r = Walk(*walk_args[0], **walk_args[1]).run(_lib.load_diag())
    monkeypatch.delenv("DFQ_BC_CHAIN")
    monkeypatch.delenv("DFQ_BC_GRID", raising=False)
    return r


@pytest.mark.parametrize("seed,kw", [(0, {}), (1, {"layers": 12}), (2, {"grouped": True, "layers": 9}),
                                     (3, {"width": (300, 1400), "layers": 5}), (4, {"width": (2, 6)}),
                                     (5, {"big_expect": True}), (6, {"alias": True})])
def test_cooperative_chain_equals_per_op_launches(seed, kw, monkeypatch):
    from data_free_quantization_amd import _lib
    ref = Walk(seed, **kw).run(_lib.load())
    got = _coop(((seed,), kw), monkeypatch)
    _same(ref, got)


@pytest.mark.parametrize("grid", ["1", "3", "17", "256"])
def test_cooperative_chain_grid_sizes(grid, monkeypatch):
    """Any grid gives the same bits: row / column owners move, orders do not."""
    from data_free_quantization_amd import _lib
    ref = Walk(11, layers=8).run(_lib.load())
    got = _coop(((11,), {"layers": 8}), monkeypatch, grid)
    _same(ref, got)


def test_cooperative_chain_repeats(monkeypatch):
    from data_free_quantization_amd import _lib
    ref = Walk(21, layers=10).run(_lib.load())
    for _ in range(5):
        _same(ref, _coop(((21,), {"layers": 10}), monkeypatch))


@pytest.mark.parametrize("seed", [31, 32])
def test_scratch_bias_vectors(seed, monkeypatch):
    """DFQ_BC_APPLY_VEC_SCRATCH: the one-launch path may leave the bias vectors
    unwritten (every reader recomputes them); everything else is bit-identical."""
    from data_free_quantization_amd import _lib
    ref = Walk(seed, layers=9, grouped=seed == 32, scratch=True).run(_lib.load())
    got = _coop(((seed,), {"layers": 9, "grouped": seed == 32, "scratch": True}), monkeypatch)
    _same(ref, got, skip=("vec",))
