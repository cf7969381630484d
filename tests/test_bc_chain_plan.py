"""dfq_bc_chain's phase planner (host code, CPU): where the cooperative launch
puts its grid barriers, which dependencies it forwards inside a phase, and
which chains it hands to the per-op launches.  Pointers are synthetic
(non-overlapping address ranges); no device call is made.  The GPU results of
the same rules are in test_gpu_bc_chain.py."""
import ctypes as C

import pytest

from data_free_quantization_amd import _lib

EXPECT, APPLY, PROPAGATE, COPY = 0, 1, 2, 3


class Mem:
    """A bump allocator of fake device addresses (float counts)."""

    def __init__(self):
        self.top = 1 << 32

    def __call__(self, n):
        a = self.top
        self.top += 4 * max(n, 1) + 256
        return a


def plan(ops, waves=512):
    try:
        L = _lib.load_diag()
    except OSError:
        pytest.skip("diagnostics library not built")
    arr = (_lib.BcOp * len(ops))()
    for j, (kind, flag, a, b, out, out2, n, i2, f) in enumerate(ops):
        arr[j].kind, arr[j].flag, arr[j].a, arr[j].b, arr[j].out, arr[j].out2 = kind, flag, a, b, out, out2
        arr[j].n, arr[j].i2, arr[j].f = n, i2, f
    nph = C.c_int32(0)
    per = (C.c_int32 * max(len(ops), 1))()
    rc = L.dfq_bc_chain_phases(arr, len(ops), waves, C.byref(nph), per)
    return rc, nph.value, list(per)[:len(ops)]


def layer_ops(m, bn_w, bn_b, E, bias, o, i, relu=1, acc_bn=None, nxt_fb=None):
    """One target layer of the walk: expect (+ an 'add' term), apply, propagate."""
    ex, vec = m(i), m(o * i)
    ops = [(EXPECT, relu, bn_w, bn_b, ex, 0, i, 0, 0)]
    if acc_bn is not None:
        ops.append((EXPECT, 1 | 2, acc_bn[0], acc_bn[1], ex, 0, i, 0, 0))
    ops.append((APPLY, 0, E, ex, bias, vec, o, i, i))
    if nxt_fb is not None:
        ops.append((PROPAGATE, 8, vec, 0, nxt_fb, 0, o * i, 0, o))
    return ops


def test_one_phase_per_layer_of_a_serial_walk():
    m = Mem()
    ch = [16, 32, 48, 24]
    fw = [m(c) for c in ch]
    fb = [m(c) for c in ch]
    ops = []
    for l in range(3):
        ops += layer_ops(m, fw[l], fb[l], m(ch[l + 1] * ch[l]), m(ch[l + 1]), ch[l + 1], ch[l], nxt_fb=fb[l + 1])
    rc, nph, per = plan(ops)
    assert rc == 0
    # each layer's expect reads the fake_bias the previous layer's propagate wrote
    assert nph == 3 and per == [0, 0, 0, 1, 1, 1, 2, 2, 2]


def test_add_branch_whose_second_bn_was_just_propagated_into():
    """The skip BN's term comes first, the fresh BN's second: the running sum's
    first term is moved into the new phase (a forced break) instead of falling
    back to per-op launches."""
    m = Mem()
    c = 32
    fw = [m(c) for _ in range(3)]
    fb = [m(c) for _ in range(3)]
    ops = layer_ops(m, fw[0], fb[0], m(c * c), m(c), c, c, nxt_fb=fb[1])
    ops += layer_ops(m, fw[2], fb[2], m(c * c), m(c), c, c, acc_bn=(fw[1], fb[1]))
    rc, nph, per = plan(ops)
    assert rc == 0
    assert nph == 2 and per == [0, 0, 0, 1, 1, 1]


def test_two_branches_of_one_bias_share_a_phase():
    m = Mem()
    o, i = 24, 40
    E, bias = m(o * i), m(o)
    ops = layer_ops(m, m(i), m(i), E, bias, o, i)
    exb, vecb = m(1), m(o * i)
    ops += [(EXPECT, 0, m(i), m(i), exb, 0, 1, 0, 0), (APPLY, 0, E, exb, bias, vecb, o, i, 1)]
    rc, nph, per = plan(ops)
    assert rc == 0 and nph == 1


def test_snapshot_copies_bracket_the_walk():
    m = Mem()
    o, i = 24, 40
    bias = m(o)
    snap0, snap1 = m(o), m(o)
    ops = [(COPY, 0, bias, 0, snap0, 0, o, 0, 0)]
    ops += layer_ops(m, m(i), m(i), m(o * i), bias, o, i)
    ops += [(COPY, 0, bias, 0, snap1, 0, o, 0, 0)]
    rc, nph, per = plan(ops)
    assert rc == 0
    # the apply writes what the first copy read; the last copy reads what the apply wrote
    assert per == [0, 0, 1, 2]


def test_chains_left_to_per_op_launches():
    m = Mem()
    i = 40
    fb = m(i)
    # an expectation written over its own input
    rc, _, _ = plan([(EXPECT, 1, m(i), fb, fb, 0, i, 0, 0)])
    assert rc == 1
    # an expectation larger than the LDS slots
    rc, _, _ = plan([(EXPECT, 1, m(9000), m(9000), m(9000), 0, 9000, 0, 0)])
    assert rc == 1
    # E written earlier in the chain (it is read without coherent loads)
    o = 8
    E = m(o * i)
    ops = [(COPY, 0, m(o * i), 0, E, 0, o * i, 0, 0)] + layer_ops(m, m(i), m(i), E, m(o), o, i)
    rc, _, _ = plan(ops)
    assert rc == 1


def test_empty_ops_are_skipped():
    m = Mem()
    ops = [(COPY, 0, m(1), 0, m(1), 0, 0, 0, 0)] + layer_ops(m, m(8), m(8), m(64), m(8), 8, 8)
    rc, nph, per = plan(ops)
    assert rc == 0 and per[0] == -1 and nph == 1
