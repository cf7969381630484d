"""dfq_bc_chain runs a layer's EXPECT+ -> APPLY (-> PROPAGATE) op group as ONE
launch (bc_layer_kernel: the expectation recomputed per block, the propagate
recomputing fl(E + expect) instead of reading the apply's bias_vec).  Checked
bit for bit against the same ops issued one dfq_bc_chain call each (one launch
per op), over dense / depthwise / Linear-like shapes, add branches (accumulated
expectations), broadcasts (i2 == 1, f == 1), with and without a propagate, at
1, 8 and 16 reference threads; and a group whose propagate writes a BN the
expectation reads is NOT fused (still bit-identical)."""
import ctypes as C

import numpy as np
import pytest
import torch

from data_free_quantization_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _chain(ops, per_op):
    L = _lib.load()
    rows = [(k, fl, a, b, o, o2, n, i2, f) for (k, fl, a, b, o, o2, n, i2, f) in ops]
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    groups = [[r] for r in rows] if per_op else [rows]
    for g in groups:
        arr = np.array(g, dtype=np.dtype([("kind", "<i4"), ("flag", "<i4"), ("a", "<u8"), ("b", "<u8"),
                                          ("out", "<u8"), ("out2", "<u8"), ("n", "<i8"), ("i2", "<i8"),
                                          ("f", "<i8")]))
        failed = C.c_int32(-1)
        _lib.check(L.dfq_bc_chain(arr.ctypes.data_as(C.POINTER(_lib.BcOp)), len(g), C.byref(failed), s),
                   "dfq_bc_chain")
    torch.cuda.synchronize()


def _case(seed, o, i2, f, nterms, F, threads, relu_mask, same_bn=False):
    g = torch.Generator(device="cpu").manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g).to(DEV)   # noqa: E731
    bn = [(r(f).abs() + 0.3, r(f)) for _ in range(nterms)]
    E = r(o * i2) * 0.01
    bias = r(o)
    slot = torch.empty(f, device=DEV)
    bcols = i2 if (i2 == f or f == 1) else f
    vec = torch.empty(o * bcols, device=DEV)
    fake_b = bn[0][1] if same_bn else r(F)
    ops = []
    for t in range(nterms):
        ops.append((_lib.DFQ_BC_OP_EXPECT, int(relu_mask[t]) | ((1 if t else 0) << 1), bn[t][0].data_ptr(),
                    bn[t][1].data_ptr(), slot.data_ptr(), 0, f, 0, 0))
    ops.append((_lib.DFQ_BC_OP_APPLY, _lib.DFQ_BC_APPLY_VEC_SCRATCH, E.data_ptr(), slot.data_ptr(), bias.data_ptr(),
                vec.data_ptr(), o, i2, f))
    if F:
        ops.append((_lib.DFQ_BC_OP_PROPAGATE, threads, vec.data_ptr(), 0, fake_b.data_ptr(), 0, o * bcols, 0, F))
    return ops, (bias, vec, slot, fake_b), [t for p in bn for t in p] + [E]


@pytest.mark.parametrize("threads", [1, 8, 16])
@pytest.mark.parametrize("o,i2,f,nterms,F", [
    (96, 16, 16, 1, 96),        # 1x1 conv, one BN, propagate into the next BN
    (144, 1, 144, 1, 144),      # depthwise: E [o, 1] broadcast over the expectation
    (1000, 1280, 1280, 1, 0),   # Linear at the end: no propagate
    (24, 144, 144, 2, 24),      # add branch: accumulated expectations
    (320, 960, 960, 3, 320),
    (64, 64, 1, 1, 64),         # one-channel expectation broadcast
    (512, 2048, 2048, 1, 2048), # ResNet-50's widest 1x1, F != o
])
def test_layer_group_equals_per_op_launches(o, i2, f, nterms, F, threads):
    res = []
    for per_op in (True, False):
        ops, outs, _ = _case(7 + o, o, i2, f, nterms, F, threads, [1, 0, 1][:nterms] + [1] * 8)
        _chain(ops, per_op)
        res.append([t.cpu() for t in outs])
    for a, b in zip(*res):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def test_propagate_into_an_expectation_bn_is_not_fused():
    res = []
    for per_op in (True, False):
        ops, outs, _ = _case(3, 64, 64, 64, 1, 64, 8, [1], same_bn=True)
        _chain(ops, per_op)
        res.append([t.cpu() for t in outs])
    for a, b in zip(*res):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
