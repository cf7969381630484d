"""HIP graph transforms (BN fold, CLE relation, absorption, BC helpers) vs the
reference's golden outputs.  Bit-exact except where the reference reduces in
an unspecified order (absorption GEMV, BC means): rtol 1e-5 / atol 1e-6."""
import numpy as np
import pytest
import torch
import torch.nn as nn
from collections import OrderedDict

from tests.helpers import transform_cases

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def test_bn_fold():
    from data_free_quantization_amd.utils.layer_transform import merge_batchnorm
    z, meta = transform_cases()
    for tag in ("bnfold_a", "bnfold_b"):
        w = z[f"{tag}_w"]
        conv = nn.Conv2d(w.shape[1], w.shape[0], w.shape[2], bias=True).to(DEV)
        bn = nn.BatchNorm2d(w.shape[0]).to(DEV)
        with torch.no_grad():
            conv.weight.copy_(T(w)); conv.bias.copy_(T(z[f"{tag}_b"]))
            bn.weight.copy_(T(z[f"{tag}_g"])); bn.bias.copy_(T(z[f"{tag}_beta"]))
            bn.running_mean.copy_(T(z[f"{tag}_m"])); bn.running_var.copy_(T(z[f"{tag}_v"]))
        graph = OrderedDict([("Data", "Data"), (1, conv), (2, bn)])
        bottoms = OrderedDict([("Data", None), (1, ["Data"]), (2, [1])])
        merge_batchnorm(None, graph, bottoms, (nn.Conv2d, nn.Linear))
        assert np.array_equal(conv.weight.detach().cpu().numpy(), z[f"{tag}_w_out"])
        assert np.array_equal(conv.bias.detach().cpu().numpy(), z[f"{tag}_b_out"])
        assert np.array_equal(bn.fake_weight.cpu().numpy(), z[f"{tag}_fw"])
        assert np.array_equal(bn.fake_bias.cpu().numpy(), z[f"{tag}_fb"])
        after = np.stack([t.detach().cpu().numpy() for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)])
        assert np.array_equal(after, z[f"{tag}_bn_after"])
        assert bn.eps == 0


@pytest.mark.parametrize("tag", ["cle_dense", "cle_pw_dw", "cle_dw_pw", "cle_signed", "cle_dead", "cle_linear",
                                 "cle_grouped2"])
def test_cle_relation(tag):
    from data_free_quantization_amd.Cross_layer_equal import _layer_equalization
    z, meta = transform_cases()
    w1, w2, b1 = T(z[f"{tag}_w1"]), T(z[f"{tag}_w2"]), T(z[f"{tag}_b1"])
    bnw, bnb = T(z[f"{tag}_bnw"]), T(z[f"{tag}_bnb"])
    W1, W2, B1, S = _layer_equalization(w1, w2, b1, bnw, bnb, s_min_max=[1e-8, 1e8], signed=meta[tag]["signed"])
    for got, key in ((W1, "w1_out"), (W2, "w2_out"), (B1, "b1_out"), (bnw, "bnw_out"), (bnb, "bnb_out"),
                     (S, "S")):
        assert np.array_equal(got.cpu().numpy(), z[f"{tag}_{key}"]), key


@pytest.mark.parametrize("tag", ["absorb_dense", "absorb_dw"])
def test_absorption(tag):
    from data_free_quantization_amd.bias_absorption import bias_absorption
    from data_free_quantization_amd.utils.relation import Relation
    z, meta = transform_cases()
    c1 = meta[tag]["c1"]
    w2 = z[f"{tag}_w2"]
    conv1 = nn.Conv2d(8, c1, 1, bias=True).to(DEV)
    groups = c1 // w2.shape[1]
    conv2 = nn.Conv2d(c1, w2.shape[0], 3, padding=1, groups=groups, bias=True).to(DEV)
    bn = nn.BatchNorm2d(c1).to(DEV)
    with torch.no_grad():
        conv1.bias.copy_(T(z[f"{tag}_b1"])); conv2.weight.copy_(T(w2)); conv2.bias.copy_(T(z[f"{tag}_b2"]))
    bn.register_buffer("fake_weight", T(z[f"{tag}_fw"]).clone())
    bn.register_buffer("fake_bias", T(z[f"{tag}_fb"]).clone())
    graph = OrderedDict([("Data", "Data"), (1, conv1), (2, bn), (3, nn.ReLU()), (4, conv2)])
    bottoms = OrderedDict([("Data", None), (1, ["Data"]), (2, [1]), (3, [2]), (4, [3])])
    bias_absorption(graph, [Relation(1, 4, 2)], bottoms, N=3)
    assert np.array_equal(conv1.bias.detach().cpu().numpy(), z[f"{tag}_b1_out"])
    assert np.array_equal(bn.fake_bias.cpu().numpy(), z[f"{tag}_fb_out"])
    np.testing.assert_allclose(conv2.bias.detach().cpu().numpy(), z[f"{tag}_b2_out"], rtol=1e-5, atol=1e-6)


def test_bias_correction_helpers():
    from data_free_quantization_amd import bias_correction as bc
    z, _ = transform_cases()
    w, b = T(z["bc_w"]), T(z["bc_b"])
    ex = bc._bc_expect(w, b, True)
    assert np.array_equal(ex.cpu().numpy(), z["bc_expect_relu"])
    ex2 = bc._bc_expect(w, b, True)
    bc._bc_expect(w.flip(0).contiguous(), b.flip(0).contiguous(), False, out=ex2)
    assert np.array_equal(ex2.cpu().numpy(), z["bc_expect_add"])
    layer = nn.Conv2d(64, 32, 1, bias=True).to(DEV)
    with torch.no_grad():
        layer.bias.copy_(T(z["bc_bias"]))
    E = T(z["bc_E"])
    vec = bc._apply_bias_correction_E(layer, E, 32, 64, "one", T(z["bc_expect_relu"]))
    assert np.array_equal(layer.bias.detach().cpu().numpy(), z["bc_bias_out"])
    assert np.array_equal(vec.cpu().numpy(), z["bc_vec"])
    fb = T(z["bc_fb"]).clone()
    from data_free_quantization_amd import _lib
    _lib.check(_lib.load().dfq_bc_propagate(_lib.ptr(vec), vec.numel(), _lib.ptr(fb), 32, 8, _lib.stream_of(fb)),
               "p")
    assert np.array_equal(fb.cpu().numpy(), z["bc_fb_out"])
    dw = nn.Conv2d(64, 64, 3, groups=64, bias=True).to(DEV)
    with torch.no_grad():
        dw.bias.zero_()
    bc._apply_bias_correction_E(dw, T(z["bc_Ed"]), 64, 1, "one", T(z["bc_expect_relu"]))
    assert np.array_equal(dw.bias.detach().cpu().numpy(), z["bc_dw_bias_out"])
    with pytest.raises(RuntimeError):   # 'cat' branch: the reference's torch.cat of 2-D with 1-D
        bc._apply_bias_correction_E(layer, E, 32, 64, "cat", T(z["bc_expect_relu"]))


def test_bc_chain_matches_single_ops():
    """dfq_bc_chain (the walk's ops in one call) == the same fixtures as the
    per-op entry points; a bad op is reported by index with nothing enqueued."""
    import ctypes as C
    from data_free_quantization_amd import _lib
    z, _ = transform_cases()
    L = _lib.load()
    w, b = T(z["bc_w"]), T(z["bc_b"])
    ex = torch.empty_like(b)
    bias = T(z["bc_bias"]).clone()
    E = T(z["bc_E"])
    vec = torch.empty(32 * 64, device=DEV)
    fb = T(z["bc_fb"]).clone()
    ops = (_lib.BcOp * 3)()
    ops[0].kind, ops[0].flag, ops[0].a, ops[0].b, ops[0].out, ops[0].n = (
        _lib.DFQ_BC_OP_EXPECT, 1, w.data_ptr(), b.data_ptr(), ex.data_ptr(), b.numel())
    ops[1].kind, ops[1].a, ops[1].b, ops[1].out, ops[1].out2, ops[1].n, ops[1].i2, ops[1].f = (
        _lib.DFQ_BC_OP_APPLY, E.data_ptr(), ex.data_ptr(), bias.data_ptr(), vec.data_ptr(), 32, 64, ex.numel())
    ops[2].kind, ops[2].flag, ops[2].a, ops[2].out, ops[2].n, ops[2].f = (
        _lib.DFQ_BC_OP_PROPAGATE, 8, vec.data_ptr(), fb.data_ptr(), vec.numel(), 32)
    failed = C.c_int32(0)
    _lib.check(L.dfq_bc_chain(ops, 3, C.byref(failed), _lib.stream_of(fb)), "dfq_bc_chain")
    assert failed.value == -1
    assert np.array_equal(ex.cpu().numpy(), z["bc_expect_relu"])
    assert np.array_equal(bias.cpu().numpy(), z["bc_bias_out"])
    assert np.array_equal(vec.cpu().numpy(), z["bc_vec"])
    assert np.array_equal(fb.cpu().numpy(), z["bc_fb_out"])
    before = fb.clone()
    ops[0].out = fb.data_ptr()          # would overwrite fb if anything ran
    ops[2].f = 30                       # 2048 % 30 != 0: .view(-1, F) fails
    assert L.dfq_bc_chain(ops, 3, C.byref(failed), _lib.stream_of(fb)) == _lib.DFQ_ERR_SHAPE
    assert failed.value == 2
    torch.cuda.synchronize()
    assert torch.equal(fb, before)


def test_bc_reference_named_helpers():
    """_compute_final_bias_correction + _apply_bias_correction (bias_correction.py:61-106)
    called by their reference names: same fixtures as the fused path."""
    from data_free_quantization_amd import bias_correction as bc
    z, _ = transform_cases()
    T = lambda a: torch.from_numpy(a).to(DEV)
    layer = nn.Conv2d(64, 32, 1, bias=True).to(DEV)
    with torch.no_grad():
        layer.bias.copy_(T(z["bc_bias"]))
    bv = bc._compute_final_bias_correction(T(z["bc_E"]), ("one", T(z["bc_expect_relu"])))
    assert np.array_equal(bv.cpu().numpy().ravel(), z["bc_vec"])
    bc._apply_bias_correction(layer, bv)
    assert np.array_equal(layer.bias.detach().cpu().numpy(), z["bc_bias_out"])
    dw = nn.Conv2d(64, 64, 3, groups=64, bias=True).to(DEV)
    with torch.no_grad():
        dw.bias.zero_()
    bc._apply_bias_correction(dw, bc._compute_final_bias_correction(T(z["bc_Ed"]), ("one", T(z["bc_expect_relu"]))))
    assert np.array_equal(dw.bias.detach().cpu().numpy(), z["bc_dw_bias_out"])
    with pytest.raises(RuntimeError):   # torch.cat of a 2-D eps with a 1-D expectation
        bc._compute_final_bias_correction(T(z["bc_E"]), ("cat", T(z["bc_expect_relu"])))
    with pytest.raises(ValueError):     # fewer elements than the bias
        bc._apply_bias_correction(layer, torch.zeros(8, device=DEV))


def test_clip_weight():
    from data_free_quantization_amd.clip_weight import clip_weight
    conv = nn.Conv2d(16, 32, 3).to(DEV)
    with torch.no_grad():
        conv.weight.normal_(0, 20)
    ref = conv.weight.detach().clamp(-15, 15)
    clip_weight({1: conv}, [-15, 15], [nn.Conv2d, nn.Linear])
    assert torch.equal(conv.weight.detach(), ref)


_FUZZ_SEEDS = [int(v) for v in __import__("os").environ.get("DFQ_FUZZ_SEEDS", "1,2,3,4").split(",")]


@pytest.mark.parametrize("seed", _FUZZ_SEEDS)
def test_cle_relation_and_bn_fold_fuzz(seed):
    """Random relations (dense, depthwise pairs, grouped W2, Linear W2, signed, dead
    channels, huge/tiny ranges hitting the s clamps) and random BN folds: the HIP
    kernels bit-exact with the oracle (pinned to the reference by the golden cases)."""
    from oracle import oracle as O
    from data_free_quantization_amd.Cross_layer_equal import _layer_equalization
    from data_free_quantization_amd.utils.layer_transform import merge_batchnorm
    rng = np.random.default_rng(seed)
    for _ in range(12):
        c1 = int(rng.choice([1, 3, 16, 96, 160, 257]))
        kind = rng.choice(["dense", "dw", "grouped", "linear"])
        k1 = int(rng.choice([1, 3]))
        w1 = (rng.standard_normal((c1, int(rng.integers(1, 40)), k1, k1)) *
              rng.choice([1e-4, 0.1, 3.0])).astype(np.float32)
        if kind == "dw":
            w2 = rng.standard_normal((c1, 1, 3, 3)).astype(np.float32)
        elif kind == "grouped":
            g = 1 if c1 % 2 else 2
            w2 = rng.standard_normal((4 * g, c1 // g, 3, 3)).astype(np.float32)
        elif kind == "linear":
            w2 = rng.standard_normal((int(rng.integers(1, 50)), c1)).astype(np.float32)
        else:
            w2 = rng.standard_normal((int(rng.integers(1, 70)), c1, 1, 1)).astype(np.float32)
        if rng.random() < 0.3:
            w1[int(rng.integers(0, c1))] = 0.0   # dead channel: s -> 1e8
        b1 = rng.standard_normal(c1).astype(np.float32)
        bnw = rng.uniform(0.5, 1.5, c1).astype(np.float32)
        bnb = rng.normal(0, 0.5, c1).astype(np.float32)
        signed = bool(rng.random() < 0.3)
        ref = O.cle_relation(w1, w2, b1, bnw, bnb, signed=signed)
        tw1, tw2, tb1, tbw, tbb = T(w1), T(w2), T(b1), T(bnw), T(bnb)
        W1, W2, B1, S = _layer_equalization(tw1, tw2, tb1, tbw, tbb, s_min_max=[1e-8, 1e8], signed=signed)
        for got, want, name in ((W1, ref[0], "w1"), (W2, ref[1], "w2"), (B1, ref[2], "b1"), (tbw, ref[3], "bnw"),
                                (tbb, ref[4], "bnb"), (S, ref[5], "S")):
            assert np.array_equal(got.cpu().numpy(), want), (name, kind, c1, w2.shape, signed)
    for _ in range(6):
        o, i, k = int(rng.integers(1, 300)), int(rng.integers(1, 64)), int(rng.choice([1, 3, 5]))
        w = rng.standard_normal((o, i, k, k)).astype(np.float32)
        b = rng.standard_normal(o).astype(np.float32)
        g, beta = rng.uniform(-1.5, 1.5, o).astype(np.float32), rng.normal(0, 1, o).astype(np.float32)
        m, v = rng.normal(0, 0.3, o).astype(np.float32), rng.uniform(1e-3, 3, o).astype(np.float32)
        eps = float(rng.choice([1e-5, 1e-3, 0.0]))
        ref = O.bn_fold(w, b, g, beta, m, v, eps)
        conv = nn.Conv2d(i, o, k, bias=True).to(DEV)
        bn = nn.BatchNorm2d(o, eps=eps).to(DEV)
        with torch.no_grad():
            conv.weight.copy_(T(w)); conv.bias.copy_(T(b))
            bn.weight.copy_(T(g)); bn.bias.copy_(T(beta)); bn.running_mean.copy_(T(m)); bn.running_var.copy_(T(v))
        graph = OrderedDict([("Data", "Data"), (1, conv), (2, bn)])
        bottoms = OrderedDict([("Data", None), (1, ["Data"]), (2, [1])])
        merge_batchnorm(None, graph, bottoms, (nn.Conv2d, nn.Linear))
        assert np.array_equal(conv.weight.detach().cpu().numpy(), ref[0])
        assert np.array_equal(conv.bias.detach().cpu().numpy(), ref[1])
        assert np.array_equal(bn.fake_weight.cpu().numpy(), ref[6]) and np.array_equal(bn.fake_bias.cpu().numpy(),
                                                                                       ref[7])


@pytest.mark.parametrize("big", [False, True])
def test_bn_fold_batch_shapes_ranges_and_identity_rows(big):
    """dfq_bn_fold_batch over many folds in one call: row lengths 1 .. 123,000 (rows
    straddling chunks), weights at unaligned offsets, identity BN rows (factor
    exactly 1: read, not rewritten), bias-less layers (DFQ_BN_FOLD_ZERO_BIAS), and
    the per-weight (min, max) by-product -- bit-exact with the oracle fold.
    ``big``: a batch past 2^27 elements (chunks wider than 8192)."""
    from oracle import oracle as O
    from data_free_quantization_amd.utils.layer_transform import _fold_batch
    rng = np.random.default_rng(7 if big else 5)
    shapes = [(1100, 123000)] if big else [(5, 1), (7, 3), (33, 9), (64, 25), (3, 4097), (2, 20000), (300, 147),
                                           (17, 2), (1, 1)]
    pairs, refs, wants = [], [], []
    for si, (o, rl) in enumerate(shapes):
        w = (rng.standard_normal((o, rl)) * 0.2).astype(np.float32)
        g = rng.uniform(-1.5, 1.5, o).astype(np.float32)
        beta = rng.normal(0, 1, o).astype(np.float32)
        m = rng.normal(0, 0.3, o).astype(np.float32)
        v = rng.uniform(1e-3, 3, o).astype(np.float32)
        ident = rng.random(o) < 0.4
        g[ident], v[ident], m[ident], beta[ident] = 1.0, 1.0, 0.0, 0.0
        eps = 0.0
        has_bias = si % 3 != 0
        b = rng.standard_normal(o).astype(np.float32) if has_bias else np.zeros(o, np.float32)
        ref = O.bn_fold(w.reshape(o, rl, 1, 1), b, g, beta, m, v, eps)
        shift = si % 4                                     # unaligned weight start
        buf = torch.zeros(o * rl + shift, device=DEV)
        wt = buf[shift:].view(o, rl, 1, 1)
        wt.copy_(T(w.reshape(o, rl, 1, 1)))
        conv = nn.Conv2d(rl, o, 1, bias=has_bias).to(DEV)
        conv.weight = nn.Parameter(wt, requires_grad=False)
        if has_bias:
            with torch.no_grad():
                conv.bias.copy_(T(b))
        bn = nn.BatchNorm2d(o, eps=eps).to(DEV)
        with torch.no_grad():
            bn.weight.copy_(T(g)); bn.bias.copy_(T(beta)); bn.running_mean.copy_(T(m)); bn.running_var.copy_(T(v))
        pairs.append((bn, conv))
        refs.append(ref)
    ranges = {}
    _fold_batch(pairs, ranges)
    torch.cuda.synchronize()
    for (bn, conv), ref in zip(pairs, refs):
        got = conv.weight.detach().cpu().numpy()
        assert np.array_equal(got, ref[0]), conv.weight.shape
        assert np.array_equal(conv.bias.detach().cpu().numpy(), ref[1])
        assert np.array_equal(bn.fake_weight.cpu().numpy(), ref[6])
        enc = ranges[conv].cpu().numpy().view(np.uint32)
        dec = lambda e: np.array([e ^ 0x80000000 if e & 0x80000000 else ~e & 0xFFFFFFFF],   # noqa: E731
                                 dtype=np.uint32).view(np.float32)[0]
        assert dec(~enc[0] & 0xFFFFFFFF) == ref[0].min() and dec(enc[1]) == ref[0].max()


def test_bias_correction_returns_before_and_after_biases():
    """bias_correction's return values (bias_correction.py:180-258): every target
    layer's bias at entry and at exit, keyed "layer_<idx>", as read-only mappings
    of views (the snapshots are COPY ops of the chain)."""
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.bias_correction import bias_correction
    from data_free_quantization_amd.utils.layer_transform import merge_batchnorm
    from data_free_quantization_amd.utils.tracer import build_graph
    m = zoo.build("mobilenetv2", seed=3, relu=True).to(DEV)
    g = build_graph(m, "positional")
    G, B = g.getGraph(), g.getBottoms()
    targ = (nn.Conv2d, nn.Linear)
    merge_batchnorm(m, G, B, targ)
    entry = {f"layer_{i}": l.bias.detach().clone() for i, l in enumerate(G.values())
             if i in B and isinstance(l, targ) and l.bias is not None}
    before, after = bias_correction(G, B, targ, bits_weight=8, signed=True)
    torch.cuda.synchronize()
    assert set(before) == set(entry) and len(after) > 0
    for k, v in entry.items():
        assert torch.equal(before[k], v)
    layers = list(G.values())
    changed = 0
    for k, v in after.items():
        b = layers[int(k.split("_")[1])].bias.detach()
        assert torch.equal(v, b)
        changed += int(not torch.equal(v, entry[k]))
    assert changed > 0
