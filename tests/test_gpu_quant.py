"""HIP quantize path vs the reference's golden vectors and the pinned oracle.

Bit-exact everywhere: dequantized fp32 values (signed zeros folded), integer
codes, scales, and the BC error sums E (summed over KH*KW in ATen's order).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import case_flags, h, quant_cases

pytestmark = pytest.mark.gpu
CASES = quant_cases()
DEV = "cuda:0"


def _run_hip(case):
    from data_free_quantization_amd.utils.quantize import fake_quant
    mode, rows, flags, given = case_flags(case)
    x = torch.from_numpy(case["x"]).to(DEV)
    kw = dict(per_channel=mode >= 2, symmetric=mode in (1, 3), khw=case["khw"], want_esum=case["esum"])
    if case["given"] is not None:
        kw.update(min_value=given[0], max_value=given[1])
    if case["default_range"]:
        kw.update(scale_f32=True)
    if case["clip"] is not None:
        kw.update(clip=tuple(case["clip"]))
    return fake_quant(x, case["bits"], **kw)


@pytest.mark.parametrize("case", CASES, ids=[f"{c['idx']}-{c['name']}-{c['mode']}-b{c['bits']}" for c in CASES])
def test_hip_quantize_matches_reference(case):
    r = _run_hip(case)
    torch.cuda.synchronize()
    dq = r.dq.cpu().numpy()
    assert h(dq) == case["dqh"], "dequantized values differ from the reference"
    if case["dq"] is not None:
        assert np.array_equal(dq, case["dq"])
    if case["esum"]:
        assert np.array_equal(r.esum.cpu().numpy(), case["esum_ref"])   # ATen's KH*KW sum order
    mode, rows, flags, given = case_flags(case)
    o = O.quantize(case["x"], case["bits"], mode, rows=rows, khw=case["khw"], flags=flags,
                   clip=tuple(case["clip"]) if case["clip"] else (0.0, 0.0), given=given)
    codes = r.codes.cpu().numpy().view(o["codes"].dtype)   # 16-bit asym: uint16 bits in an int16 tensor
    assert np.array_equal(codes, o["codes"]), "codes differ from the oracle"
    assert np.array_equal(r.scale.cpu().numpy(), o["scale"])
    assert np.array_equal(r.zero.cpu().numpy() + np.float32(0), o["zero"] + np.float32(0))


def test_grouped_sweep_matches_single_calls():
    """All golden cases in ONE grouped plan (mixed modes, bits, rows, khw)."""
    from data_free_quantization_amd.sweep import SweepItem, SweepPlan
    items, cases = [], []
    for c in CASES:
        if c["given"] is not None or c["default_range"]:
            continue
        mode, rows, flags, _ = case_flags(c)
        x = torch.from_numpy(c["x"]).to(DEV).contiguous()
        sym = mode in (1, 3)
        npar = rows if mode >= 2 else 1
        cdt = (torch.int8 if sym else torch.uint8) if c["bits"] <= 8 else torch.int16
        it = SweepItem(src=x, bits=c["bits"], per_channel=mode >= 2, symmetric=sym, dst=torch.empty_like(x),
                       codes=torch.empty(x.shape, dtype=cdt, device=DEV),
                       scale=torch.empty(npar, device=DEV), zero=torch.empty(npar, device=DEV),
                       esum=torch.empty(x.numel() // c["khw"], device=DEV) if c["esum"] else None,
                       khw=c["khw"], clip=tuple(c["clip"]) if c["clip"] else None, rows=rows)
        items.append(it)
        cases.append(c)
    plan = SweepPlan(items)
    for _ in range(2):   # replay: identical results
        plan.execute()
        torch.cuda.synchronize()
        for it, c in zip(items, cases):
            assert h(it.dst.cpu().numpy()) == c["dqh"], c["name"]
            if c["esum"]:
                assert np.array_equal(it.esum.cpu().numpy(), c["esum_ref"])
    plan.destroy()


@pytest.mark.parametrize("model", ["mobilenetv2", "resnet50", "deeplab"])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_full_model_sweep_vs_oracle(model, mode):
    """Every target weight of the model in one plan, vs the oracle layer by layer."""
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.sweep import allocate, SweepPlan, khw_of
    m = zoo.build(model, seed=3)
    layers = [l.weight.detach() for l in zoo.target_layers(m)]
    bits = 8 if mode != 1 else 4
    items = []
    for w in layers:
        wd = w.to(DEV).contiguous()
        items.append(allocate(wd, bits=bits, per_channel=mode >= 2, symmetric=mode in (1, 3), khw=khw_of(wd),
                              want_esum=True, clip=(-0.5, 0.5) if mode == 3 else None))
    plan = SweepPlan(items)
    plan.execute()
    torch.cuda.synchronize()
    for w, it in zip(layers, items):
        x = w.numpy()
        rows = x.shape[0] if mode >= 2 else 1
        o = O.quantize(x, bits, mode, rows=rows, khw=it.khw, flags=1 if mode == 3 else 0, clip=(-0.5, 0.5),
                       want_esum=True)
        assert np.array_equal(it.dst.cpu().numpy(), o["dq"])
        assert np.array_equal(it.codes.cpu().numpy().view(o["codes"].dtype), o["codes"])
        assert np.array_equal(it.scale.cpu().numpy(), o["scale"])
        assert np.array_equal(it.esum.cpu().numpy(), o["esum"])
    plan.destroy()


def _filler(items):
    """A 32 MiB per-tensor item appended to a small list: past one round of
    resident blocks, so the plan takes the 2,048-element tasks (variant 6)
    instead of the small-list 1,536 (variant 10)."""
    from data_free_quantization_amd.sweep import allocate
    items.append(allocate(torch.randn(2048, 4096, device=DEV), bits=8, per_channel=False, symmetric=False))


@pytest.mark.parametrize("small", [True, False], ids=["small_list", "large_list"])
def test_long_rows_and_odd_sizes_vs_oracle(small):
    """rows longer than one wave task (two-launch path), odd row lengths
    (scalar path), empty tensors, a single element -- as a small list (1,536-element
    tasks) and with a 2M-element tensor and a filler that make the list large (2,048)."""
    from data_free_quantization_amd.sweep import allocate, SweepPlan
    rng = np.random.default_rng(7)
    shapes = [(3, 4608), (2, 20000), (7, 27), (5, 9), (1, 1), (33, 13), (0, 9)] + ([] if small else [(513, 4100)])
    filler = not small
    items, xs = [], []
    for shp in shapes:
        x = rng.normal(0, 1, shp).astype(np.float32)
        xs.append(x)
        for mode in range(4):
            items.append(allocate(torch.from_numpy(x).to(DEV), bits=8, per_channel=mode >= 2,
                                  symmetric=mode in (1, 3), want_esum=True))
    if filler:
        _filler(items)
    plan = SweepPlan(items)
    assert plan.stats["variant"] == (6 if filler else 10), plan.stats
    plan.execute()
    torch.cuda.synchronize()
    k = 0
    for x in xs:
        for mode in range(4):
            it = items[k]
            k += 1
            if x.size == 0:
                continue
            o = O.quantize(x, 8, mode, rows=x.shape[0] if mode >= 2 else 1, want_esum=True)
            assert np.array_equal(it.dst.cpu().numpy(), o["dq"]), (x.shape, mode)
            assert np.array_equal(it.codes.cpu().numpy(), o["codes"]), (x.shape, mode)
            assert np.array_equal(it.esum.cpu().numpy(), o["esum"])
    plan.destroy()


@pytest.mark.parametrize("filler", [False, True], ids=["small_list", "with_filler"])
def test_block_row_pieces_vs_oracle(filler):
    """Rows of 2049..4 pieces (one workgroup, single HBM pass) and just past it
    (slot path), with KH*KW error sums; small per-tensor ranges (block path) next
    to large ones (reduce launch); odd lengths (scalar loads).  Small list and
    behind a filler (both task sizes, _filler)."""
    from data_free_quantization_amd.sweep import allocate, SweepPlan, khw_of
    rng = np.random.default_rng(11)
    shapes = [(4, 320, 3, 3), (2, 160, 7, 7), (2, 161, 7, 7), (3, 512, 3, 3), (3, 2051), (2, 8192), (2, 8193),
              (5, 1025, 1, 1), (1, 3, 3, 3), (64, 32, 3, 3)]
    items, xs = [], []
    for shp in shapes:
        x = rng.normal(0, 1, shp).astype(np.float32)
        xs.append(x)
        for mode in range(4):
            t = torch.from_numpy(x).to(DEV)
            items.append(allocate(t, bits=8 if mode != 1 else 5, per_channel=mode >= 2, symmetric=mode in (1, 3),
                                  khw=khw_of(t), want_esum=True, clip=(-1.0, 1.0) if mode == 3 else None))
    if filler:
        _filler(items)
    plan = SweepPlan(items)
    assert plan.stats["variant"] == (6 if filler else 10), plan.stats
    for _ in range(2):
        plan.execute()
        torch.cuda.synchronize()
        k = 0
        for x in xs:
            for mode in range(4):
                it = items[k]
                k += 1
                o = O.quantize(x, 8 if mode != 1 else 5, mode, rows=x.shape[0] if mode >= 2 else 1, khw=it.khw,
                               flags=1 if mode == 3 else 0, clip=(-1.0, 1.0), want_esum=True)
                assert np.array_equal(it.dst.cpu().numpy(), o["dq"]), (x.shape, mode)
                assert np.array_equal(it.codes.cpu().numpy().view(o["codes"].dtype), o["codes"]), (x.shape, mode)
                assert np.array_equal(it.scale.cpu().numpy(), o["scale"]), (x.shape, mode)
                assert np.array_equal(it.zero.cpu().numpy() + np.float32(0), o["zero"] + np.float32(0))
                assert np.array_equal(it.esum.cpu().numpy(), o["esum"]), (x.shape, mode)
    plan.destroy()


def test_large_sweep_properties():
    """Full-size (1 GiB) sweep: properties that need no oracle -- codes in range,
    the dequant identity dq == code*s + zero (bit-exact), the rounding bound
    |dq - x| <= s/2, and E == dq - x for 1x1 layers."""
    from data_free_quantization_amd.sweep import allocate, SweepPlan
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(65536, 4096, device=DEV, generator=g)
    it = allocate(x, bits=8, per_channel=True, symmetric=True, want_esum=True)
    plan = SweepPlan([it])
    plan.execute()
    torch.cuda.synchronize()
    assert int(it.codes.min()) >= -128 and int(it.codes.max()) <= 127
    regen = it.codes.float() * it.scale.view(-1, 1) + it.zero.view(-1, 1)
    assert torch.equal(regen, it.dst)
    # |x/s - q| <= 1/2 exactly; fl(x/s) and fl(q*s) add <= 127 * 2^-24 s each
    err = (it.dst - x).abs()
    assert bool((err <= it.scale.view(-1, 1) * 0.50002).all())
    assert torch.equal(it.esum.view_as(x), it.dst - x)
    plan.destroy()


def test_reference_quantize_api_on_gpu():
    from data_free_quantization_amd.utils.quantize import quantize
    for c in CASES:
        if c["mode"].startswith("channel") or c["clip"] is not None:
            continue
        x = torch.from_numpy(c["x"]).to(DEV)
        sym = c["mode"] == "tensor_sym"
        if c["given"] is not None:
            y = quantize(x, c["bits"], c["given"][0], c["given"][1], symmetric=sym)
        elif c["default_range"]:
            y = quantize(x, c["bits"], symmetric=sym)
        else:
            y = quantize(x, c["bits"], float(x.min()), float(x.max()), symmetric=sym)
        assert h(y.cpu().numpy()) == c["dqh"]
    # in-place + STE backward
    x = torch.randn(64, 32, device=DEV, requires_grad=True)
    y = quantize(x, 8, float(x.min()), float(x.max()))
    y.sum().backward()
    assert torch.equal(x.grad, torch.ones_like(x))


def test_large_ranges_vs_oracle(monkeypatch):
    """Per-tensor ranges from one workgroup (8192) up to 4M elements and just past,
    long per-channel rows, KH*KW sums, a single outlier setting a whole tensor's
    range: bit-exact with the oracle, and identical with block-row pieces off
    (DFQ_SWEEP_BLOCKROW=0: every range > one wave task through the reduce launch)."""
    from data_free_quantization_amd.sweep import allocate, SweepPlan, khw_of
    rng = np.random.default_rng(23)
    big = 512 * 4 * 2048
    shapes = [(8193,), (3, 4097, 3, 3), (1000, 1000), (big,), (big + 4,), (4, 20000), (2, 70001),
              (96, 144, 1, 1), (320, 1280)]
    xs = [rng.normal(0, 1, s).astype(np.float32) for s in shapes]
    xs[2][17, 3] = 40.0
    modes = [0, 1, 2, 3]

    def run():
        items = []
        for x in xs:
            for mode in modes:
                t = torch.from_numpy(x).to(DEV)
                items.append(allocate(t, bits=8 if mode != 1 else 4, per_channel=mode >= 2 and x.ndim > 1,
                                      symmetric=mode in (1, 3), khw=khw_of(t) if x.ndim > 2 else 1, want_esum=True,
                                      clip=(-2.0, 2.0) if mode == 3 else None))
        plan = SweepPlan(items)
        for _ in range(2):   # replay re-initialises the range slots
            plan.execute()
        torch.cuda.synchronize()
        return plan, items

    plan, items = run()
    k = 0
    for x in xs:
        for mode in modes:
            it = items[k]
            k += 1
            ch = mode >= 2 and x.ndim > 1
            m = mode if (ch or mode < 2) else mode - 2
            o = O.quantize(x, 8 if mode != 1 else 4, m, rows=x.shape[0] if ch else 1, khw=it.khw,
                           flags=1 if mode == 3 else 0, clip=(-2.0, 2.0), want_esum=True)
            assert np.array_equal(it.dst.cpu().numpy(), o["dq"]), (x.shape, mode)
            assert np.array_equal(it.codes.cpu().numpy().view(o["codes"].dtype), o["codes"]), (x.shape, mode)
            assert np.array_equal(it.scale.cpu().numpy(), o["scale"]), (x.shape, mode)
            assert np.array_equal(it.esum.cpu().numpy(), o["esum"]), (x.shape, mode)
    from data_free_quantization_amd import _lib
    monkeypatch.setattr(_lib, "_LIB", _lib.load_diag())   # the switch is a diagnostics-library A/B
    monkeypatch.setenv("DFQ_SWEEP_BLOCKROW", "0")
    plan2, items2 = run()
    for a, b in zip(items, items2):
        assert torch.equal(a.dst, b.dst) and torch.equal(a.codes, b.codes) and torch.equal(a.esum, b.esum)
    plan.destroy()
    plan2.destroy()


def test_many_models_per_tensor():
    """quantize_targ_layer's mode over 24 MobileNetV2 weight sets in one plan
    (reduce launch + quantize launch); every layer bit-exact with the oracle.  The
    two-stream slab pipeline (diagnostics A/B) is covered below."""
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.sweep import allocate, SweepPlan, khw_of
    m = zoo.build("mobilenetv2", seed=9)
    layers = [l.weight.detach() for l in zoo.target_layers(m)]
    ref = [O.quantize(w.numpy(), 8, O.TENSOR_ASYM, rows=1, khw=khw_of(w), flags=1, clip=(-0.3, 0.3),
                      want_esum=True) for w in layers]
    items = []
    for c in range(24):
        for w in layers:
            wd = (w.to(DEV) if c == 0 else w.to(DEV).clone()).contiguous()
            items.append(allocate(wd, bits=8, per_channel=False, symmetric=False, khw=khw_of(wd), want_esum=True,
                                  clip=(-0.3, 0.3)))
    plan = SweepPlan(items)
    for _ in range(2):   # replay: the range slots are re-armed
        plan.execute()
    torch.cuda.synchronize()
    assert plan.stats["launches"] == 2   # one reduce launch, one quantize launch
    for i, it in enumerate(items):
        o = ref[i % len(layers)]
        assert np.array_equal(it.dst.cpu().numpy(), o["dq"])
        assert np.array_equal(it.codes.cpu().numpy(), o["codes"])
        assert np.array_equal(it.esum.cpu().numpy(), o["esum"])
    plan.destroy()


@pytest.mark.parametrize("source", ["dfq_range", "bn_fold"])
def test_device_range_single_pass(source):
    """DFQ_DEVICE_RANGE: per-tensor sweeps taking their (min, max) from device words
    -- written by dfq_range, or by the second BN fold (identity BN, factor exactly
    1: weights read, not rewritten) -- are ONE launch and bit-exact with the
    oracle's two-pass result (MobileNetV2 ×4, asym and sym, clip + E)."""
    import ctypes as C
    import torch.nn as nn
    from data_free_quantization_amd import _lib, zoo
    from data_free_quantization_amd.sweep import allocate, SweepPlan, khw_of
    from data_free_quantization_amd.utils.layer_transform import _fold_batch
    m = zoo.build("mobilenetv2", seed=11)
    layers = [l.weight.detach() for l in zoo.target_layers(m)]
    L = _lib.load()
    for sym in (False, True):
        mode = O.TENSOR_SYM if sym else O.TENSOR_ASYM
        ref = [O.quantize(w.numpy(), 8, mode, rows=1, khw=khw_of(w), flags=1, clip=(-0.3, 0.3), want_esum=True)
               for w in layers]
        items, keep = [], []
        for c in range(4):
            ws = [w.to(DEV).clone().contiguous() for w in layers]
            if source == "dfq_range":
                rng = []
                for w in ws:
                    r = torch.empty(2, dtype=torch.int32, device=DEV)
                    _lib.check(L.dfq_range(w.data_ptr(), w.numel(), r.data_ptr(), _lib.stream_of(w)), "dfq_range")
                    rng.append(r)
            else:   # merge_batchnorm #2: identity BatchNorms after the first fold
                pairs = []
                for w in ws:
                    conv = nn.Conv2d(1, w.shape[0], 1).to(DEV)
                    conv.weight = nn.Parameter(w, requires_grad=False)
                    bn = nn.BatchNorm2d(w.shape[0]).to(DEV)   # weight 1, bias 0, mean 0, var 1
                    bn.eps = 0
                    pairs.append((bn, conv))
                    keep.append((bn, conv))
                before = [w.clone() for w in ws]
                ranges = {}
                _fold_batch(pairs, ranges)
                torch.cuda.synchronize()
                assert all(torch.equal(a, b) for a, b in zip(before, ws))   # factor 1: weights untouched
                rng = [ranges[conv] for _, conv in pairs]
            for w, r in zip(ws, rng):
                it = allocate(w, bits=8, per_channel=False, symmetric=sym, khw=khw_of(w), want_esum=True,
                              clip=(-0.3, 0.3))
                it.range_enc = r
                items.append(it)
        plan = SweepPlan(items)
        assert plan.stats["launches"] == 1 and plan.stats["n_tasks_reduce"] == 0
        plan.execute()
        torch.cuda.synchronize()
        for i, it in enumerate(items):
            o = ref[i % len(layers)]
            assert np.array_equal(it.dst.cpu().numpy(), o["dq"])
            assert np.array_equal(it.codes.cpu().numpy(), o["codes"])
            assert np.array_equal(it.esum.cpu().numpy(), o["esum"])
            assert np.array_equal(it.scale.cpu().numpy(), o["scale"])
        plan.destroy()


def _chunk_cases():
    from tests.helpers import chunk_cases
    return chunk_cases()


@pytest.mark.parametrize("case", _chunk_cases(), ids=lambda c: f"chunk{c['idx']}")
def test_quantize_num_chunks_matches_reference(case):
    """quantize() with num_chunks / one None bound on the GPU (dfq_chunk_range +
    the sweep): bit-exact with the reference's output; the chunk range itself equals
    the reference's y.min(-1)[0].mean(-1) / y.max(-1)[0].mean(-1); shapes the
    reference rejects raise RuntimeError."""
    from data_free_quantization_amd.utils.quantize import _chunk_range, quantize
    from tests.helpers import chunk_kwargs
    x = torch.from_numpy(case["x"]).to(DEV)
    if case["error"] is not None:
        with pytest.raises(RuntimeError):
            quantize(x, case["bits"], **chunk_kwargs(case))
        return
    rows = case["x"].shape[0] // case["num_chunks"]
    assert np.array_equal(np.array(_chunk_range(x, rows), np.float32), case["range"])
    y = quantize(x, case["bits"], **chunk_kwargs(case))
    torch.cuda.synchronize()
    assert h(y.cpu().numpy()) == case["dqh"]
    assert np.array_equal(y.cpu().numpy(), case["dq"])


def _pack_nibbles(codes):
    c = codes.reshape(-1).astype(np.uint8) & 0xF
    if c.size % 2:
        c = np.append(c, np.uint8(0))   # odd count: the last byte's high nibble is 0
    return (c[0::2] | (c[1::2] << 4)).astype(np.uint8)


def test_packed_int4_codes_vs_oracle():
    """DFQ_PACK_INT4: two codes per byte (element 2k low nibble), every mode and
    2-4 bits, on ResNet-50 layer shapes plus block-row and long-row cases; dq,
    scale and E unchanged; a layout without 16-B vectors is rejected."""
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.sweep import allocate, SweepPlan, khw_of
    m = zoo.build("resnet50", seed=4)
    ws = [l.weight.detach() for l in zoo.target_layers(m)][::6] + \
        [torch.randn(3, 4608) * 0.1, torch.randn(2, 20000) * 0.1, torch.randn(5, 4100) * 0.1,
         torch.randn(7, 5) * 0.1, torch.randn(33, 1, 3, 3) * 0.1, torch.randn(9, 3, 3, 3) * 0.1, torch.randn(1001) * 0.1,
         torch.randn(1, 4099) * 0.1]   # scalar layouts: odd rows (packed in pairs), odd numel, one odd long row
    cases = [(mode, bits) for mode in range(4) for bits in (4, 3, 2)]
    items, refs = [], []
    for w in ws:
        for mode, bits in cases:
            wd = w.to(DEV).contiguous()
            items.append(allocate(wd, bits=bits, per_channel=mode >= 2, symmetric=mode in (1, 3), khw=khw_of(wd),
                                  want_esum=True, clip=(-0.2, 0.2) if mode == 3 else None, pack_int4=True))
            refs.append((w.numpy(), mode, bits, khw_of(wd)))
    plan = SweepPlan(items)
    plan.execute()
    torch.cuda.synchronize()
    for it, (x, mode, bits, khw) in zip(items, refs):
        o = O.quantize(x, bits, mode, rows=x.shape[0] if mode >= 2 else 1, khw=khw, flags=1 if mode == 3 else 0,
                       clip=(-0.2, 0.2), want_esum=True)
        assert np.array_equal(it.dst.cpu().numpy(), o["dq"]), (x.shape, mode, bits)
        assert np.array_equal(it.codes.cpu().numpy(), _pack_nibbles(o["codes"])), (x.shape, mode, bits)
        assert np.array_equal(it.esum.cpu().numpy(), o["esum"])
    plan.destroy()
    # per channel, odd rows longer than half a task cannot pair up: rejected
    bad = allocate(torch.randn(3, 1025, device=DEV), bits=4, per_channel=True, pack_int4=True)
    with pytest.raises(NotImplementedError):
        SweepPlan([bad])


def test_tensor_past_int32_elements():
    """Maximum sizes: one tensor of 2^31 + 36 elements (64-bit element offsets in
    the task table, 1M+ tasks, two-launch per-tensor range) and per-channel rows
    of 2^20 elements; checked with oracle-free properties on the device and the
    oracle on slices (the per-tensor range taken from torch's min/max)."""
    from data_free_quantization_amd.sweep import allocate, SweepPlan
    n = (1 << 31) + 36
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.empty(n, device=DEV).normal_(0, 1, generator=g)
    x[n - 1] = 9.0   # the range's max sits past 2^31
    it = allocate(x, bits=8, per_channel=False, symmetric=False)
    plan = SweepPlan([it])
    plan.execute()
    torch.cuda.synchronize()
    mn, mx = float(x.min()), float(x.max())
    assert mx == 9.0
    for lo in (0, (1 << 31) - 1000, n - 2048):
        xs = x[lo:lo + 2048].cpu().numpy()
        o = O.quantize(xs, 8, O.TENSOR_ASYM, rows=1, flags=O.F_GIVEN, given=(mn, mx))
        assert np.array_equal(it.dst[lo:lo + 2048].cpu().numpy(), o["dq"])
        assert np.array_equal(it.codes[lo:lo + 2048].cpu().numpy(), o["codes"])
    assert float(it.zero[0]) == mn
    regen = it.codes.float() * it.scale[0] + it.zero[0]
    assert torch.equal(regen, it.dst)
    plan.destroy()
    del x, it, regen
    torch.cuda.empty_cache()
    w = torch.empty(8, 1 << 20, device=DEV).normal_(0, 1, generator=g)
    it = allocate(w, bits=4, per_channel=True, symmetric=True, want_esum=True)
    plan = SweepPlan([it])
    plan.execute()
    torch.cuda.synchronize()
    o = O.quantize(w.cpu().numpy(), 4, O.CHANNEL_SYM, rows=8, want_esum=True)
    assert np.array_equal(it.dst.cpu().numpy(), o["dq"]) and np.array_equal(it.esum.cpu().numpy(), o["esum"])
    plan.destroy()


_FUZZ_SEEDS = [int(v) for v in __import__("os").environ.get("DFQ_FUZZ_SEEDS", "1,2,3").split(",")]


@pytest.mark.parametrize("seed", _FUZZ_SEEDS)
def test_random_mixed_plans_vs_oracle(seed):
    """Fuzz: one plan of 40 random tensors -- rows 1..300, odd and even row lengths,
    KH*KW in {1, 4, 9, 25, 49}, all four modes, 2..16 bits, clip, given per-tensor
    ranges (Python doubles and fp32 bounds), device-resident ranges
    (DFQ_DEVICE_RANGE, fp64 or fp32 scale), E sums, packed nibbles, unaligned
    views -- every output bit-exact with the oracle."""
    from data_free_quantization_amd import _lib
    import ctypes as C
    from data_free_quantization_amd.sweep import SweepItem, SweepPlan, code_dtype
    rng = np.random.default_rng(seed)
    items, refs = [], []
    for _ in range(40):
        khw = int(rng.choice([1, 1, 4, 9, 25, 49]))
        rows = int(rng.integers(1, 300))
        row_len = khw * int(rng.choice([1, 3, 7, 16, 32, 100, 257, 512])) + (0 if khw > 1 else int(rng.integers(0, 3)))
        mode = int(rng.integers(0, 4))
        bits = int(rng.choice([2, 3, 4, 5, 8, 8, 8, 12, 16]))
        sym = mode in (1, 3)
        x = (rng.standard_normal((rows, row_len)) * rng.choice([1e-3, 0.1, 1.0, 30.0])).astype(np.float32)
        offset = int(rng.integers(0, 2))   # an unaligned view (scalar path) now and then
        base = torch.from_numpy(np.concatenate([np.zeros(offset, np.float32), x.reshape(-1)])).to(DEV)
        src = base[offset:].view(rows, row_len)
        flags, given = 0, (0.0, 0.0)
        clip = None
        if rng.random() < 0.3:
            clip = tuple(sorted(float(v) for v in rng.normal(0, np.abs(x).max() / 2 + 1e-6, 2)))
            flags |= O.F_CLIP
        if mode < 2 and rng.random() < 0.3:
            flags |= O.F_GIVEN | (O.F_F32 if rng.random() < 0.5 else 0)
            given = (float(x.min()) * 0.8, float(x.max()) * 0.9)
        dev_range = mode < 2 and not (flags & O.F_GIVEN) and rng.random() < 0.4   # DFQ_DEVICE_RANGE
        if dev_range and rng.random() < 0.5:
            flags |= O.F_F32
        esum = rng.random() < 0.5
        pack = bits <= 4 and rng.random() < 0.5 and not (mode >= 2 and row_len % 2 and 2 * row_len > 2048 and rows > 1)
        npar = rows if mode >= 2 else 1
        it = SweepItem(src=src, bits=bits, per_channel=mode >= 2, symmetric=sym, dst=torch.empty_like(src),
                       codes=(torch.empty((rows * row_len + 1) // 2, dtype=torch.uint8, device=DEV) if pack else
                              torch.empty(src.shape, dtype=code_dtype(bits, sym), device=DEV)),
                       scale=torch.empty(npar, device=DEV), zero=torch.empty(npar, device=DEV),
                       esum=torch.empty(rows * row_len // khw, device=DEV) if esum else None, khw=khw, clip=clip,
                       rows=rows if mode >= 2 else 1, pack_int4=pack)
        items.append(it)
        refs.append((x, mode, bits, khw, flags, clip, given, esum, pack, dev_range))
    plan = SweepPlan(items)
    # given ranges go through the descriptor (SweepItem has no field for them)
    L = _lib.load()
    descs = (_lib.TensorDesc * len(items))()
    ranges = []
    for i, (it, r) in enumerate(zip(items, refs)):
        x, mode, bits, khw, flags, clip, given, esum, pack, dev_range = r
        d = descs[i]
        d.src, d.dst = it.src.data_ptr(), it.dst.data_ptr()
        d.codes, d.scale, d.zero = it.codes.data_ptr(), it.scale.data_ptr(), it.zero.data_ptr()
        d.esum = it.esum.data_ptr() if esum else None
        d.rows = x.shape[0] if mode >= 2 else 1
        d.row_len = x.size // d.rows
        d.khw, d.bits, d.mode = khw, bits, mode
        d.flags = (flags & 7) | (_lib.DFQ_PACK_INT4 if pack else 0)
        if clip is not None:
            d.clip_lo, d.clip_hi = clip
        d.given_min, d.given_max = given
        if dev_range:   # the tensor's range left on the device by dfq_range
            rb = torch.empty(2, dtype=torch.int32, device=DEV)
            _lib.check(L.dfq_range(it.src.data_ptr(), it.src.numel(), rb.data_ptr(),
                                   C.c_void_p(torch.cuda.current_stream().cuda_stream)), "dfq_range")
            ranges.append(rb)
            d.flags |= _lib.DFQ_DEVICE_RANGE
            d.range_enc = rb.data_ptr()
    plan.destroy()
    p = C.c_void_p()
    _lib.check(L.dfq_sweep_plan_create(descs, len(items), C.byref(p)), "create")
    _lib.check(L.dfq_sweep_plan_execute(p, C.c_void_p(torch.cuda.current_stream().cuda_stream)), "execute")
    torch.cuda.synchronize()
    for it, (x, mode, bits, khw, flags, clip, given, esum, pack, _dr) in zip(items, refs):
        o = O.quantize(x, bits, mode, rows=x.shape[0] if mode >= 2 else 1, khw=khw, flags=flags,
                       clip=clip or (0.0, 0.0), given=given, want_esum=esum)
        tag = (x.shape, mode, bits, khw, flags, pack)
        assert np.array_equal(it.dst.cpu().numpy(), o["dq"]), tag
        if pack:
            c = o["codes"].reshape(-1).astype(np.uint8) & 0xF
            c = np.append(c, np.zeros(c.size % 2, np.uint8))
            assert np.array_equal(it.codes.cpu().numpy(), c[0::2] | (c[1::2] << 4)), tag
        else:
            assert np.array_equal(it.codes.cpu().numpy().view(o["codes"].dtype).reshape(x.shape),
                                  o["codes"].reshape(x.shape)), tag
        assert np.array_equal(it.scale.cpu().numpy(), o["scale"]), tag
        assert np.array_equal(it.zero.cpu().numpy() + np.float32(0), o["zero"] + np.float32(0)), tag
        if esum:
            assert np.array_equal(it.esum.cpu().numpy(), o["esum"]), tag
    L.dfq_sweep_plan_destroy(p)


@pytest.mark.parametrize("pack", [False, True])
def test_row_groups_equal_default_tasks(pack, monkeypatch):
    """Row groups (diagnostics library, DFQ_SWEEP_GROUP_ROWS=1: R whole rows of
    1,025-8,192 elements split over the 4 waves of a block, row ranges combined
    through LDS) give the same bytes as the product's whole-row tasks and
    block-row pieces, including the KH*KW error sums and packed INT4 codes."""
    from data_free_quantization_amd import _lib
    from data_free_quantization_amd.sweep import allocate, SweepPlan, khw_of
    rng = np.random.default_rng(41)
    shapes = [(37, 128, 3, 3), (21, 256, 3, 3), (9, 320, 3, 3), (40, 1280), (13, 1100), (5, 512, 3, 3), (7, 2048)]
    xs = [rng.normal(0, 1, s).astype(np.float32) for s in shapes]
    outs = []
    for lib in ("product", "groups"):
        if lib == "groups":
            monkeypatch.setattr(_lib, "_LIB", _lib.load_diag())
            monkeypatch.setenv("DFQ_SWEEP_GROUP_ROWS", "1")
        items = []
        for x in xs:
            t = torch.from_numpy(x).to(DEV)
            items.append(allocate(t, bits=4 if pack else 8, per_channel=True, symmetric=not pack, khw=khw_of(t),
                                  want_esum=True, clip=(-1.5, 1.5), pack_int4=pack))
        plan = SweepPlan(items)
        plan.execute()
        torch.cuda.synchronize()
        outs.append((plan.stats["n_tasks_main"], items))
        plan.destroy()
    assert outs[0][0] != outs[1][0]   # the group layout really was used
    for a, b in zip(outs[0][1], outs[1][1]):
        for f in ("dst", "codes", "scale", "zero", "esum"):
            assert torch.equal(getattr(a, f), getattr(b, f)), f


def test_device_range_argument_errors():
    """DFQ_DEVICE_RANGE is a per-tensor flag with a range pointer: per-channel
    modes, a missing pointer, or DFQ_GIVEN_RANGE together with it are rejected
    before anything is enqueued (include/dfq_hip.h)."""
    import ctypes as C
    from data_free_quantization_amd import _lib
    from data_free_quantization_amd.sweep import _DESC
    L = _lib.load()
    w = torch.randn(8, 16, device=DEV)
    r = torch.zeros(2, dtype=torch.int32, device=DEV)

    def rc(mode, flags, rng):
        tab = np.zeros(1, dtype=_DESC)
        tab[0]["src"] = tab[0]["dst"] = w.data_ptr()
        tab[0]["rows"], tab[0]["row_len"], tab[0]["khw"], tab[0]["bits"] = 8 if mode >= 2 else 1, \
            128 if mode < 2 else 16, 1, 8
        tab[0]["mode"], tab[0]["flags"], tab[0]["range_enc"] = mode, flags, rng
        return int(L.dfq_sweep_plan_ws_bytes(tab.ctypes.data_as(C.POINTER(_lib.TensorDesc)), 1))

    assert rc(_lib.DFQ_TENSOR_ASYM, _lib.DFQ_DEVICE_RANGE, r.data_ptr()) > 0
    assert rc(_lib.DFQ_CHANNEL_ASYM, _lib.DFQ_DEVICE_RANGE, r.data_ptr()) < 0
    assert rc(_lib.DFQ_TENSOR_ASYM, _lib.DFQ_DEVICE_RANGE, 0) < 0
    assert rc(_lib.DFQ_TENSOR_SYM, _lib.DFQ_DEVICE_RANGE | _lib.DFQ_GIVEN_RANGE, r.data_ptr()) < 0


def test_preload_is_idempotent():
    """dfq_preload (code objects + the CLE stream on the current device) can run
    any number of times."""
    from data_free_quantization_amd import _lib
    L = _lib.load()
    assert L.dfq_preload() == 0 and L.dfq_preload() == 0
    _lib.preload()


@pytest.mark.parametrize("bits,mode", [(8, 3), (8, 2), (4, 2), (4, 3), (2, 2), (16, 3)])
def test_screened_quantize_at_rounding_boundaries(bits, mode):
    """The sweep's screened reciprocal quantize (csrc/dfq_common.h qdq_screen) takes
    the IEEE divide only near a half-integer quotient.  Rows built so that most
    elements sit ON a half-integer of their row's scale or 1-3 ulps either side
    (ties to even, the screen's decision band), plus the clamp edges: dq, codes,
    scale and E bit-exact with the oracle (oracle/dfq_oracle.c, the reference's
    true division)."""
    from data_free_quantization_amd.sweep import allocate, SweepPlan
    rng = np.random.default_rng(bits * 10 + mode)
    sym = mode in (1, 3)
    qmax = (1 << (bits - 1)) - 1 if sym else (1 << bits) - 1
    rows, cols = 96, 2 * 9 * 64
    x = np.empty((rows, cols), np.float32)
    for o in range(rows):
        lo, hi = float(np.float32(-rng.uniform(0.1, 3.0))), float(np.float32(rng.uniform(0.1, 3.0)))
        # the row's own scale and zero (what the kernel will derive from its range)
        s = np.float32(max(max(abs(lo), abs(hi)) / qmax, 1e-8)) if sym else np.float32(max((hi - lo) / qmax, 1e-8))
        mn = np.float32(0.0) if sym else np.float32(lo)
        k = rng.integers(-qmax - 1 if sym else 0, qmax, cols)
        v = ((k + 0.5) * s.astype(np.float64) + mn).astype(np.float32)
        steps = rng.integers(-3, 4, cols).astype(np.int32)
        v = (v.view(np.int32) + steps).view(np.float32)
        v[0], v[1] = lo, hi   # pin the row's range
        x[o] = np.clip(v, lo, hi)
    t = torch.from_numpy(x.reshape(rows, 2, 9 * 64 // 9, 9)).to(DEV)   # KH*KW = 9 (3x3 error sums)
    t = t.reshape(rows, 128, 3, 3).contiguous()
    it = allocate(t, bits=bits, per_channel=True, symmetric=sym, khw=9, want_esum=True, clip=(-2.5, 2.5))
    plan = SweepPlan([it])
    plan.execute()
    torch.cuda.synchronize()
    xh = t.cpu().numpy()
    o = O.quantize(xh, bits, mode, rows=rows, khw=9, flags=O.F_CLIP, clip=(-2.5, 2.5), want_esum=True)
    assert np.array_equal(it.dst.cpu().numpy(), o["dq"])
    assert np.array_equal(it.codes.cpu().numpy().view(o["codes"].dtype), o["codes"])
    assert np.array_equal(it.scale.cpu().numpy(), o["scale"])
    assert np.array_equal(it.esum.cpu().numpy(), o["esum"])
    plan.destroy()


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("row_len", [64, 9])
@pytest.mark.parametrize("bits,clip", [(8, None), (8, (-0.75, 0.75)), (4, None)])
def test_signed_zeros_and_tiny_values_bitwise(mode, row_len, bits, clip):
    """The sweep's fixed-form loop rounds with (t + 1.5*2^23) - 1.5*2^23, which gives
    +0 where rintf gives -0 (t in (-0.5, -0]); the dequantized value is q*s + mn,
    so the sign only survives when mn is -0.  Rows with -0.0 / +0.0 entries, a -0.0
    row minimum, all-zero rows of either sign and denormal-to-tiny magnitudes,
    on the vector (64) and scalar (9) paths: dq compared BIT FOR BIT with the
    oracle (signed zeros not folded), codes, scale and zero exactly."""
    from data_free_quantization_amd.sweep import allocate, SweepPlan
    rng = np.random.default_rng(bits * 100 + mode * 10 + row_len)
    rows = 48
    x = rng.standard_normal((rows, row_len)).astype(np.float32) * np.float32(0.5)
    x[0] = 0.0
    x[1] = -0.0
    x[2, :] = np.abs(x[2]); x[2, 0] = -0.0            # row minimum -0.0 (asym mn = -0)
    x[3, :] = np.abs(x[3]); x[3, 0] = 0.0             # row minimum +0.0
    x[4] = np.float32(1e-40) * rng.choice([-1, 1], row_len)   # denormals
    x[5] = np.float32(1e-30) * rng.standard_normal(row_len).astype(np.float32)
    x[6, ::2] = -0.0
    x[7, ::3] = 0.0
    x[8] = -np.abs(x[8]); x[8, -1] = -0.0             # row maximum -0.0
    t = torch.from_numpy(x).to(DEV)
    per_channel, sym = mode >= 2, mode in (1, 3)
    it = allocate(t, bits=bits, per_channel=per_channel, symmetric=sym, khw=1, want_esum=True, clip=clip,
                  pack_int4=False)
    plan = SweepPlan([it])
    plan.execute()
    torch.cuda.synchronize()
    o = O.quantize(x, bits, mode, rows=rows, khw=1, flags=O.F_CLIP if clip else 0, clip=clip or (0.0, 0.0),
                   want_esum=True)
    got = it.dst.cpu().numpy()
    assert np.array_equal(got.view(np.int32), o["dq"].view(np.int32)), "dq differs bitwise (signed zero or value)"
    assert np.array_equal(it.codes.cpu().numpy().view(o["codes"].dtype), o["codes"])
    assert np.array_equal(it.scale.cpu().numpy().view(np.int32), o["scale"].view(np.int32))
    assert np.array_equal(it.zero.cpu().numpy().view(np.int32), o["zero"].view(np.int32))
    assert np.array_equal(it.esum.cpu().numpy().view(np.int32), o["esum"].view(np.int32))
    plan.destroy()
