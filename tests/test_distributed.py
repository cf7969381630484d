"""Layer-sharded sweep across ranks (data_free_quantization_amd/distributed.py).

CPU: world_size-2 (and 3) gloo processes; the per-rank compute is the oracle
(the checker), so what is under test is the partition, the slab layout and the
collectives (scatter / broadcast from rank 0, gather to rank 0, in-place
all-gather).  The GPU tests run the same object with the HIP sweep under RCCL
("nccl") at world size 1, so the RCCL branch executes, and a 2-rank gloo
rehearsal with both ranks on the one GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from data_free_quantization_amd import distributed as D

SHAPES = [(32, 3, 3, 3), (32, 1, 3, 3), (16, 32, 1, 1), (96, 16, 1, 1), (96, 1, 3, 3), (24, 96, 1, 1),
          (10, 24), (7, 5, 3, 3), (1, 1), (64, 24, 1, 1)]


def _weights(seed=0, shapes=SHAPES):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(s, generator=g) * (0.1 + i) for i, s in enumerate(shapes)]


def _specs(shapes=SHAPES, **kw):
    cfg = dict(bits=8, per_channel=True, symmetric=True, want_esum=True)
    cfg.update(kw)
    return D.uniform_specs(shapes, **cfg)


def _pack_nibbles(c):
    c = (np.asarray(c).reshape(-1).astype(np.int32) & 0xF).astype(np.uint8)
    if c.size % 2:
        c = np.concatenate([c, np.zeros(1, np.uint8)])
    return (c[0::2] | (c[1::2] << 4)).astype(np.uint8)


def _oracle_layer(w, s):
    """The oracle's outputs for one layer spec (codes packed like DFQ_PACK_INT4)."""
    r = _oracle_layer_raw(w, s)
    if s.pack_int4:
        r = dict(r, codes=_pack_nibbles(r["codes"]))
    return r


def _oracle_layer_raw(w, s):
    from oracle import oracle as O
    mode = (O.CHANNEL_SYM if s.symmetric else O.CHANNEL_ASYM) if s.per_channel else \
        (O.TENSOR_SYM if s.symmetric else O.TENSOR_ASYM)
    flags = O.F_CLIP if s.clip is not None else 0
    return O.quantize(w.cpu().numpy(), s.bits, mode, rows=s.rows, khw=s.khw, flags=flags,
                      clip=s.clip or (0.0, 0.0), want_esum=s.want_esum)


def _oracle_compute(sw, indices):
    """The checker as the per-rank compute: writes into the rank's output slab."""
    for i in indices:
        r = _oracle_layer(sw.weight(i), sw.specs[i])
        o = sw.outputs(i)
        for f in D.FIELDS:
            t = getattr(o, f)
            if t is not None:
                t.copy_(torch.from_numpy(np.ascontiguousarray(r[f])).view(t.dtype).view(t.shape))


def _check(out, w, spec):
    r = _oracle_layer(w, spec)
    for f in D.FIELDS:
        t = getattr(out, f)
        if t is None:
            continue
        np.testing.assert_array_equal(t.cpu().numpy(), np.asarray(r[f]).reshape(t.shape))


def test_partition_lpt():
    sizes = [100, 90, 10, 10, 10, 5, 1]
    parts = D.partition(sizes, 2)
    assert sorted(i for p in parts for i in p) == list(range(len(sizes)))
    loads = [sum(sizes[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(sizes)
    assert D.partition(sizes, 2) == parts                      # deterministic
    assert D.partition([], 3) == [[], [], []]
    assert D.partition(sizes, 1) == [list(range(len(sizes)))]
    many = D.partition(sizes, 16)
    assert sum(1 for p in many if p) == len(sizes)
    with pytest.raises(ValueError):
        D.partition(sizes, 0)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_layout_slabs(world):
    specs = _specs(pack_int4=False) + _specs([(5, 7), (33,)], bits=4, per_channel=False, symmetric=False,
                                             pack_int4=True, want_esum=False)
    L = D.ShardLayout(specs, world)
    assert sorted(i for p in L.parts for i in p) == list(range(len(specs)))
    for r, p in enumerate(L.parts):
        for f in L.fields:
            spans = []
            for i in p:
                assert L.owner[i] == r
                if f not in L.off[i]:
                    continue
                assert L.off[i][f] % (D.SMALL_ALIGN if f in ("scale", "zero") else D.ALIGN) == 0
                spans.append((L.off[i][f], L.off[i][f] + L.nbytes(i, f)))
            spans.sort()
            assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))   # no overlap inside a slab
            assert (spans[-1][1] if spans else 0) <= L.used[f][r] <= L.cap[f]
            assert L.cap[f] % D.ALIGN == 0
    # packed INT4 codes: ceil(n/2) bytes
    assert specs[-1].outputs()["codes"][0] == (17,)


def test_single_process_no_dist():
    """world 1 without torch.distributed: run() + gather() are local."""
    ws = _weights()
    specs = _specs()
    sw = D.ShardedSweep(specs, device="cpu", compute=_oracle_compute)
    for i, w in enumerate(ws):
        sw.weight(i).copy_(w)
    sw.run()
    sw.gather("root")
    for i, w in enumerate(ws):
        _check(sw.outputs(i), w, specs[i])


def test_sources_mode_cpu():
    ws = _weights(3)
    specs = _specs(symmetric=False, clip=(-0.5, 0.5))
    sw = D.ShardedSweep(specs, sources=ws, compute=_oracle_compute)
    assert sw.in_arena is None
    sw.run()
    for i, w in enumerate(ws):
        assert sw.weight(i) is ws[i]
        _check(sw.outputs(i), w, specs[i])
    with pytest.raises(RuntimeError):
        sw.scatter()


def test_bad_sources():
    with pytest.raises(ValueError):
        D.ShardedSweep(_specs(), sources=_weights()[:3], compute=_oracle_compute)
    ws = _weights()
    ws[0] = ws[0].reshape(-1)
    with pytest.raises(ValueError):
        D.ShardedSweep(_specs(), sources=ws, compute=_oracle_compute)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ws = _weights()
        specs = _specs()
        flat = {}
        if mode == "sources_all":            # main_dfq: every rank holds the model
            sw = D.ShardedSweep(specs, sources=ws, replicate=True, compute=_oracle_compute, device="cpu")
            sw.run()
            sw.gather("all")
        else:                                # bench: rank 0 holds the layer list
            sw = D.ShardedSweep(specs, replicate=(mode == "broadcast_all"), compute=_oracle_compute, device="cpu")
            if rank == 0:
                for i, w in enumerate(ws):
                    sw.weight(i).copy_(w)
            if mode == "broadcast_all":
                sw.broadcast()
            else:
                sw.scatter()
            for i in sw.mine:                # every rank now holds its own inputs
                assert torch.equal(sw.weight(i), ws[i])
            sw.run()
            if mode == "scatter_root":
                sw.gather("root")
            elif mode == "broadcast_all":
                sw.gather("all")
        for i, o in sw.result().items():
            if mode == "scatter_none" and i not in sw.mine:
                continue
            for f in D.FIELDS:
                t = getattr(o, f)
                if t is not None:
                    flat[f"{i}_{f}"] = t.numpy()
        flat["tmax"] = np.array([D.max_over_ranks(1.5 + rank)])     # bench.py's max-over-ranks step time
        flat["mine"] = np.array(sw.mine, dtype=np.int64)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **flat)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "scatter_root"), (2, "scatter_none"), (2, "broadcast_all"),
                                        (2, "sources_all"), (3, "scatter_root")])
def test_sharded_sweep_gloo(tmp_path, world, mode):
    mp.spawn(_worker, args=(world, _free_port(), mode, str(tmp_path)), nprocs=world, join=True)
    ws = _weights()
    specs = _specs()
    parts = D.ShardLayout(specs, world).parts
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npz")
        assert got["tmax"][0] == 1.5 + world - 1
        assert list(got["mine"]) == parts[r]
        have = sorted({int(k.split("_")[0]) for k in got.files if k not in ("tmax", "mine")})
        if mode in ("broadcast_all", "sources_all") or (mode == "scatter_root" and r == 0):
            assert have == list(range(len(ws)))
        else:
            assert have == parts[r]
        for i in have:
            r_ = _oracle_layer(ws[i], specs[i])
            for f in D.FIELDS:
                if f"{i}_{f}" in got.files:
                    np.testing.assert_array_equal(got[f"{i}_{f}"], np.asarray(r_[f]).reshape(got[f"{i}_{f}"].shape))


# ---------------------------------------------------------------------------- GPU
def _gpu_specs_mixed():
    return (_specs() +
            D.uniform_specs([(64, 16, 3, 3), (48, 40)], bits=4, per_channel=True, symmetric=False,
                            clip=(-1.0, 1.0), pack_int4=True) +
            D.uniform_specs([(128, 64, 1, 1)], bits=8, per_channel=False, symmetric=False))


@pytest.mark.gpu
def test_sharded_sweep_rccl_world1():
    """The RCCL branch: init_process_group("nccl") at world size 1; broadcast, the
    HIP sweep into the arena, in-place all_gather_into_tensor; bit-exact vs the
    oracle."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        specs = _gpu_specs_mixed()
        ws = _weights(5, [s.shape for s in specs])
        sw = D.ShardedSweep(specs, replicate=True, device=dev)
        for i, w in enumerate(ws):
            sw.weight(i).copy_(w)
        sw.broadcast()
        sw.run()
        sw.gather("all")
        sw.gather("root")
        assert D.max_over_ranks(2.5, dev) == 2.5
        torch.cuda.synchronize()
        for i, w in enumerate(ws):
            _check(sw.outputs(i), w, specs[i])
        # sources mode (main_dfq): the sweep reads the replicated tensors in place
        src = [w.to(dev) for w in ws]
        sw2 = D.ShardedSweep(specs, sources=src, replicate=True)
        sw2.run()
        sw2.gather("all")
        torch.cuda.synchronize()
        for i, w in enumerate(ws):
            _check(sw2.outputs(i), w, specs[i])
        sw.destroy()
        sw2.destroy()
    finally:
        dist.destroy_process_group()


def _configs4_specs():
    """BASELINE configs[4]'s layer list: every ResNet-50 target layer, per-channel
    asymmetric INT4 + clip [-15, 15], packed int4 codes (bench.SECONDARY's
    "resnet50 per-ch asym INT4 + clip, packed int4 codes")."""
    from data_free_quantization_amd import zoo
    shapes = [tuple(m.weight.shape) for m in zoo.target_layers(zoo.MODELS["resnet50"]())]
    return D.uniform_specs(shapes, bits=4, per_channel=True, symmetric=False, want_esum=False,
                           clip=(-15.0, 15.0), pack_int4=True)


def _configs4_weights(specs):
    """Synthetic conv init of bench.synth_weight (N(0, sqrt(2 / (k*k*O))), Linear N(0, 0.01))."""
    g = torch.Generator().manual_seed(9)
    out = []
    for s in specs:
        shp = s.shape
        std = (2.0 / (shp[2] * shp[3] * shp[0])) ** 0.5 if len(shp) == 4 else 0.01
        out.append(torch.randn(shp, generator=g) * std)
    return out


def _gpu_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        specs = _configs4_specs()
        ws = _configs4_weights(specs)
        sw = D.ShardedSweep(specs, replicate=True, device=torch.device("cuda:0"))
        if rank == 0:
            for i, w in enumerate(ws):
                sw.weight(i).copy_(w)
        sw.scatter()
        sw.run()
        sw.gather("root")
        torch.cuda.synchronize()
        ok_root = 0
        if rank == 0:   # rank 0 holds every layer's outputs after gather("root")
            for i in range(len(specs)):
                _check(sw.outputs(i), ws[i], specs[i])
                ok_root += 1
        sw.gather("all")
        torch.cuda.synchronize()
        ok_all = 0
        for i in range(len(specs)):   # every rank holds every layer's outputs after gather("all")
            _check(sw.outputs(i), ws[i], specs[i])
            ok_all += 1
        np.save(os.path.join(outdir, f"r{rank}.npy"), np.array([ok_root, ok_all, len(sw.mine)]))
        sw.destroy()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_sweep_two_ranks_one_gpu(tmp_path):
    """2-rank rehearsal of BASELINE configs[4] on the one GPU (gloo between the
    processes): the ResNet-50 INT4 + clip layer list (54 layers, 25.5 M weights),
    LPT-sharded; rank 0 holds the list and scatters, both ranks run the HIP sweep
    on their shard, then gather("root") (rank 0 checks every layer against the
    oracle) and gather("all") (both ranks check every layer): bit-exact."""
    mp.spawn(_gpu_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    n = len(_configs4_specs())
    r0, r1 = np.load(tmp_path / "r0.npy"), np.load(tmp_path / "r1.npy")
    assert r0[0] == n and r1[0] == 0
    assert r0[1] == n and r1[1] == n
    assert r0[2] > 0 and r1[2] > 0 and r0[2] + r1[2] == n
