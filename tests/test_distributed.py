"""Layer-sharded sweep across ranks (data_free_quantization_amd/distributed.py).

CPU: world_size-2 gloo processes; the per-rank compute is the oracle (the
checker), so what is under test is the partition, the pack/unpack layout and the
gather.  The GPU test runs the same sharded path with the HIP sweep at world 1.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from data_free_quantization_amd import distributed as D


def _weights(seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(32, 3, 3, 3), (32, 1, 3, 3), (16, 32, 1, 1), (96, 16, 1, 1), (96, 1, 3, 3), (24, 96, 1, 1),
              (10, 24), (7, 5, 3, 3), (1, 1), (64, 24, 1, 1)]
    return [torch.randn(s, generator=g) * (0.1 + i) for i, s in enumerate(shapes)]


def _khw(w):
    return int(w[0, 0].numel()) if w.dim() >= 3 else 1


def _oracle_compute(weights):
    from oracle import oracle as O

    def run(idx):
        outs = []
        for i in idx:
            w = weights[i]
            r = O.quantize(w.numpy(), 8, O.CHANNEL_SYM, khw=_khw(w), want_esum=True)
            outs.append(D.LayerOut(torch.from_numpy(r["dq"]), torch.from_numpy(r["codes"]),
                                   torch.from_numpy(r["scale"]), torch.from_numpy(r["zero"]),
                                   torch.from_numpy(r["esum"])))
        return outs
    return run


def _specs(weights):
    return [D.output_spec(w, True, 8, True, _khw(w), True) for w in weights]


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


def test_pack_unpack_roundtrip():
    ws = _weights()
    outs = _oracle_compute(ws)(list(range(len(ws))))
    specs = _specs(ws)
    buf = D._pack(outs, specs, torch.device("cpu"))
    back = D._unpack(buf, specs)
    for a, b in zip(outs, back):
        for f in ("dq", "codes", "scale", "zero", "esum"):
            assert torch.equal(getattr(a, f), getattr(b, f))
            assert getattr(a, f).dtype == getattr(b, f).dtype


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, gather, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ws = _weights()
        res = D.sharded_sweep(ws, _oracle_compute(ws), _specs(ws), gather=gather)
        flat = {f"{i}_{f}": getattr(o, f).numpy() for i, o in res.items()
                for f in ("dq", "codes", "scale", "zero", "esum")}
        flat["tmax"] = np.array([D.max_over_ranks(1.5 + rank)])     # bench.py's max-over-ranks step time
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **flat)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("gather", ["all", "rank0", "none"])
def test_sharded_sweep_gloo_world2(tmp_path, gather):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), gather, str(tmp_path)), nprocs=world, join=True)
    ws = _weights()
    full = _oracle_compute(ws)(list(range(len(ws))))
    parts = D.partition([w.numel() for w in ws], world)
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npz")
        assert got["tmax"][0] == 1.5 + world - 1
        have = sorted({int(k.split("_")[0]) for k in got.files if k != "tmax"})
        if gather == "all" or (gather == "rank0" and r == 0):
            assert have == list(range(len(ws)))
        else:
            assert have == parts[r]
        for i in have:
            for f in ("dq", "codes", "scale", "zero", "esum"):
                np.testing.assert_array_equal(got[f"{i}_{f}"], getattr(full[i], f).numpy())


@pytest.mark.gpu
def test_sharded_sweep_gpu_world1():
    from oracle import oracle as O
    ws = [w.cuda() for w in _weights()]
    res = D.sharded_sweep(ws, D.gpu_sweep(ws), _specs(ws))
    torch.cuda.synchronize()
    for i, w in enumerate(ws):
        r = O.quantize(w.cpu().numpy(), 8, O.CHANNEL_SYM, khw=_khw(w), want_esum=True)
        for f in ("dq", "codes", "scale", "zero", "esum"):
            np.testing.assert_array_equal(getattr(res[i], f).cpu().numpy(), r[f])
