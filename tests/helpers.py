"""Shared test helpers: golden fixture access and mode names."""
import hashlib
import json
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"

MODE_IDS = {"tensor_asym": 0, "tensor_sym": 1, "channel_asym": 2, "channel_sym": 3}


def h(a) -> str:
    """sha256 of fp32 bytes with -0 folded into +0 (as tests/golden/make_golden.py)."""
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32)) + np.float32(0.0)
    return hashlib.sha256(a.tobytes()).hexdigest()


def hb(a) -> bytes:
    return bytes.fromhex(h(a))


def quant_cases():
    z = np.load(GOLDEN / "quant_cases.npz", allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    out = []
    for i, m in enumerate(meta):
        case = dict(m)
        case["idx"] = i
        case["x"] = z[f"in{m['input']}"]
        case["dq"] = z[f"dq{i}"] if f"dq{i}" in z.files else None
        case["dqh"] = str(z[f"dqh{i}"])
        case["esum_ref"] = z[f"esum{i}"] if f"esum{i}" in z.files else None
        out.append(case)
    return out


def case_flags(case):
    """(mode, rows, flags, given) for the oracle/kernels."""
    mode = MODE_IDS[case["mode"]]
    x = case["x"]
    rows = x.shape[0] if mode >= 2 else 1
    flags = 0
    given = (0.0, 0.0)
    if case["given"] is not None:
        flags |= 2
        given = tuple(case["given"])
    if case["default_range"]:
        flags |= 4
    if case["clip"] is not None:
        flags |= 1
    return mode, rows, flags, given


def transform_cases():
    z = np.load(GOLDEN / "transform_cases.npz", allow_pickle=False)
    return z, json.loads(str(z["meta"]))


def pipeline(name, threads=8, bits_weight=8):
    """The reference's main_dfq stage order on the synthetic model, run with
    ``threads`` torch intra-op threads (tests/golden/make_golden.py:pipeline);
    ``bits_weight`` 4: the --bits_weight 4 run (pipeline_<name>_w4.npz, 8 threads)."""
    if bits_weight != 8:
        assert threads == 8, "the W4 fixtures are 8-thread runs"
        return np.load(GOLDEN / f"pipeline_{name}_w{bits_weight}.npz", allow_pickle=False)
    f = f"pipeline_{name}.npz" if threads == 8 else f"pipeline_{name}_t{threads}.npz"
    return np.load(GOLDEN / f, allow_pickle=False)


def recover_codes_consistent(dq, codes, scale, zero):
    """dq == fl(fl(code * s) + zero) elementwise (codes regenerate the output)."""
    s = np.float32(scale)
    z = np.float32(zero)
    regen = (codes.astype(np.float32) * s).astype(np.float32) + z
    return np.array_equal(regen.astype(np.float32), dq)


def chunk_cases():
    """quantize() with num_chunks / a None bound (tests/golden/chunk_cases.npz)."""
    z = np.load(GOLDEN / "chunk_cases.npz", allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    out = []
    for i, m in enumerate(meta):
        case = dict(m)
        case["idx"] = i
        case["x"] = z[f"in{m['input']}"]
        if m["error"] is None:
            case["range"] = z[f"range{i}"]
            case["dq"] = z[f"dq{i}"]
            case["dqh"] = str(z[f"dqh{i}"])
        out.append(case)
    return out


def chunk_kwargs(case):
    """quantize() keyword arguments of a chunk case."""
    kw = dict(symmetric=case["sym"], num_chunks=case["num_chunks"])
    if case["given"] is not None:
        kw[f"{case['given'][0]}_value"] = case["given"][1]
    return kw
