"""Quantized-weight export: the integer grid the sweep produced, in a deployable
file (an extension on the output side of the DFQ path; the reference keeps only
fake-quantized fp32 weights).

``save(path, graph, state, ...)`` writes one safetensors file with, per target
layer key ``k``: ``k.codes`` (the grid indices as the sweep wrote them: int8 /
uint8 / int16, or packed nibbles; asymmetric codes above 8 bits are unsigned
16-bit patterns held in int16, recorded as ``code_storage: "u16_in_i16"``),
``k.scale``, ``k.zero`` ([rows] per channel, [1] per tensor) and ``k.bias`` (the final fp32 bias after bias correction), plus
metadata (bits, granularity, symmetric, clip, shapes).  ``load(path)`` returns
the tensors; ``dequantize(entry)`` rebuilds the fp32 weight exactly as the sweep
did: ``clamp(fl(fl(q * s) + zero), clip)``.
"""
from __future__ import annotations

import json
from typing import Dict, Optional, Sequence

import torch

from safetensors.torch import load_file, save_file


def save(path, graph, state: Dict, *, bits: int, granularity: str, symmetric: bool,
         clip: Optional[Sequence[float]] = None, packed: bool = False) -> Dict[str, dict]:
    tensors, layers = {}, {}
    for key, st in state.items():
        layer = graph[key]
        k = str(key)
        w = layer.weight
        tensors[f"{k}.codes"] = st["codes"].detach().contiguous()
        tensors[f"{k}.scale"] = st["scale"].detach().contiguous()
        tensors[f"{k}.zero"] = st["zero"].detach().contiguous()
        if layer.bias is not None:
            tensors[f"{k}.bias"] = layer.bias.detach().contiguous()
        layers[k] = {"shape": list(w.shape), "type": type(layer).__name__}
    storage = "nibbles" if packed else ("i8" if symmetric else "u8") if bits <= 8 else \
        ("i16" if symmetric else "u16_in_i16")
    meta = {"format": "dfq-mi355x/1", "bits": bits, "granularity": granularity, "symmetric": symmetric,
            "clip": list(clip) if clip is not None else None, "packed_int4": packed, "code_storage": storage,
            "layers": layers}
    save_file({n: t.cpu() for n, t in tensors.items()}, str(path), metadata={"dfq": json.dumps(meta)})
    return layers


def load(path, device="cpu"):
    """(meta, {layer key: {codes, scale, zero[, bias]}}) from a file written by save()."""
    from safetensors import safe_open
    with safe_open(str(path), framework="pt") as f:
        meta = json.loads(f.metadata()["dfq"])
    flat = load_file(str(path), device=str(device))
    out = {}
    for name, t in flat.items():
        k, field = name.rsplit(".", 1)
        out.setdefault(k, {})[field] = t
    return meta, out


def dequantize(meta: dict, key: str, entry: Dict[str, torch.Tensor]) -> torch.Tensor:
    """fp32 weight of one exported layer, bit-identical to the sweep's output."""
    shape = meta["layers"][key]["shape"]
    q = entry["codes"]
    n = 1
    for s in shape:
        n *= s
    if meta.get("packed_int4"):
        c = q.to(torch.int32)
        q = torch.stack([c & 0xF, c >> 4], 1).view(-1)[:n]
        if meta["symmetric"]:
            q = torch.where(q >= 8, q - 16, q)
    elif not meta["symmetric"] and meta["bits"] > 8:
        # asymmetric codes 0 .. 2^b - 1 > 32767 are uint16 bit patterns in an int16
        # tensor (the sweep's (int16_t)(int)q): reinterpret, do not sign-extend
        q = q.to(torch.int32) & 0xFFFF
    rows = entry["scale"].numel()
    qf = q.reshape(rows, -1).to(torch.float32)
    y = qf * entry["scale"].view(-1, 1)      # fl(q * s)
    y = y + entry["zero"].view(-1, 1)        # fl(. + zero): separate roundings, as the kernel
    if meta.get("clip") is not None:
        y = y.clamp(meta["clip"][0], meta["clip"][1])
    return y.view(shape)
