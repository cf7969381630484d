"""TEST INFRASTRUCTURE: parity checks shared by the GPU tests, __graft_entry__.smoke()
and bench.py (which reports their mismatch counts in its JSON line).

* ``pipeline_mismatches``: the whole main_dfq stage order (main_dfq.py:188-231)
  on the GPU vs the reference's own run on the same synthetic model
  (tests/golden/pipeline_<model>.npz, written by make_golden.py by importing the
  reference).  Per stage: how many target weights / biases differ from the
  reference's bytes, plus the CLE iteration count, every per-iteration diff, the
  relations and the accumulated scales.
* ``sweep_mismatches``: sweep items (the bench's timed outputs) vs the C oracle
  (oracle/dfq_oracle.c) on the same input tensors: dq, codes, scale, zero, E.

Both return plain dicts of counts; 0 everywhere means parity.
"""
from __future__ import annotations

import numpy as np

try:
    from tests.helpers import hb, pipeline
except ImportError:   # imported with tests/ itself on sys.path
    from helpers import hb, pipeline

STAGES = ("bn1", "cle", "absorb", "bn2", "quant", "clip", "bc")


def pipeline_mismatches(name: str = "mobilenetv2", threads: int = 8, device="cuda:0", bits_weight: int = 8) -> dict:
    """Run run_dfq(bc_mode="reference") on zoo.build(name, seed=0, relu=True) and
    compare every stage with the reference fixture.  Tolerances are those of
    tests/test_gpu_pipeline.py: bit-exact except ResNet-50's post-absorption
    biases before bias correction (the reference's MKL sgemv order: 1e-5).
    ``bits_weight`` 4: main_dfq --bits_weight 4 (BASELINE configs[4]) against
    pipeline_<name>_w4.npz."""
    import torch
    import torch.nn as nn
    from data_free_quantization_amd import _lib, zoo
    from data_free_quantization_amd import Cross_layer_equal as cle
    from data_free_quantization_amd.pipeline import run_dfq
    from data_free_quantization_amd.utils.tracer import build_graph
    targ = (nn.Conv2d, nn.Linear)
    P = pipeline(name, threads, bits_weight)
    old_threads = _lib.REF_THREADS
    _lib.REF_THREADS = threads
    try:
        model = zoo.build(name, seed=0, relu=True).to(device)
        g = build_graph(model, "positional")
        graph, bottoms = g.getGraph(), g.getBottoms()
        tkeys = [k for k in graph if type(graph[k]) in targ]
        out = {"model": name, "ref_threads": threads, "bits_weight": bits_weight, "targets": len(tkeys),
               "target_keys_match": tkeys == list(P["targets"])}
        stage_bad = {}
        cle_info = {}

        def hook(stage):
            if stage not in STAGES:
                return
            ws = [hb(graph[k].weight.detach().cpu().numpy()) for k in tkeys]
            wbad = sum(int(w != bytes(P[f"{stage}_wh"][i])) for i, w in enumerate(ws))
            biases = [graph[k].bias.detach().cpu().numpy() if graph[k].bias is not None else np.zeros(0, np.float32)
                      for k in tkeys]
            if f"{stage}_bias" in P.files:
                got, ref = np.concatenate(biases), P[f"{stage}_bias"]
                if stage == "bc" or name != "resnet50":
                    bbad = int((got != ref).sum()) if got.shape == ref.shape else int(ref.size)
                else:
                    bbad = int((~np.isclose(got, ref, rtol=1e-5, atol=1e-5)).sum()) if got.shape == ref.shape \
                        else int(ref.size)
            else:
                bbad = sum(int(hb(b) != bytes(P[f"{stage}_bh"][i])) for i, b in enumerate(biases))
            stage_bad[stage] = {"weights": wbad, "biases": bbad}
            if stage == "cle":
                cle_info.update(iterations=cle.LAST_RUN["iterations"], diffs=list(cle.LAST_RUN["diffs"]))

        bc_error = str(P["bc_error"])
        raised = None
        rels = None
        try:
            rels = run_dfq(model, graph, bottoms, targ, bc_mode="reference", stage_hook=hook,
                           bits_weight=bits_weight, bits_bias=8)
        except RuntimeError as e:   # DeepLab: the reference's own cat-branch crash
            raised = str(e)
        torch.cuda.synchronize(device)
    finally:
        _lib.REF_THREADS = old_threads
    ref_diffs = list(P["cle_diffs"])
    out["stages"] = stage_bad
    out["cle_iterations"] = cle_info.get("iterations")
    out["cle_iterations_ref"] = len(ref_diffs)
    out["cle_diff_mismatches"] = (sum(int(a != b) for a, b in zip(cle_info.get("diffs", []), ref_diffs)) +
                                  abs(len(cle_info.get("diffs", [])) - len(ref_diffs)))
    out["bc_raised_as_reference"] = bool(bc_error) == (raised is not None)
    if rels is not None:
        out["relations_match"] = [[r.layer_first, r.layer_second, r.bn_idx] for r in rels] == P["relations"].tolist()
        Sh = [hb(r.S.cpu().numpy()) for r in rels]
        out["scale_mismatches"] = sum(int(s != bytes(P["cle_Sh"][i])) for i, s in enumerate(Sh)) \
            if len(Sh) == len(P["cle_Sh"]) else len(P["cle_Sh"])
    else:
        out["relations_match"] = None
        out["scale_mismatches"] = 0
    out["mismatches"] = (sum(v["weights"] + v["biases"] for v in stage_bad.values()) + out["cle_diff_mismatches"] +
                         out["scale_mismatches"] + int(not out["target_keys_match"]) +
                         int(not out["bc_raised_as_reference"]) + int(out["relations_match"] is False) +
                         int(out["cle_iterations"] != out["cle_iterations_ref"]) +
                         sum(1 for s in STAGES if s not in stage_bad and not (s == "bc" and bc_error)))
    return out


def _ne(a, b) -> int:
    """Elements that differ as np.array_equal sees them (-0 == +0; NaN == NaN)."""
    a, b = np.asarray(a).reshape(-1), np.asarray(b).reshape(-1)
    if a.shape != b.shape:
        return max(a.size, b.size)
    return int(((a != b) & ~(np.isnan(a) & np.isnan(b))).sum())


def sweep_mismatches(items, clip=(-15.0, 15.0)) -> dict:
    """Sweep items (already executed) vs the C oracle on the same inputs.  Counts
    differing elements of dq, codes, scale, zero and E (all bit-exact fields)."""
    from oracle import oracle as O
    bad = {"tensors": 0, "elements": 0, "dq": 0, "codes": 0, "scale": 0, "zero": 0, "esum": 0}
    for it in items:
        x = it.src.detach().cpu().numpy()
        mode = it.mode()
        rows = it.rows if it.rows is not None else (x.shape[0] if it.per_channel else 1)
        o = O.quantize(x, it.bits, mode, rows=rows, khw=it.khw, flags=O.F_CLIP if it.clip is not None else 0,
                       clip=tuple(it.clip) if it.clip is not None else (0.0, 0.0), want_esum=it.esum is not None)
        bad["tensors"] += 1
        bad["elements"] += int(x.size)
        bad["dq"] += _ne(it.dst.cpu().numpy(), o["dq"])
        if it.codes is not None:
            c = it.codes.cpu().numpy()
            if it.pack_int4:
                oc = o["codes"].reshape(-1).astype(np.uint8) & 0xF
                oc = np.append(oc, np.zeros(oc.size % 2, np.uint8))
                bad["codes"] += int((c != (oc[0::2] | (oc[1::2] << 4))).sum())
            else:
                bad["codes"] += int((c.view(o["codes"].dtype).reshape(-1) != o["codes"].reshape(-1)).sum())
        bad["scale"] += int((it.scale.cpu().numpy().view(np.uint32) != o["scale"].view(np.uint32)).sum())
        # zero: +0 in symmetric modes (compare values: -0 == +0 there by construction)
        bad["zero"] += int((it.zero.cpu().numpy() != o["zero"]).sum())
        if it.esum is not None:
            bad["esum"] += _ne(it.esum.cpu().numpy(), o["esum"])
    bad["mismatches"] = bad["dq"] + bad["codes"] + bad["scale"] + bad["zero"] + bad["esum"]
    return bad
