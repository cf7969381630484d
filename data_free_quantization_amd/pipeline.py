"""The DFQ weight-transform pipeline in main_dfq's stage order
(main_dfq.py:188-231), on the GPU:

  merge_batchnorm -> create_relation -> cross_layer_equalization ->
  bias_absorption -> set_layer_bits -> merge_batchnorm -> quantize_targ_layer ->
  clip_weight -> bias_correction

``bc_mode``:
  * "literal"   -- exactly the reference: BC walks with the graph's keys (a no-op
                   with opaque keys)
  * "reference" -- the reference's coded arithmetic (requires positional keys)
  * "fused"     -- extension: E comes from the quantize sweep itself (the error
                   of the quantization actually applied), clip fused in the sweep
"""
from __future__ import annotations

import time
from typing import Callable, Dict, Optional

import torch
import torch.nn as nn

from . import Cross_layer_equal as cle
from .bias_absorption import bias_absorption
from .bias_correction import bias_correction
from .clip_weight import clip_weight
from .utils.layer_transform import esum_source, merge_batchnorm, quantize_targ_layer
from .utils.quantize import set_layer_bits
from .utils.relation import create_relation


def run_dfq(model: nn.Module, graph, bottoms, targ, *, relu: bool = True, equalize: bool = True,
            absorption: bool = True, quantize: bool = True, clip: bool = True, correction: bool = True,
            bits_weight: int = 8, bits_activation: int = 8, bits_bias: int = 8, granularity: str = "tensor",
            symmetric: bool = False, bc_mode: str = "literal", clip_range=(-15, 15),
            stage_hook: Optional[Callable[[str], None]] = None, timings: Optional[Dict] = None):
    """Run the DFQ stages on ``model`` (already on the GPU) in place; returns the
    equalization relations."""
    assert relu or relu == equalize, "must replace relu6 to relu while equalization"
    assert equalize or absorption == equalize, "must use absorption with equalize"
    t = timings if timings is not None else {}
    timed = timings is not None   # per-stage times need a device sync around each stage

    def stage(name, fn, *a, **k):
        if timed:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn(*a, **k)
        if timed:
            torch.cuda.synchronize()
            t[name] = time.perf_counter() - t0
        if stage_hook:
            stage_hook(name)
        return out

    stage("bn1", merge_batchnorm, model, graph, bottoms, targ)
    res = []
    if equalize:
        res = stage("relations", create_relation, graph, bottoms, targ, delete_single=False)
        # launched: the next stages' host work overlaps the device loop (their kernels
        # are ordered behind it on the current stream); wait() below joins it
        stage("cle", cle.cross_layer_equalization, graph, res, targ, Save_state=False, Treshhold=2e-7, launch=True)
    if absorption:
        stage("absorb", bias_absorption, graph, res, bottoms, N=3)
    state = {} if (correction and bc_mode == "fused") else None
    if quantize:
        set_layer_bits(graph, bits_weight, bits_activation, bits_bias, targ)
        # the second fold hands the folded weights' ranges to the quantize sweep
        fold_ranges = {} if granularity == "tensor" else None
        stage("bn2", merge_batchnorm, model, graph, bottoms, targ, ranges=fold_ranges)
        fused_clip = tuple(clip_range) if (clip and bc_mode == "fused") else None
        stage("quant", quantize_targ_layer, graph, bits_weight, bits_bias, targ, granularity=granularity,
              symmetric=symmetric, clip=fused_clip, state=state, weight_ranges=fold_ranges)
    if clip and not (quantize and bc_mode == "fused"):
        stage("clip", clip_weight, graph, range_clip=list(clip_range), targ_type=targ)
    if correction:
        err = None
        if bc_mode == "fused":
            err = {k: esum_source(v) for k, v in (state or {}).items()}
        stage("bc", bias_correction, graph, bottoms, targ, bits_weight=bits_weight, signed=symmetric,
              error_sums=err)
    cle.wait()   # a launched CLE loop's error surfaces here (its results are already ordered on the stream)
    return res
