"""TEST INFRASTRUCTURE ONLY: the reference's CPU weight arithmetic restated with the
same torch CPU eager ops, for bench.py's ``cpu_baseline`` leg (kind "port") and
the CPU tests.  Never imported by the product package.

The reference runs its DFQ weight path on the CPU in eager PyTorch
(main_dfq.py:145); this file performs the identical op sequence so the baseline
measures what the reference's code costs on the GPU box's host cores, where the
reference itself is not available:
  * ``quantize``            -- UniformQuantize.forward (utils/quantize.py:25-78):
    clone, add_(-min), div_(scale), clamp_(qmin, qmax), round_(), mul_(scale),
    add_(min), with the scale computed in Python floats (float64) and
    ``max(scale, 1e-8)``;
  * ``per_channel_sweep``   -- the per-channel composition the SURVEY (8a row a3)
    defines: the reference ``quantize`` on every W[o] slice with
    float(W[o].min()) / float(W[o].max()), then clip_weight's clamp_
    (clip_weight.py:29) and the bias-correction error sums
    (bias_correction.py:128-131,231: (Q(W) - W).view(O, I, -1).sum(-1));
  * ``per_tensor_sweep``    -- quantize_targ_layer's arithmetic
    (utils/layer_transform.py:296-299): one range per weight tensor.
"""
from __future__ import annotations

import torch


def quantize(x: torch.Tensor, num_bits=8, min_value=None, max_value=None, symmetric=False) -> torch.Tensor:
    """utils/quantize.py:25-78 with given (Python float) min/max."""
    output = x.clone()
    if symmetric:
        qmin = -2.0 ** (num_bits - 1)
        qmax = 2 ** (num_bits - 1) - 1
        max_value = abs(max_value)
        min_value = abs(min_value)
        if max_value < min_value:
            max_value = min_value
        scale = max_value / qmax
        min_value = 0.0
    else:
        qmin = 0.0
        qmax = 2.0 ** num_bits - 1.0
        scale = (max_value - min_value) / (qmax - qmin)
    scale = max(scale, 1e-8)
    output.add_(-min_value).div_(scale)
    output.clamp_(qmin, qmax).round_()
    output.mul_(scale).add_(min_value)
    return output


def per_channel_sweep(w: torch.Tensor, bits=8, symmetric=True, clip=(-15.0, 15.0), want_esum=True):
    """Per-channel quantize-dequantize of one weight (reference quantize per W[o]),
    clamp, and E[o, i] = sum_k (Q(W) - W)[o, i, k].  Returns (dq, E)."""
    rows = [quantize(w[o], bits, float(w[o].min()), float(w[o].max()), symmetric) for o in range(w.shape[0])]
    dq = torch.stack(rows)
    if clip is not None:
        dq.clamp_(clip[0], clip[1])
    e = None
    if want_esum:
        e = (dq - w).view(w.shape[0], w.shape[1] if w.dim() > 1 else 1, -1).sum(-1)
    return dq, e


def per_tensor_sweep(w: torch.Tensor, bits=8, symmetric=False):
    """quantize_targ_layer's weight arithmetic (utils/layer_transform.py:296-299)."""
    return quantize(w, bits, float(w.min()), float(w.max()), symmetric)
