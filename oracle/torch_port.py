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


def layer_equalization(W1, W2, B1, bn_w=None, bn_b=None, s_min_max=(1e-8, 1e8), signed=False, eps=0):
    """Cross_layer_equal.py:11-59 with the same torch CPU ops: the per-channel
    Python loop over W2's input channels (the reference's 62-75 s on MobileNetV2)."""
    groups = 1
    if W1.shape[0] != W2.shape[1]:
        groups = W1.shape[0] // W2.shape[1]
    c_in = W1.shape[0] // groups
    c_out = W2.shape[0] // groups
    S = torch.zeros(W1.size(0))
    for g in range(groups):
        a0, a1 = g * c_in, (g + 1) * c_in
        o0, o1 = g * c_out, (g + 1) * c_out
        W1g, W2g = W1[a0:a1], W2[o0:o1]
        for i in range(W2g.shape[1]):
            if signed:
                r1 = torch.max(torch.abs(W1g[i]))
                r2 = torch.max(torch.abs(W2g[:, i]))
            else:
                r1 = torch.max(W1g[i]) - torch.min(W1g[i])
                r2 = torch.max(W2g[:, i]) - torch.min(W2g[:, i])
            s = (1 / (r1 + eps)) * torch.sqrt(r1 * r2 + eps)
            s = max(s_min_max[0], min(s_min_max[1], s))
            S[a0 + i] = s
            W1[a0 + i].mul_(s)
            if B1 is not None:
                B1[a0 + i].mul_(s)
            if bn_w is not None:
                bn_w[a0 + i].mul_(s)
            if bn_b is not None:
                bn_b[a0 + i].mul_(s)
            W2[o0:o1, i].mul_(1 / s)
    return W1, W2, B1, S


def cle_iteration(weights, biases, bn, relations):
    """One pass of cross_layer_equalization's while-loop body
    (Cross_layer_equal.py:81-115): snapshot every target weight (the deepcopy's
    cost on the weights), equalize every relation in order, then the metric
    np.sum([float(mean(|W - W_old|))]).  ``weights``/``biases``: name -> CPU
    tensor (updated in place); ``bn``: name -> (fake_weight, fake_bias);
    ``relations``: [(first, second, bn_name)].  Returns the iteration's diff."""
    import numpy as np
    old = {k: w.clone() for k, w in weights.items()}
    for a, b, n in relations:
        if biases.get(a) is None:
            biases[a] = torch.zeros(weights[a].size(0), dtype=torch.float32)
        fw, fb = bn[n]
        layer_equalization(weights[a], weights[b], biases[a], fw, fb)
    return float(np.sum([float(torch.mean(torch.abs(weights[k] - old[k]))) for k in weights]))


def quantize_error_spatial(w: torch.Tensor, num_bits=8, signed=False) -> torch.Tensor:
    """bias_correction.py:111-144 (_quantize_error: per-tensor quantize of a
    clone, minus the weight) followed by the spatial sum bias correction takes of
    it (bias_correction.py:231): E[o, i] = sum_k (Q(W) - W)[o, i, k]."""
    p = w.detach().clone()
    q = quantize(p, num_bits, float(p.min()), float(p.max()), signed)
    err = q - p
    return err.view(err.size(0), err.size(1) if err.dim() > 1 else 1, -1).sum(-1)
