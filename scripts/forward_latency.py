"""Quantized-model forward latency (diagnostic, GPU): MobileNetV2 with the
reference's Quant* layers after main_dfq's stages, batch N, fp32 vs quantized
forward (activation quantizers + weight/bias fake-quant per layer)."""
import json
import sys
import time
from pathlib import Path

import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from data_free_quantization_amd import zoo  # noqa: E402
from data_free_quantization_amd.utils import layer_transform as L  # noqa: E402
from data_free_quantization_amd.utils.quantize import QuantConv2d, QuantLinear, frozen_weights, set_layer_bits  # noqa: E402,E501
from data_free_quantization_amd.utils.tracer import TorchTransformer  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dev = torch.device("cuda:0")
model = zoo.build("mobilenetv2", seed=0, relu=True).to(dev).eval()
x = torch.randn(batch, 3, 224, 224, device=dev)


def timed(fn, reps=10):
    with torch.no_grad():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


fp32_ms = timed(lambda: model(x))
tr = TorchTransformer("positional")
model, tr = L.switch_layers(model, tr, x, {1: [(nn.Conv2d, QuantConv2d), (nn.Linear, QuantLinear)]})
graph, bottoms = tr.log.getGraph(), tr.log.getBottoms()
targ = (QuantConv2d, QuantLinear)
L.merge_batchnorm(model, graph, bottoms, targ)
set_layer_bits(graph, 8, 8, 8, targ)
L.set_quant_minmax(graph, bottoms, verbose=False)
L.replace_op()
try:   # as the reference's main_dfq runs it: set_layer_bits made new observers, left in training mode
    train_obs_ms = timed(lambda: model(x))
finally:
    L.restore_op()
model.eval()
L.replace_op()
try:
    q_ms = timed(lambda: model(x))          # the default: weights re-quantized every forward
    with frozen_weights():                  # main_dfq's evaluation scope: weight fake quant kept
        qf_ms = timed(lambda: model(x))
finally:
    L.restore_op()
print(json.dumps({"batch": batch, "fp32_ms": round(fp32_ms, 3), "quant_ms": round(q_ms, 3),
                  "quant_frozen_weights_ms": round(qf_ms, 3),
                  "quant_training_mode_observers_ms": round(train_obs_ms, 3)}))

# breakdown: observers frozen (no update_stat), then without the op interception
for m in graph.values():
    if hasattr(m, "quant"):
        m.quant.update_stat = False
for q in L.module_tensor_op.quants:
    q.update_stat = False
L.replace_op()
try:
    frozen_ms = timed(lambda: model(x))
    import cProfile
    import pstats
    pr = cProfile.Profile()
    with torch.no_grad():
        pr.enable()
        for _ in range(3):
            model(x)
        torch.cuda.synchronize()
        pr.disable()
finally:
    L.restore_op()
noop_ms = timed(lambda: model(x))
print(json.dumps({"frozen_observers_ms": round(frozen_ms, 3), "no_op_interception_ms": round(noop_ms, 3)}))
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
