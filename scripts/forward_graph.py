"""Quantized MobileNetV2 forward (batch N) eager vs captured in one HIP graph
(diagnostic, GPU): the reference's Quant* layers after main_dfq's stages, weight
fake quant inside frozen_weights(), observers frozen (update_stat off) so every
forward returns the same bytes; eager and graph outputs compared bit for bit."""
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


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t2 - t0) / reps * 1e3, (t1 - t0) / reps * 1e3   # wall per forward, host enqueue per forward


res = {"batch": batch}
with torch.no_grad():
    res["fp32_ms"], res["fp32_host_ms"] = timed(lambda: model(x))
    tr = TorchTransformer("positional")
    model, tr = L.switch_layers(model, tr, x, {1: [(nn.Conv2d, QuantConv2d), (nn.Linear, QuantLinear)]})
    graph, bottoms = tr.log.getGraph(), tr.log.getBottoms()
    targ = (QuantConv2d, QuantLinear)
    L.merge_batchnorm(model, graph, bottoms, targ)
    set_layer_bits(graph, 8, 8, 8, targ)
    L.set_quant_minmax(graph, bottoms, verbose=False)
    model.eval()
    for m in graph.values():
        if hasattr(m, "quant"):
            m.quant.update_stat = False
    L.replace_op()
    for q in L.module_tensor_op.quants:
        q.update_stat = False
    try:
        with frozen_weights():
            res["quant_ms"], res["quant_host_ms"] = timed(lambda: model(x))
            ref = model(x).clone()
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            sx = x.clone()
            with torch.cuda.stream(s):
                for _ in range(3):
                    model(sx)
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                sy = model(sx)
            g.replay()
            torch.cuda.synchronize()
            res["graph_equal_eager"] = bool(torch.equal(sy, ref))
            res["graph_max_abs_diff"] = float((sy - ref).abs().max())
            res["graph_ms"], _ = timed(g.replay)
    finally:
        L.restore_op()
print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
