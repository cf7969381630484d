"""set_quant_minmax (utils/layer_transform.py:356-618) on the GPU vs the
reference's own output (tests/golden/act_ranges_*.npz, made by
tests/golden/make_golden.py act): QuantMeasure ranges of every target layer and
every add / cat / mean / interpolate input, after the first BN fold (random BN
statistics: ReLU/ReLU6 Gaussian moments, add merges, cat min/max) and after the
second (main_dfq's order).  Bit-exact; quantizers set through case (d.) (a
conv/linear between BN and quantizer: an MKL GEMV in the reference) within 1e-5.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from tests.helpers import GOLDEN

pytestmark = pytest.mark.gpu
TARG = (nn.Conv2d, nn.Linear)


@pytest.mark.parametrize("name", ["mobilenetv2", "resnet50", "deeplab"])
def test_set_quant_minmax_matches_reference(name):
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.utils import layer_transform as L
    from data_free_quantization_amd.utils.quantize import QuantMeasure
    from data_free_quantization_amd.utils.tracer import build_graph
    A = np.load(GOLDEN / f"act_ranges_{name}.npz")
    model = zoo.build(name, seed=0, relu=True).cuda()
    g = build_graph(model, "positional")
    graph, bottoms = g.getGraph(), g.getBottoms()
    tkeys = [k for k in graph if type(graph[k]) in TARG]
    assert tkeys == list(A["targets"])
    for k in tkeys:
        graph[k].quant = QuantMeasure(num_bits=8).cuda()
    L.module_tensor_op = L.CustomTensorOP(graph, bottoms).cuda()
    assert L.module_tensor_op.names == list(A["op_keys"])
    mods = [graph[k].quant for k in tkeys] + list(L.module_tensor_op.quants)
    try:
        for tag in ("bn1", "bn2"):
            L.merge_batchnorm(model, graph, bottoms, TARG)
            assert str(A[f"{tag}_error"]) == ""
            L.set_quant_minmax(graph, bottoms, verbose=False)
            got_min = np.array([float(q.running_min) for q in mods], dtype=np.float32)
            got_max = np.array([float(q.running_max) for q in mods], dtype=np.float32)
            d = np.array([any(q is c for c in L.CASE_D) for q in mods])
            assert np.array_equal(got_min[~d], A[f"{tag}_min"][~d]), (tag, np.nonzero(got_min != A[f"{tag}_min"]))
            assert np.array_equal(got_max[~d], A[f"{tag}_max"][~d]), (tag, np.nonzero(got_max != A[f"{tag}_max"]))
            np.testing.assert_allclose(got_min[d], A[f"{tag}_min"][d], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(got_max[d], A[f"{tag}_max"][d], rtol=1e-5, atol=1e-6)
    finally:
        L.module_tensor_op = None


def test_replace_op_quantizes_tensor_op_inputs():
    """replace_op routes every add / mean call of a MobileNetV2 forward through the
    quantizers of the graph node it executes: the quantized model's output equals
    a forward where the same QuantMeasures are applied explicitly."""
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.utils import layer_transform as L
    from data_free_quantization_amd.utils.quantize import QuantConv2d, QuantLinear
    from data_free_quantization_amd.utils.tracer import TorchTransformer
    torch.manual_seed(0)
    model = zoo.build("mobilenetv2", seed=0, relu=True).cuda().eval()
    tr = TorchTransformer("positional")
    x = torch.randn(2, 3, 224, 224, device="cuda")
    model, tr = L.switch_layers(model, tr, x, {1: [(nn.Conv2d, QuantConv2d), (nn.Linear, QuantLinear)]})
    graph, bottoms = tr.log.getGraph(), tr.log.getBottoms()
    try:
        L.merge_batchnorm(model, graph, bottoms, (QuantConv2d, QuantLinear))
        L.set_quant_minmax(graph, bottoms, verbose=False)
        calls = []
        for q in L.module_tensor_op.quants:
            q.register_forward_hook(lambda m, i, o: calls.append(m))
        with torch.no_grad():
            y0 = model(x)
            assert calls == []                       # no interception without replace_op
            L.replace_op()
            try:
                y1 = model(x)
            finally:
                L.restore_op()
        assert len(calls) == len(L.module_tensor_op.quants)   # every op input quantized once, in order
        assert [id(c) for c in calls] == [id(q) for q in L.module_tensor_op.quants]
        assert L.module_tensor_op.idx_name_tensor_op == 0      # cycled back for the next forward
        assert not torch.equal(y0, y1)
        assert torch.isfinite(y1).all()
    finally:
        L.module_tensor_op = None


def test_set_quant_minmax_error_keeps_earlier_fills(monkeypatch):
    """An error raised inside the walk (the reference's asserts) leaves the
    quantizers set before it with their ranges and the later ones untouched,
    as the reference's sequential fill_ calls do -- also with the recorded /
    replayed walk that batches the readbacks."""
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.utils import layer_transform as L
    from data_free_quantization_amd.utils.quantize import QuantMeasure
    from data_free_quantization_amd.utils.tracer import build_graph
    model = zoo.build("mobilenetv2", seed=0, relu=True).cuda()
    g = build_graph(model, "positional")
    graph, bottoms = g.getGraph(), g.getBottoms()
    tkeys = [k for k in graph if type(graph[k]) in TARG]
    for k in tkeys:
        graph[k].quant = QuantMeasure(num_bits=8).cuda()
    L.merge_batchnorm(model, graph, bottoms, TARG)
    ref = [(float(graph[k].quant.running_min), float(graph[k].quant.running_max)) for k in tkeys]
    L.set_quant_minmax(graph, bottoms, verbose=False)
    full = [(float(graph[k].quant.running_min), float(graph[k].quant.running_max)) for k in tkeys]
    for k in tkeys:   # back to the unset state
        graph[k].quant.running_min.zero_()
        graph[k].quant.running_max.zero_()
    real, stop = L.find_prev_bn, list(bottoms[tkeys[20]])

    def failing(bn_module, relu_attached, graph_, bottoms_, bot):
        if list(bot) == stop:   # the same point of the walk in every pass
            raise AssertionError("walk error")
        return real(bn_module, relu_attached, graph_, bottoms_, bot)

    monkeypatch.setattr(L, "find_prev_bn", failing)
    with pytest.raises(AssertionError, match="walk error"):
        L.set_quant_minmax(graph, bottoms, verbose=False)
    got = [(float(graph[k].quant.running_min), float(graph[k].quant.running_max)) for k in tkeys]
    set_before = [g_ == f for g_, f in zip(got, full)]
    untouched = [g_ == (0.0, 0.0) for g_ in got]
    assert all(s or u for s, u in zip(set_before, untouched))
    n_set = sum(1 for g_, r in zip(got, ref) if g_ != (0.0, 0.0))
    assert 0 < n_set < len(tkeys)
