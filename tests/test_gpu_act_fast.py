"""Inference fast paths of the activation/weight fake quant (dfq_range +
dfq_fake_quant_given: async, no host round trip) against the generic quantize()
path that mirrors utils/quantize.py line by line.  Bit-exact."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("bits", [8, 4, 16])
@pytest.mark.parametrize("shape", [(32, 96, 28, 28), (7, 13), (5, 3, 3)])
def test_given_range_matches_quantize(bits, shape):
    from data_free_quantization_amd.utils.quantize import device_range, fake_quant_given, quantize
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(shape, device=DEV, generator=g) * 3
    mn, mx = torch.tensor([-2.5], device=DEV), torch.tensor([4.1], device=DEV)
    ref = quantize(x, bits, float(mn), float(mx))
    assert torch.equal(fake_quant_given(x, bits, min_dev=mn, max_dev=mx), ref)
    assert torch.equal(fake_quant_given(x, bits, min_value=float(mn), max_value=float(mx)), ref)
    for sym in (False, True):
        ref = quantize(x, bits, float(x.min()), float(x.max()), symmetric=sym)      # Python-float bounds
        assert torch.equal(fake_quant_given(x, bits, sym, range_enc=device_range(x)), ref)
        ref = quantize(x, bits, symmetric=sym)                                       # 0-d fp32 bounds
        assert torch.equal(fake_quant_given(x, bits, sym, range_enc=device_range(x), scale_f32=True), ref)


def test_quant_measure_and_layers_inference_equals_autograd_path():
    from data_free_quantization_amd.utils.quantize import QuantConv2d, QuantLinear, QuantMeasure
    torch.manual_seed(0)
    conv = QuantConv2d(16, 32, 3, padding=1, num_bits=8, num_bits_bias=8).to(DEV).eval()
    lin = QuantLinear(32, 10, num_bits=4, num_bits_bias=8).to(DEV).eval()
    for q in (conv.quant, lin.quant):
        q.running_min.fill_(-1.5)
        q.running_max.fill_(2.25)
    x = torch.randn(4, 16, 12, 12, device=DEV)
    with torch.no_grad():
        fast = lin(conv(x).mean((2, 3)))
    xg = x.clone().requires_grad_(True)
    slow = lin(conv(xg).mean((2, 3)))                 # STE path: the generic quantize()
    assert torch.equal(fast, slow.detach())
    # update_stat (the reference's set_layer_bits quirk: a truthy bit count)
    qm = QuantMeasure(update_stat=8).to(DEV).eval()
    a = torch.randn(8, 50, device=DEV) * 2
    with torch.no_grad():
        y = qm(a)
    flat = a.view(8, -1).cpu()   # the statistics follow ATen's CPU order (dfq_act_observe)
    assert float(qm.running_max) == max(0.0, float(flat.max(-1)[0].mean()))
    assert float(qm.running_min) == min(0.0, float(flat.min(-1)[0].mean()))
    from data_free_quantization_amd.utils.quantize import quantize
    assert torch.equal(y, quantize(a, 8, float(qm.running_min), float(qm.running_max)))
    # training mode (how the reference's main_dfq runs its fresh observers at inference):
    # batch statistics + momentum update, quantized with the batch range
    qt = QuantMeasure(num_bits=8).to(DEV)
    with torch.no_grad():
        yt = qt(a)
    mn, mx = flat.min(-1)[0].mean(), flat.max(-1)[0].mean()
    assert torch.equal(yt, quantize(a, 8, float(mn), float(mx)))
    assert float(qt.running_max) == float(torch.zeros(1).mul_(0.9).add_(mx * 0.1))


def test_quantized_mobilenetv2_forward_fast_equals_generic():
    """Whole quantized MobileNetV2 (main_dfq's stages, activation quantizers on every
    target layer and tensor op): the no-grad forward equals the autograd-path forward."""
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.utils import layer_transform as L
    from data_free_quantization_amd.utils.quantize import QuantConv2d, QuantLinear, set_layer_bits
    from data_free_quantization_amd.utils.tracer import TorchTransformer
    model = zoo.build("mobilenetv2", seed=0, relu=True).to(DEV).eval()
    x = torch.randn(2, 3, 224, 224, device=DEV)
    tr = TorchTransformer("positional")
    model, tr = L.switch_layers(model, tr, x, {1: [(nn.Conv2d, QuantConv2d), (nn.Linear, QuantLinear)]})
    graph, bottoms = tr.log.getGraph(), tr.log.getBottoms()
    targ = (QuantConv2d, QuantLinear)
    try:
        L.merge_batchnorm(model, graph, bottoms, targ)
        set_layer_bits(graph, 8, 8, 8, targ)
        L.set_quant_minmax(graph, bottoms, verbose=False)
        model.eval()   # inference_all's model.eval(): set_layer_bits made new (training-mode) observers
        for m in graph.values():   # fixed observers, so both forwards see the same ranges
            if hasattr(m, "quant"):
                m.quant.update_stat = False
        for q in L.module_tensor_op.quants:
            q.update_stat = False
        L.replace_op()
        try:
            with torch.no_grad():
                fast = model(x)
            slow = model(x.clone().requires_grad_(True)).detach()
        finally:
            L.restore_op()
        assert torch.equal(fast, slow)
        assert torch.isfinite(fast).all()
    finally:
        L.module_tensor_op = None
