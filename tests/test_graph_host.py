"""Host-side graph logic (no GPU): the tracer reproduces the reference graph
structure (node / target / relation counts of SURVEY.md 8), create_relation
matches the reference's relations on the same graphs, find_prev_bn walks, and
the literal bias_correction is the reference's no-op with opaque keys."""
from collections import OrderedDict

import numpy as np
import pytest
import torch.nn as nn

from data_free_quantization_amd import zoo
from data_free_quantization_amd.utils.layer_transform import find_prev_bn
from data_free_quantization_amd.utils.relation import Relation, create_relation
from data_free_quantization_amd.utils.tracer import TorchTransformer, build_graph
from tests.helpers import pipeline

TARG = (nn.Conv2d, nn.Linear)
EXPECT = {
    "mobilenetv2": (152, 53, 3_469_760, 37),
    "resnet50": (175, 54, 25_502_912, 32),
    "deeplab": (201, 61, 5_780_288, 35),
    "resnet18": (69, 21, 11_678_912, 8),    # torchvision resnet18 (the reference's --resnet)
}


@pytest.mark.parametrize("name", list(EXPECT))
def test_graph_shape_and_relations(name):
    model = zoo.build(name, seed=0, relu=True)
    g = build_graph(model, "positional")
    graph, bottoms = g.getGraph(), g.getBottoms()
    nodes, ntarg, nelem, nrel = EXPECT[name]
    targets = [m for m in graph.values() if type(m) in TARG]
    assert len(graph) == nodes
    assert len(targets) == ntarg
    assert sum(t.weight.numel() for t in targets) == nelem
    rels = create_relation(graph, bottoms, TARG)
    assert len(rels) == nrel
    P = pipeline(name)
    assert [[r.layer_first, r.layer_second, r.bn_idx] for r in rels] == P["relations"].tolist()
    assert list(P["targets"]) == [k for k in graph if type(graph[k]) in TARG]


def test_opaque_keys_have_same_structure():
    model = zoo.build("mobilenetv2", relu=True)
    gp = build_graph(model, "positional")
    go = build_graph(model, "opaque")
    assert len(gp.getGraph()) == len(go.getGraph())
    assert all(not isinstance(k, int) for k in go.getGraph())
    assert len(create_relation(go.getGraph(), go.getBottoms(), TARG)) == 37


def test_relu6_blocks_relations():
    """Without --relu, ReLU6 is not a pass-through (utils/relation.py:53): only the
    linear-bottleneck pairs (no activation in between) remain."""
    model = zoo.build("mobilenetv2", relu=False)
    g = build_graph(model, "positional")
    graph, bottoms = g.getGraph(), g.getBottoms()
    rels = create_relation(graph, bottoms, TARG)
    assert 0 < len(rels) < 37
    for r in rels:
        k = r.layer_second
        while k != r.layer_first:
            k = bottoms[k][0]
            assert type(graph[k]) is not nn.ReLU6


def test_delete_single_keeps_chains():
    model = zoo.build("mobilenetv2", relu=True)
    g = build_graph(model, "positional")
    rels = create_relation(g.getGraph(), g.getBottoms(), TARG, delete_single=True)
    assert 0 < len(rels) <= 37
    firsts = {r.layer_first for r in rels}
    seconds = {r.layer_second for r in rels}
    assert all(r.layer_first in seconds or r.layer_second in firsts for r in rels)


def test_find_prev_bn_branch_types():
    model = zoo.build("mobilenetv2", relu=True)
    g = build_graph(model, "positional")
    graph, bottoms = g.getGraph(), g.getBottoms()
    bn_module, relu_attached = {}, {}
    for k, m in graph.items():
        if type(m) == nn.BatchNorm2d:
            bn_module[k] = m
            relu_attached[k] = False
        if type(m) == nn.ReLU and bottoms[k][0] in bn_module:
            relu_attached[bottoms[k][0]] = True
    seen = set()
    for k, m in graph.items():
        if type(m) in TARG and bottoms[k][0] != "Data":
            bl, rl, tl, tw = find_prev_bn(bn_module, relu_attached, graph, bottoms, bottoms[k][:])
            assert bl and not tw
            seen.update(tl)
    assert "one" in seen and any(t.startswith("add") for t in seen)


def test_literal_bias_correction_is_reference_noop_on_cpu():
    """Opaque keys: every layer is skipped (bias_correction.py:185-190), so the
    call touches no tensor (and needs no GPU)."""
    from data_free_quantization_amd.bias_correction import bias_correction
    model = zoo.build("mobilenetv2", relu=True)
    g = build_graph(model, "opaque")
    graph, bottoms = g.getGraph(), g.getBottoms()
    before = [m.weight.detach().clone() for m in graph.values() if type(m) in TARG]
    b, a = bias_correction(graph, bottoms, TARG, bits_weight=8)
    assert b == {} and a == {}
    after = [m.weight.detach() for m in graph.values() if type(m) in TARG]
    assert all(np.array_equal(x.numpy(), y.numpy()) for x, y in zip(before, after))


def test_transformer_swaps_layers():
    from data_free_quantization_amd.utils.quantize import QuantConv2d, QuantLinear
    model = zoo.build("mobilenetv2")
    w0 = model.features[0][0].weight.detach().clone()
    t = TorchTransformer()
    t.register(nn.Conv2d, QuantConv2d)
    t.register(nn.Linear, QuantLinear)
    model = t.trans_layers(model, update=True)
    t.register(nn.ReLU6, nn.ReLU)
    model = t.trans_layers(model, update=False)
    t._build_graph(model)
    graph = t.log.getGraph()
    types = {type(m) for m in graph.values()}
    assert QuantConv2d in types and QuantLinear in types and nn.ReLU in types and nn.ReLU6 not in types
    assert nn.Conv2d not in types
    assert len(graph) == 152
    assert np.array_equal(model.features[0][0].weight.detach().numpy(), w0.numpy())
    assert len(create_relation(graph, t.log.getBottoms(), (QuantConv2d, QuantLinear))) == 37


def test_reference_checkpoint_keys_load(tmp_path):
    """A checkpoint with the reference's module names loads into the zoo models:
    MobileNetV2 keys are identical; the reference DeepLab's aliased backbone keys
    (low_level_features / high_level_features) map back to backbone.features."""
    import torch
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.main_dfq import canonical_state_dict
    m = zoo.build("deeplab", seed=1)
    sd = dict(m.state_dict())
    ref_style = dict(sd)
    for k, v in sd.items():   # what the reference's DeepLab state_dict looks like
        if k.startswith("backbone.features."):   # Sequential slices keep the child names
            i = int(k[len("backbone.features."):].split(".", 1)[0])
            pre = "backbone.low_level_features." if i < 4 else "backbone.high_level_features."
            ref_style[pre + k[len("backbone.features."):]] = v.clone()
    m2 = zoo.build("deeplab", seed=2)
    m2.load_state_dict(canonical_state_dict(ref_style))
    for k, v in m2.state_dict().items():
        assert torch.equal(v, sd[k])
    bad = dict(ref_style)
    first_alias = next(k for k in bad if k.startswith("backbone.low_level_features."))
    bad[first_alias] = bad[first_alias] + 1
    with pytest.raises(ValueError):
        canonical_state_dict(bad)


def test_zoo_matches_reference_checkpoint_format():
    """tests/golden/state_dict_keys.json (the reference models' state_dict names and
    shapes): MobileNetV2 identical, DeepLab identical after canonical_state_dict,
    ResNet-50 = the reference backbone + the fc head."""
    import json
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.main_dfq import canonical_state_dict
    from tests.helpers import GOLDEN
    ref = json.loads((GOLDEN / "state_dict_keys.json").read_text())
    shapes = lambda m: {k: list(v.shape) for k, v in m.state_dict().items()}   # noqa: E731
    assert shapes(zoo.build("mobilenetv2", seed=0)) == {k: s for k, s in ref["mobilenetv2"]}
    fake = {k: __import__("torch").zeros(s) for k, s in ref["deeplab"]}
    assert {k: list(v.shape) for k, v in canonical_state_dict(fake).items()} == shapes(zoo.build("deeplab", seed=0))
    r50 = shapes(zoo.build("resnet50", seed=0))
    assert {k: s for k, s in r50.items() if not k.startswith("fc.")} == {k: s for k, s in ref["resnet50_backbone"]}


def test_export_dequantize_u16_codes(tmp_path):
    """Asymmetric codes above 8 bits are uint16 patterns held in int16:
    dequantize must not sign-extend them."""
    import torch
    from data_free_quantization_amd import export
    codes = torch.tensor([[0, 1, 32767, -32768, -1]], dtype=torch.int16)    # 0, 1, 32767, 32768, 65535
    meta = {"bits": 16, "symmetric": False, "packed_int4": False, "clip": None,
            "layers": {"k": {"shape": [1, 5]}}}
    s, z = torch.tensor([0.5]), torch.tensor([-1.0])
    y = export.dequantize(meta, "k", {"codes": codes, "scale": s, "zero": z})
    want = torch.tensor([[0, 1, 32767, 32768, 65535]], dtype=torch.float32) * 0.5 - 1.0
    assert torch.equal(y, want)
    meta["symmetric"] = True       # symmetric int16 stays signed
    y = export.dequantize(meta, "k", {"codes": codes, "scale": s, "zero": torch.tensor([0.0])})
    assert torch.equal(y, codes.float() * 0.5)


def test_bc_chain_scratch_slot_growth_on_cpu():
    """The walk's torch.cat of expectations (DeepLab's concat branches) grows the
    last scratch slot: in place while its chunk has room, else into a fresh slot
    filled by a COPY op; a recorded walk keeps each chunk's fill for its replay
    (symbolic refs are 4-tuples: tensor, float offset, address, symbol)."""
    import torch
    from data_free_quantization_amd import _lib
    from data_free_quantization_amd import bias_correction as bc
    ch = bc._BcChain(torch.device("cpu"), record=True)
    ref = ch.alloc(100)
    assert len(ref) == 4 and ref[3] == (bc._S_SCRATCH, 0, 0)
    assert ch.extend_last(ref, 100, 50) is ref and ch.chunk_fill == [192]
    big = ch.alloc(bc._SCRATCH_CHUNK - 256)
    new = ch.extend_last(big, bc._SCRATCH_CHUNK - 256, 128)
    assert new[0] is not big[0] and new[3] == (bc._S_SCRATCH, 1, 0)
    kind, _, src, _, dst, _, n = ch.ops[-1][:7]
    assert kind == _lib.DFQ_BC_OP_COPY and (src, dst, n) == (big[2], new[2], bc._SCRATCH_CHUNK - 256)
    assert ch.sym[-1][1][0] == big[3] and ch.sym[-1][1][2] == new[3]
    assert ch.chunk_fill == [bc._SCRATCH_CHUNK - 64, bc._SCRATCH_CHUNK - 128]
