"""The reference CLI driver (main_dfq.py:36-267) on the MI355X DFQ path.

Same flags and stage order; the transforms run on the GPU.  Additive flags:
  --model {mobilenetv2,resnet50,deeplab,resnet18}   (default: from --task/--resnet:
                       --resnet = ResNet-18 as in the reference, torchvision layout)
  --weights PATH       state_dict to load (torch.load(weights_only=True)); synthetic
                       random-init weights otherwise (the reference checkpoints are
                       not shipped, .MISSING_LARGE_BLOBS)
  --granularity {tensor,channel}, --symmetric   weight quantizer (reference: tensor, asym)
  --bc_mode {literal,reference,fused}          see pipeline.py (default literal = the
                       reference's effective behaviour)
  --val PATH           ImageNet-val folder (ImageFolder layout) for --task cls evaluation
  --voc PATH           VOCdevkit/VOC2012 for --task seg evaluation (mIoU)
  --batch_size, --workers   evaluation DataLoader (reference: 256 / 4 cls, 32 / 2 seg)
  --world_size N       shard quantize_targ_layer's layer list over N ranks (one
                       process per GPU under torchrun, RCCL all-gather of the
                       results; distributed.py); rank 0 evaluates / logs / exports

Example (README.md:137 of the reference):
  python -m data_free_quantization_amd.main_dfq --task cls --relu --equalize --absorption \
      --quantize --correction --clip_weight --bits_weight 8 --bits_activation 8 --bits_bias 8
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.nn as nn

from . import _lib, zoo
from .bias_absorption import bias_absorption
from .bias_correction import bias_correction
from .clip_weight import clip_weight
from .Cross_layer_equal import cross_layer_equalization, wait as cle_wait
from .utils.layer_transform import (esum_source, merge_batchnorm, quantize_targ_layer, replace_op, restore_op,
                                    set_quant_minmax, switch_layers)
from .utils.quantize import QuantConv2d, QuantLinear, QuantMeasure, set_layer_bits
from .utils.relation import create_relation
from .utils.tracer import TorchTransformer


def get_argument(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpu", action="store_true")
    p.add_argument("--sizedisp", action="store_true")
    p.add_argument("--visualize", action="store_true")
    p.add_argument("--quantize", action="store_true")
    p.add_argument("--equalize", action="store_true")
    p.add_argument("--correction", action="store_true")
    p.add_argument("--absorption", action="store_true")
    p.add_argument("--relu", action="store_true")
    p.add_argument("--clip_weight", action="store_true")
    p.add_argument("--task", default="cls", type=str, choices=["cls", "seg"])
    p.add_argument("--resnet", action="store_true")
    p.add_argument("--log", action="store_true")
    p.add_argument("--bits_weight", type=int, default=8)
    p.add_argument("--bits_activation", type=int, default=8)
    p.add_argument("--bits_bias", type=int, default=8)
    # additive
    p.add_argument("--model", default=None, choices=list(zoo.MODELS))
    p.add_argument("--weights", default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--granularity", default="tensor", choices=["tensor", "channel"])
    p.add_argument("--symmetric", action="store_true")
    p.add_argument("--bc_mode", default="literal", choices=["literal", "reference", "fused"])
    p.add_argument("--val", default="./val")
    p.add_argument("--voc", default="./VOCdevkit/VOC2012/")
    p.add_argument("--batch_size", type=int, default=256)
    p.add_argument("--workers", type=int, default=4)
    p.add_argument("--device", default="cuda:0")
    p.add_argument("--export", default=None,
                   help="write the integer weights (codes, scale, zero, bias) to this safetensors file")
    p.add_argument("--world_size", type=int, default=1,
                   help="ranks sharing quantize_targ_layer's layer list (launch with torchrun --nproc-per-node N)")
    return p.parse_args(argv)


def _model_name(args):
    if args.model:
        return args.model
    if args.task == "seg":
        return "deeplab"
    return "resnet18" if args.resnet else "mobilenetv2"   # main_dfq.py:126-131


def canonical_state_dict(state):
    """A reference checkpoint's state_dict in this package's module names.  The
    reference's DeepLab backbone exposes features[0:4] / features[4:] a second
    time as low_level_features / high_level_features
    (modeling/segmentation/backbone/mobilenet.py:115-116), so its checkpoints hold
    every backbone tensor twice; a slice of an nn.Sequential keeps the original
    child names, so ``low_level_features.N`` / ``high_level_features.N`` map back
    to ``backbone.features.N`` (and must agree with it)."""
    out = {}
    alias = ("backbone.low_level_features.", "backbone.high_level_features.")
    for k, v in state.items():
        for pre in alias:
            if k.startswith(pre):
                canon = "backbone.features." + k[len(pre):]
                if canon in state and not torch.equal(state[canon], v):
                    raise ValueError(f"checkpoint alias {k} disagrees with {canon}")
                out.setdefault(canon, v)
                break
        else:
            out[k] = v
    return out


def build_model(args):
    name = _model_name(args)
    model = zoo.build(name, seed=args.seed)
    if args.weights:
        state = torch.load(args.weights, map_location="cpu", weights_only=True)
        state = state.get("state_dict", state) if isinstance(state, dict) else state
        model.load_state_dict(canonical_state_dict(state))
    return model, name


def inference_all(model, task, args):
    """main_dfq.py:66-113 on the GPU: ImageNet-val top-1 (``--val``, ImageFolder
    layout) for cls, PASCAL VOC 2012 val mIoU (``--voc``) for seg, through the
    torchvision-free harness in evaluate.py.  Returns None (with a message) when
    the dataset is not there -- neither ships with the reference or this image."""
    from . import evaluate
    if task == "cls":
        if not os.path.isdir(args.val):
            print(f"Evaluation skipped: no ImageFolder at {args.val}")
            return None
        print("Start inference")
        acc = evaluate.inference_cls(model, args.val, args.device, batch_size=args.batch_size,
                                     workers=args.workers)
        print(f"Final Accuracy: {acc * 100:.2f}%")
        return acc
    if not os.path.isdir(args.voc):
        print(f"Evaluation skipped: no VOC 2012 tree at {args.voc}")
        return None
    print("Start inference")
    miou = evaluate.inference_seg(model, args.voc, args.device, batch_size=min(args.batch_size, 32),
                                  workers=args.workers)
    print(f"mIoU: {miou * 100:.2f}%")
    return miou


def main(argv=None):
    args = get_argument(argv)
    assert args.relu or args.relu == args.equalize, "must replace relu6 to relu while equalization"
    assert args.equalize or args.absorption == args.equalize, "must use absorption with equalize"
    rank = 0
    if args.world_size > 1:
        from . import distributed as D
        world, rank, dev = D.init_from_env()
        if world != args.world_size:
            raise ValueError(f"--world_size {args.world_size} but WORLD_SIZE={world} (launch with torchrun "
                             f"--nproc-per-node {args.world_size})")
        args.device = str(dev)
    model, name = build_model(args)
    if args.sizedisp:
        print("param size:", sum(p.numel() for p in model.parameters()) * 4 / 2 ** 20, "MB")
    model = model.to(args.device).eval()

    transformer = TorchTransformer(key_mode="positional" if args.bc_mode != "literal" else "opaque")
    module_dict = {}
    if args.quantize:
        module_dict[1] = [(nn.Conv2d, QuantConv2d), (nn.Linear, QuantLinear)]
    if args.relu:
        module_dict[0] = [(torch.nn.ReLU6, torch.nn.ReLU)]
    data = torch.ones(zoo.INPUT_SHAPES[name])
    model, transformer = switch_layers(model, transformer, data, module_dict, ignore_layer=[QuantMeasure],
                                       quant_op=args.quantize)
    model = model.to(args.device)
    graph = transformer.log.getGraph()
    bottoms = transformer.log.getBottoms()
    targ_layer = (QuantConv2d, QuantLinear) if args.quantize else (nn.Conv2d, nn.Linear)
    if str(args.device).startswith("cuda"):
        _lib.preload()   # library + code objects: process setup, outside the timed stages

    t0 = time.perf_counter()
    model = merge_batchnorm(model, graph, bottoms, targ_layer)
    res = []
    if args.equalize:
        res = create_relation(graph, bottoms, targ_layer, delete_single=False)
        cross_layer_equalization(graph, res, targ_layer, Save_state=False, Treshhold=2e-7, launch=True)
    if args.absorption:
        bias_absorption(graph, res, bottoms, N=3, visualize=args.visualize)
    state = {} if (args.bc_mode == "fused" or args.export) else None
    if args.quantize:
        set_layer_bits(graph, args.bits_weight, args.bits_activation, args.bits_bias, targ_layer)
        sharded = args.world_size > 1
        fold_ranges = {} if (args.granularity == "tensor" and not sharded) else None
        model = merge_batchnorm(model, graph, bottoms, targ_layer, ranges=fold_ranges)
        fused_clip = [-15, 15] if (args.clip_weight and args.bc_mode == "fused") else None
        graph = quantize_targ_layer(graph, args.bits_weight, args.bits_bias, targ_layer,
                                    granularity=args.granularity, symmetric=args.symmetric, clip=fused_clip,
                                    state=state, shard=sharded, weight_ranges=fold_ranges)
        set_quant_minmax(graph, bottoms)   # main_dfq.py:217
    if args.clip_weight and not (args.quantize and args.bc_mode == "fused"):
        clip_weight(graph, range_clip=[-15, 15], targ_type=targ_layer)
    if args.correction:
        # main_dfq.py:231 passes visualize= to a signature without it (TypeError in the
        # reference); this driver calls the documented signature.
        err = {k: esum_source(v) for k, v in state.items()} if (state and args.bc_mode == "fused") else None
        bias_correction(graph, bottoms, targ_layer, bits_weight=args.bits_weight, signed=args.symmetric,
                        error_sums=err)
    cle_wait()   # the launched CLE loop's error, if any, surfaces here
    torch.cuda.synchronize()
    print(f"DFQ weight transforms took {time.perf_counter() - t0:.3f} s on {args.device}")
    if args.export and args.quantize and state and rank == 0:
        from . import export
        clip = [-15, 15] if args.clip_weight else None   # fused in the sweep or clip_weight after it: same clamp
        export.save(args.export, graph, state, bits=args.bits_weight, granularity=args.granularity,
                    symmetric=args.symmetric, clip=clip)
        print(f"Exported {len(state)} quantized layers to {args.export}")

    # main_dfq.py:237-240: inference in eval mode -- also the observers set_layer_bits
    # created (new modules start in training mode)
    model.eval()
    accuracy = None
    if rank == 0:
        if args.quantize:
            replace_op()
        start = time.time()
        # the weights are final from here: the Quant* layers keep their weight /
        # bias fake-quant between batches (utils.quantize.frozen_weights)
        from .utils.quantize import frozen_weights
        with frozen_weights():
            accuracy = inference_all(model, args.task, args)
        print(f"Inference time is {time.time() - start} seconds")
        if args.quantize:
            restore_op()
    if args.world_size > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    if args.log and rank == 0:
        with open("dfq_result.txt", "a+") as ww:
            ww.write("task: {}, resnet: {}, relu: {}, equalize: {}, absorption: {}, quantize: {}, correction: {}, "
                     "clip: {}, bits_weight: {}, bits_activation: {}, bits_bias: {}\n".format(
                         args.task, args.resnet, args.relu, args.equalize, args.absorption, args.quantize,
                         args.correction, args.clip_weight, args.bits_weight, args.bits_activation, args.bits_bias))
            ww.write("Accuracy: {} %\n\n".format(accuracy * 100 if accuracy is not None else "n/a"))
    return model, graph, accuracy


if __name__ == "__main__":
    main(sys.argv[1:])
