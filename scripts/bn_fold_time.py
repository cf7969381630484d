import sys, time, ctypes as C
sys.path.insert(0, '.')
import torch, torch.nn as nn
from data_free_quantization_amd import zoo, _lib
from data_free_quantization_amd.utils import layer_transform as LT
from data_free_quantization_amd.utils.tracer import build_graph
for rep in range(3):
    m = zoo.build("mobilenetv2", seed=0, relu=True).cuda()
    g = build_graph(m, "positional"); graph, bottoms = g.getGraph(), g.getBottoms()
    torch.cuda.synchronize()
    orig = _lib.load().dfq_bn_fold_batch
    tc = {}
    def wrapped(*a):
        t0 = time.perf_counter(); r = orig(*a); tc['c'] = time.perf_counter() - t0; return r
    L = _lib.load()
    L.dfq_bn_fold_batch = wrapped
    t0 = time.perf_counter()
    LT.merge_batchnorm(m, graph, bottoms, (nn.Conv2d, nn.Linear))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    L.dfq_bn_fold_batch = orig
    print(rep, "merge_batchnorm ms", round((t1 - t0) * 1e3, 3), "C call ms", round(tc.get('c', 0) * 1e3, 3))
