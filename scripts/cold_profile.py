"""cProfile of a cold full-DFQ run (after dfq_preload): which host calls carry the
first-run cost (allocator growth, pinned staging, graph capture, torch op loading)."""
import contextlib
import cProfile
import io
import logging
import pstats
import sys
from pathlib import Path

import torch
import torch.nn as nn

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from data_free_quantization_amd import _lib, zoo  # noqa: E402
from data_free_quantization_amd.pipeline import run_dfq  # noqa: E402
from data_free_quantization_amd.utils.tracer import build_graph  # noqa: E402

logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
args = [a for a in sys.argv[1:] if not a.startswith("--")]
name = args[0] if args else "mobilenetv2"
torch.zeros(1, device="cuda:0")
_lib.preload()
# host time per C entry point (ctypes calls do not show up in cProfile)
import collections, time  # noqa: E401,E402
L = _lib.load()
c_ms = collections.defaultdict(float)


def _wrap(name, fn):
    def call(*a):
        t = time.perf_counter()
        try:
            return fn(*a)
        finally:
            c_ms[name] += (time.perf_counter() - t) * 1e3
    return call


for _n in _lib.EXPORTS:
    setattr(L, _n, _wrap(_n, getattr(L, _n)))
if "--warm" in sys.argv:   # one untimed run first: the C-call times of a warm run
    m = zoo.build(name, seed=0, relu=True).cuda()
    g = build_graph(m, "positional")
    with contextlib.redirect_stdout(io.StringIO()):
        run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True,
                bc_mode="fused")
    torch.cuda.synchronize()
    c_ms.clear()
m = zoo.build(name, seed=0, relu=True).cuda()
g = build_graph(m, "positional")
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
with contextlib.redirect_stdout(io.StringIO()):
    run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True,
            bc_mode="fused")
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue())
print({k: round(v, 3) for k, v in sorted(c_ms.items(), key=lambda kv: -kv[1])})
