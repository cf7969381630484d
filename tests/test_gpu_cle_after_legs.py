"""The CLE loop after the bench's other legs ran in the same
process: round 3 once saw MobileNetV2's pipeline take 2.4x
longer after the secondary / single-model legs (HIP-graph captures of sweep
plans, many plan creations over 2 GB layer lists).  Here the CLE stage is timed
fresh, then after those legs (the single-model latency leg with its HIP-graph
captures, and two >= 2 GiB sweep plans built, run and destroyed).  The ratio is
printed, not asserted (a wall-clock bound would make a correctness suite flaky
on a shared box; the bench line carries the figure as
``pipeline_ms.mobilenetv2.end_to_end_after_other_legs``).  What is asserted is
that the stage order is still bit-exact with the reference after those legs."""
import contextlib
import io
import logging
import statistics

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _cle_ms(reps=5):
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.pipeline import run_dfq
    from data_free_quantization_amd.utils.tracer import build_graph
    logging.getLogger("data_free_quantization_amd.bias_correction").setLevel(logging.ERROR)
    out = []
    for _ in range(reps + 1):
        m = zoo.build("mobilenetv2", seed=0, relu=True).cuda()
        g = build_graph(m, "positional")
        t = {}
        with contextlib.redirect_stdout(io.StringIO()):
            run_dfq(m, g.getGraph(), g.getBottoms(), (nn.Conv2d, nn.Linear), granularity="channel", symmetric=True,
                    bc_mode="fused", timings=t)
        out.append(t["cle"] * 1e3)
    return statistics.median(out[1:])


def test_cle_after_other_bench_legs():
    import bench
    from data_free_quantization_amd.sweep import SweepPlan
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    fresh = _cle_ms()
    bench.single_model_latency(dev, stream, reps=20)          # HIP-graph captures of sweep plans
    for model in ("resnet50", "mobilenetv2"):                 # plan churn over >= 2 GiB lists
        items, _, _, _ = bench.build_batch(model, dev, seed=99)
        plan = SweepPlan(items)
        bench.time_plan(plan, stream, dev, 3, 1)
        plan.destroy()
        del items, plan
        torch.cuda.empty_cache()
    after = _cle_ms()
    print(f"CLE stage: fresh {fresh:.3f} ms, after the other legs {after:.3f} ms (ratio {after / fresh:.3f})")
    from tests.parity import pipeline_mismatches
    par = pipeline_mismatches("mobilenetv2", 8, dev)
    assert par["mismatches"] == 0, par
