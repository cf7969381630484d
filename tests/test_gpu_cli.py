"""main_dfq flag surface on the GPU (reference README.md:137 command)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("extra", [[], ["--granularity", "channel", "--symmetric", "--bc_mode", "fused"],
                                   ["--bc_mode", "reference"]])
def test_main_dfq_full_flags(extra, tmp_path, monkeypatch):
    from data_free_quantization_amd import main_dfq
    from data_free_quantization_amd.utils.quantize import QuantConv2d, QuantLinear
    monkeypatch.chdir(tmp_path)
    argv = ["--task", "cls", "--relu", "--equalize", "--absorption", "--quantize", "--correction", "--clip_weight",
            "--bits_weight", "8", "--bits_activation", "8", "--bits_bias", "8", "--log"] + extra
    model, graph, acc = main_dfq.main(argv)
    targets = [m for m in graph.values() if type(m) in (QuantConv2d, QuantLinear)]
    assert len(targets) == 53
    for m in targets:
        w = m.weight.detach()
        assert w.is_cuda and torch.isfinite(w).all()
        if "--granularity" not in extra:   # per-tensor 8-bit grid: at most 256 distinct values
            assert torch.unique(w).numel() <= 256
    assert (tmp_path / "dfq_result.txt").read_text().startswith("task: cls")
    # set_quant_minmax ran (main_dfq.py:217): every activation quantizer has a range;
    # after the second BN fold the statistics are N(0, 1) -> ReLU inputs [0, 6]
    from data_free_quantization_amd.utils import layer_transform as L
    qs = [m.quant for m in targets] + list(L.module_tensor_op.quants)
    assert all(float(q.running_max) > float(q.running_min) for q in qs)
    assert float(targets[0].quant.running_max) == np.float32(2.64)
    assert sum(float(q.running_min) == 0.0 and float(q.running_max) == 6.0 for q in qs) > 30


@pytest.mark.parametrize("extra", [[], ["--granularity", "channel", "--symmetric", "--bc_mode", "fused"],
                                   ["--bits_weight", "16"], ["--bits_weight", "16", "--granularity", "channel"]])
def test_main_dfq_export_roundtrip(extra, tmp_path, monkeypatch):
    """--export writes the integer grid (codes, scale, zero) and final biases; the
    exported layers dequantize to the model's weights bit for bit."""
    from data_free_quantization_amd import export, main_dfq
    monkeypatch.chdir(tmp_path)
    out = tmp_path / "mbv2_int8.safetensors"
    argv = ["--task", "cls", "--relu", "--equalize", "--absorption", "--quantize", "--correction", "--clip_weight",
            "--export", str(out)] + extra
    model, graph, _ = main_dfq.main(argv)
    meta, layers = export.load(out, device="cuda:0")
    assert meta["bits"] == (16 if "16" in extra else 8) and len(layers) == 53
    by_name = {str(k): k for k in graph}
    for key, entry in layers.items():
        layer = graph[by_name[key]]
        w = export.dequantize(meta, key, entry)
        assert torch.equal(w, layer.weight.detach()), key
        assert torch.equal(entry["bias"], layer.bias.detach()), key
        if "--symmetric" not in extra and "16" not in extra:
            assert entry["codes"].dtype == torch.uint8 and entry["scale"].numel() == 1
    if "16" in extra:   # the unsigned 16-bit grid really uses codes >= 32768
        assert meta["code_storage"] == "u16_in_i16"
        assert any(int((e["codes"] < 0).sum()) > 0 for e in layers.values())


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("gran", ["tensor", "channel"])
def test_quantize_targ_layer_sharded_rccl_world1(gran, monkeypatch):
    """quantize_targ_layer(shard=True) under an RCCL ("nccl") process group: the
    same weights, biases, codes, scales and E as the unsharded call."""
    import os
    import torch.distributed as dist
    from data_free_quantization_amd import zoo
    from data_free_quantization_amd.utils.layer_transform import quantize_targ_layer
    from data_free_quantization_amd.utils.tracer import build_graph
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    dev = torch.device("cuda:0")
    models, states = [], []
    for shard in (False, True):
        m = zoo.build("resnet50", seed=3).to(dev)
        g = build_graph(m, "positional").getGraph()
        st = {}
        if shard:
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        try:
            quantize_targ_layer(g, 8, 8, (nn.Conv2d, nn.Linear), granularity=gran, symmetric=gran == "channel",
                                clip=(-0.3, 0.3), state=st, shard=shard)
            torch.cuda.synchronize()
        finally:
            if shard:
                dist.destroy_process_group()
        models.append(m)
        states.append(st)
    for (n, a), (_, b) in zip(models[0].state_dict().items(), models[1].state_dict().items()):
        assert torch.equal(a, b), n
    assert states[0].keys() == states[1].keys() and len(states[0]) == 54
    for k in states[0]:
        for f in ("codes", "scale", "zero", "esum"):
            assert torch.equal(states[0][k][f], states[1][k][f]), (k, f)


def test_main_dfq_world2_one_gpu(tmp_path, monkeypatch):
    """main_dfq --world_size 2 under torchrun (two ranks on the one GPU, gloo
    between them): rank 0's export equals a single-process run's, tensor for
    tensor."""
    import os
    import subprocess
    import sys
    from safetensors.torch import load_file
    flags = ["--task", "cls", "--relu", "--equalize", "--absorption", "--quantize", "--correction", "--clip_weight",
             "--granularity", "channel", "--symmetric", "--bc_mode", "fused"]
    monkeypatch.chdir(tmp_path)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DFQ_DIST_BACKEND="gloo", PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    # both sides in fresh processes (the single-process side used to run inside the
    # test process, after the other GPU tests)
    one = tmp_path / "one.safetensors"
    r1 = subprocess.run([sys.executable, "-m", "data_free_quantization_amd.main_dfq"] + flags + ["--export", str(one)],
                        cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    assert r1.returncode == 0, r1.stdout[-3000:] + r1.stderr[-3000:]
    two = tmp_path / "two.safetensors"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "data_free_quantization_amd.main_dfq", "--world_size", "2"] + flags + ["--export", str(two)]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    a, b = load_file(str(one)), load_file(str(two))
    assert a.keys() == b.keys() and len(a) > 0
    bad = [(k, int((a[k] != b[k]).sum()), a[k].numel()) for k in a if not torch.equal(a[k], b[k])]
    assert not bad, (len(bad), bad[:12])


def test_main_dfq_evaluates_an_image_folder(tmp_path, monkeypatch):
    """inference_all (main_dfq.py:66-113) through the torchvision-free harness: a
    synthetic ImageFolder, the quantized MobileNetV2 with the tensor ops quantized
    (replace_op), an accuracy in [0, 1] written to dfq_result.txt."""
    from PIL import Image
    from data_free_quantization_amd import main_dfq
    rng = np.random.default_rng(0)
    for c in range(3):
        d = tmp_path / "val" / f"n{c:08d}"
        d.mkdir(parents=True)
        for k in range(3):
            Image.fromarray(rng.integers(0, 256, (240, 300, 3), dtype=np.uint8)).save(d / f"{k}.png")
    monkeypatch.chdir(tmp_path)
    argv = ["--task", "cls", "--relu", "--equalize", "--absorption", "--quantize", "--correction", "--clip_weight",
            "--val", str(tmp_path / "val"), "--batch_size", "4", "--workers", "0", "--log"]
    model, graph, acc = main_dfq.main(argv)
    assert acc is not None and 0.0 <= acc <= 1.0
    assert "Accuracy: " in (tmp_path / "dfq_result.txt").read_text()


def test_main_dfq_in_process_runs_are_identical(tmp_path, monkeypatch):
    """Two main_dfq runs inside one process (after whatever ran before in it) export
    the same bytes as a fresh process: no state carries over between runs."""
    import os
    import subprocess
    import sys
    from safetensors.torch import load_file
    from data_free_quantization_amd import main_dfq
    flags = ["--task", "cls", "--relu", "--equalize", "--absorption", "--quantize", "--correction", "--clip_weight",
             "--granularity", "channel", "--symmetric", "--bc_mode", "fused"]
    monkeypatch.chdir(tmp_path)
    paths = [tmp_path / f"in{i}.safetensors" for i in range(2)]
    for p in paths:
        main_dfq.main(flags + ["--export", str(p)])
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fresh = tmp_path / "fresh.safetensors"
    r = subprocess.run([sys.executable, "-m", "data_free_quantization_amd.main_dfq"] + flags + ["--export", str(fresh)],
                       cwd=tmp_path, env=dict(os.environ, PYTHONPATH=root), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    ref = load_file(str(fresh))
    for p in paths:
        got = load_file(str(p))
        bad = [(k, int((ref[k] != got[k]).sum()), ref[k].numel()) for k in ref if not torch.equal(ref[k], got[k])]
        assert not bad, (p.name, len(bad), bad[:12])
