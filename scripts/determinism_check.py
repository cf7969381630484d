"""Repeat main_dfq (MobileNetV2, channel sym INT8, fused BC, --export) in fresh
processes -- sequentially and two at a time on the same GPU -- and compare every
exported tensor: the DFQ path must be deterministic."""
import hashlib
import os
import subprocess
import sys
import tempfile

from safetensors.torch import load_file

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FLAGS = ["--task", "cls", "--relu", "--equalize", "--absorption", "--quantize", "--correction", "--clip_weight",
         "--granularity", "channel", "--symmetric", "--bc_mode", "fused"]
d = tempfile.mkdtemp()
env = dict(os.environ, PYTHONPATH=ROOT)


def start(i):
    out = os.path.join(d, f"run{i}.safetensors")
    return out, subprocess.Popen([sys.executable, "-m", "data_free_quantization_amd.main_dfq"] + FLAGS +
                                 ["--export", out], cwd=d, env=env, stdout=subprocess.DEVNULL,
                                 stderr=subprocess.DEVNULL)


def digest(path):
    t = load_file(path)
    return {k: hashlib.sha1(v.numpy().tobytes()).hexdigest()[:12] for k, v in t.items()}


runs = []
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):          # sequential
    out, p = start(i)
    assert p.wait(timeout=200) == 0
    runs.append(out)
for j in range(int(sys.argv[2]) if len(sys.argv) > 2 else 2):          # pairs sharing the GPU
    o1, p1 = start(100 + 2 * j)
    o2, p2 = start(101 + 2 * j)
    assert p1.wait(timeout=200) == 0 and p2.wait(timeout=200) == 0
    runs += [o1, o2]
ref = digest(runs[0])
for r in runs[1:]:
    h = digest(r)
    bad = [k for k in ref if ref[k] != h[k]]
    print(os.path.basename(r), "differs in", len(bad), bad[:6], flush=True)
