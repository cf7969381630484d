"""bench.py's N-rank launcher: ``python bench.py --gpus N`` with
no torchrun environment must start N ranks (torchrun as a child process, before
any GPU call), every rank must check the world size against ``--gpus``, and a
mismatch must fail the run.  CPU: ``--probe-ranks`` joins a gloo group without
touching the GPU.  GPU: the real bench at N = 2 on the one card (gloo between
the two processes)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(DFQ_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    env.update(kw)
    return env


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_launch_command_child_count():
    sys.path.insert(0, str(ROOT))
    import bench
    cmd = bench.launch_command(8, ["--gpus", "8", "--steps", "3"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert cmd[-5].endswith("bench.py")


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    """No WORLD_SIZE in the environment: the parent starts torchrun with n ranks,
    each joins the group, and rank 0's line lists n distinct processes."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--probe-ranks"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    rows = lines[0]["probe_ranks"]
    assert lines[0]["n_gpus"] == n and lines[0]["backend"] == "gloo"
    assert sorted(x[0] for x in rows) == list(range(n))
    assert all(x[1] == n for x in rows)
    assert len({x[3] for x in rows}) == n            # one process per rank
    assert os.getpid() not in {x[3] for x in rows}    # none of them is the caller


def test_world_mismatch_fails():
    """A rank whose process group does not have --gpus ranks exits non-zero."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3", "--probe-ranks"],
                       capture_output=True, text=True, timeout=120, cwd=str(ROOT),
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                                MASTER_PORT="29599"))
    assert r.returncode != 0
    assert "--gpus 3 but the process group has 2" in r.stderr


def test_launched_mismatch_fails():
    """torchrun with 2 ranks but --gpus 3 in the bench arguments: every rank refuses."""
    sys.path.insert(0, str(ROOT))
    import bench
    cmd = bench.launch_command(2, ["--gpus", "3", "--probe-ranks"], bench._free_port())
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=_env(), cwd=str(ROOT))
    assert r.returncode != 0
    assert not _json_lines(r.stdout)


def test_single_gpu_no_spawn():
    """--gpus 1 runs in this process (no torchrun child)."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--probe-ranks"],
                       capture_output=True, text=True, timeout=120, env=_env(), cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_lines(r.stdout)[0]
    assert line["n_gpus"] == 1 and line["probe_ranks"][0][3] != os.getpid()


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu():
    """The real bench at --gpus 2 as the driver may call it (no torchrun env), both
    ranks on the one GPU with gloo between them.  The headline must be the ONE
    N = 1 list (MobileNetV2 x155, 8,215 layers) LPT-sharded over the two ranks
    (strong scaling, outputs left sharded), every rank's share checked against the
    oracle with 0 mismatches and both ranks holding checked layers; the gathers,
    weak scaling and configs[4]'s sharded list beside it."""
    r = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--no-secondary", "--no-pipeline", "--prewarm-ms", "50"],
                       capture_output=True, text=True, timeout=600, env=_env(OMP_NUM_THREADS="4"), cwd=str(ROOT))
    print(r.stderr[-3000:])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    res = lines[0]
    print(json.dumps({k: res[k] for k in ("value", "ms_per_step", "n_gpus", "rccl_ranks", "backend", "scaling")}))
    print(json.dumps(res["sharded_gathers"]), json.dumps(res["weak_scaling"]))
    print(json.dumps(res["configs4_sharded"]))
    assert res["n_gpus"] == 2 and res["rccl_ranks"] == 2 and res["scaling"] == "strong"
    cfg = res["config"]
    assert cfg["layers"] == 8215 and cfg["copies"] == 155
    assert sum(cfg["layers_per_rank"]) == 8215 and all(n > 0 for n in cfg["layers_per_rank"])
    assert len(cfg["algo_bytes_per_rank"]) == 2
    # value = the whole list's weight bytes (not N lists) over the max-over-ranks step
    assert abs(res["value"] - 4 * cfg["weights_per_copy"] * 155 / (res["ms_per_step"] / 1e3) / 1e9) \
        <= 0.01 * res["value"]
    tp = res["parity"]["timed_sweep"]
    assert tp["all_ranks"]["tensors"] == 3 * 53 and tp["owners"] == [0, 1]
    assert res["parity"]["mismatches"] == 0 and tp["mismatches"] == 0
    g = res["sharded_gathers"]
    assert g["layers_per_rank"] == cfg["layers_per_rank"]
    assert all(g[k] > 0 for k in ("sweep_ms", "sweep_gather_root_ms", "sweep_allgather_ms"))
    assert res["weak_scaling"]["lists"] == 2
    c4 = res["configs4_sharded"]
    assert c4["rccl_ranks"] == 2 and all(n > 0 for n in c4["layers_per_rank"])
    assert c4["parity"]["mismatches"] == 0 and c4["parity"]["owners"] == [0, 1]
    assert len(res["roofline"]["launch_ms_per_rank"]) == 2
