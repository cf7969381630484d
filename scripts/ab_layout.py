"""N=1 placement A/B: per-tensor allocations vs the sharded path's per-field
arenas (seeded per-field layer order), fresh processes interleaved; sweep ms per
step (HIP events) of the default bench list.  argv: repeats, then the --layout
values to interleave (a field-major per-tensor order measured equal to the
eager order, 1.108-1.110 vs 1.109-1.115 ms, and was dropped)."""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for r in range(reps):
    for layout in (sys.argv[2:] or ["tensor", "arena"]):
        out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "30", "--warmup", "5",
                              "--cpu-seconds", "0", "--no-pipeline", "--no-secondary", "--layout", layout],
                             capture_output=True, text=True, timeout=300, cwd=ROOT)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        if not line:
            print(json.dumps({"layout": layout, "error": out.stderr[-300:]}), flush=True)
            continue
        d = json.loads(line[-1])
        print(json.dumps({"rep": r, "layout": layout, "launch_ms": d["roofline"]["launch_ms"],
                          "frac": d["roofline"]["frac"], "ms_per_step": d["ms_per_step"]}), flush=True)
