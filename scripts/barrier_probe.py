"""Cost of the persistent CLE loop's grid barrier (diagnostics library):
microseconds per barrier for the two-level XCD barrier and the flat one."""
import json
import os
import sys
from pathlib import Path

os.environ.setdefault("DFQ_LIB", "diag")
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import ctypes as C  # noqa: E402
import torch  # noqa: E402
from data_free_quantization_amd import _lib  # noqa: E402

L = _lib.load_diag()
ws = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda:0")
s = torch.cuda.current_stream()
out = []
for mode in (0, 1):
    for bpc in (1, 2, 4):
        res = {}
        for nbar in (1, 401):
            best = None
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                _lib.check(L.dfq_probe_grid_barrier(nbar, bpc, mode, C.c_void_p(ws.data_ptr()), C.c_void_p(s.cuda_stream)),
                           "probe")
                e1.record(s)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
            res[nbar] = best
        out.append({"mode": ["xcd", "flat"][mode], "blocks_per_cu": bpc,
                    "us_per_barrier": round((res[401] - res[1]) / 400 * 1e3, 3), "launch_us": round(res[1] * 1e3, 1)})
print(json.dumps(out))
