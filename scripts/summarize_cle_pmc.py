"""profiles/<round>/cle_traffic_<model>.json from scripts/cle_pmc.sh's passes
(gpurun_out/<tag>): HBM bytes per CLE iteration of cle_loop_step_kernel (FETCH_SIZE
x2 per the gfx950 correction for wide streaming reads -- the loop's accesses are
mostly 16-B vector loads; narrower ones are uncalibrated, so the raw value is kept
beside it -- + WRITE_SIZE), next to the plan's algorithmic bytes per iteration and
the kernel's rocprof average; copies the kernel stats and counter CSVs.

  python scripts/summarize_cle_pmc.py <tag> <round> [models...]
"""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def lines(p):
    return [json.loads(ln) for ln in Path(p).read_text().splitlines() if ln.startswith("{")]


def main(tag, rnd, models):
    src, dst = ROOT / "gpurun_out" / tag, ROOT / "profiles" / rnd
    dst.mkdir(parents=True, exist_ok=True)
    for m in models:
        runs = lines(src / f"fetch_{m}.log")
        iters = sum(r["iterations"] for r in runs)
        groups = sum(r["iterations_launched"] for r in runs)
        vals = {}
        for name in ("fetch", "write"):
            f = next((src / f"{name}_{m}").rglob("*counter_collection.csv"))
            shutil.copy(f, dst / f"cle_pmc_{name}_{m}.csv")
            rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("cle_loop_step")]
            vals[name] = sum(float(r["Counter_Value"]) for r in rows) * 1024   # KB -> B
            vals[name + "_dispatches"] = len(rows)
        ks = next((src / f"kt_{m}").rglob("*kernel_stats.csv"))
        shutil.copy(ks, dst / f"cle_kernel_stats_{m}.csv")
        stats = {r["Name"].split("(")[0].replace("void ", "").replace("dfq::", ""): r for r in csv.DictReader(open(ks))}
        step = {k: v for k, v in stats.items() if k.startswith("cle_loop_step")}
        kt_runs = lines(src / f"kt_{m}.log")
        rd, wr = 2 * vals["fetch"], vals["write"]
        res = {"model": m, "kernel": "cle_loop_step_kernel", "runs": len(runs), "iterations": iters,
               "iteration_groups_launched": groups, "dispatches": vals["fetch_dispatches"],
               "FETCH_SIZE_bytes_raw_per_iteration": vals["fetch"] / iters,
               "hbm_read_bytes_per_iteration": rd / iters, "hbm_write_bytes_per_iteration": wr / iters,
               "hbm_bytes_per_iteration": (rd + wr) / iters,
               "algo_bytes_per_iteration": runs[-1]["bytes_per_iteration"],
               "correction": "FETCH_SIZE x2 (gfx950: 1/2 of 16 B/lane streaming reads), WRITE_SIZE as is; per "
                             "iteration = all step dispatches of the runs / their iterations (the queued no-op "
                             "group and the rolled-back speculative one included)",
               "rocprof_step_kernel": {k: {"calls": int(v["Calls"]), "avg_ns": float(v["AverageNs"])}
                                       for k, v in step.items()},
               "loop_device_ms_under_trace": [r["device_ms"] for r in kt_runs]}
        (dst / f"cle_traffic_{m}.json").write_text(json.dumps(res, indent=1))
        print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:] or ["mobilenetv2", "resnet50"])
