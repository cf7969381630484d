"""CLE loop kernel timeline from a rocprofv3 ``--kernel-trace --output-format
csv`` run: the last run of consecutive ``cle_loop_*`` dispatches (one device
loop), per kernel kind the calls and mean / median duration, the gaps between
dispatches, and the span per iteration (tiles/stop-rule launch to the next).

  python scripts/cle_trace_summary.py <kernel_trace.csv> [--iterations N]
"""
import csv
import statistics
import sys


def main(path, iters=None):
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("empty trace")
        return
    k = lambda r, *names: next(r[n] for n in names if n in r)   # noqa: E731
    ev = []
    for r in rows:
        ev.append((int(k(r, "Start_Timestamp", "start")), int(k(r, "End_Timestamp", "end")),
                   k(r, "Kernel_Name", "kernel_name"), int(k(r, "Grid_Size_X", "Grid_Size", "grid_size") or 0),
                   int(k(r, "Workgroup_Size_X", "Workgroup_Size", "workgroup_size") or 1)))
    ev.sort()
    # the last maximal run of CLE loop kernels (gate / snapshot kernels included)
    is_cle = lambda name: "cle_loop" in name or "cle_caller_gate" in name   # noqa: E731
    end = max(i for i, e in enumerate(ev) if is_cle(e[2]))
    start = end
    while start > 0 and is_cle(ev[start - 1][2]):
        start -= 1
    run = [e for e in ev[start:end + 1] if "cle_caller_gate" not in e[2]]
    kinds = {}
    for i, (s, e, name, g, w) in enumerate(run):
        short = name.split("(")[0].replace("dfq::", "")
        if "apply" in short:
            short += f"[grid {g // max(w, 1)}]"
        d = kinds.setdefault(short, {"dur": [], "gap": []})
        d["dur"].append((e - s) / 1e3)
        if i:
            d["gap"].append((s - run[i - 1][1]) / 1e3)
    print(f"CLE run: {len(run)} dispatches, span {(run[-1][1] - run[0][0]) / 1e3:.1f} us")
    print(f"{'kernel':60s} {'calls':>6s} {'mean_us':>8s} {'med_us':>8s} {'gap_med':>8s}")
    for n, d in kinds.items():
        print(f"{n[:60]:60s} {len(d['dur']):6d} {statistics.mean(d['dur']):8.2f} {statistics.median(d['dur']):8.2f} "
              f"{statistics.median(d['gap']) if d['gap'] else 0:8.2f}")
    tiles = [i for i, e in enumerate(run) if "tiles_fin" in e[2]]
    if len(tiles) > 2:
        per = [(run[b][1] - run[a][1]) / 1e3 for a, b in zip(tiles, tiles[1:])]
        print(f"per iteration (tiles end to tiles end): median {statistics.median(per):.2f} us, "
              f"min {min(per):.2f}, max {max(per):.2f}, iterations {len(per) + 1}")
        mid = tiles[len(tiles) // 2]
        prev = tiles[len(tiles) // 2 - 1]
        print("one iteration (middle of the loop):")
        for s, e, name, g, w in run[prev + 1:mid + 1]:
            print(f"  {name.split('(')[0].replace('dfq::', '')[:50]:50s} dur {(e - s) / 1e3:7.2f} us  grid {g // max(w, 1)}")


if __name__ == "__main__":
    main(sys.argv[1])
