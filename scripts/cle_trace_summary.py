"""CLE loop kernel timeline from a rocprofv3 ``--kernel-trace --output-format
csv`` run: the last device loop (the dispatches of the loop's kernels after the
last ``cle_loop_snap_kernel``; the caller's kernels that run beside a launched
loop are skipped), per launch position of an iteration the median duration and
the gap before it, the span per iteration, and the no-op launches after
convergence.  ``--launches`` is the loop's launches per iteration and
``--iterations`` its iteration count (both in the cle_ab line); ``--csv``
writes the loop's dispatches (small) for later reading.

  python scripts/cle_trace_summary.py <kernel_trace.csv> --launches 4 --iterations 44 [--csv out.csv]
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--launches", type=int, required=True)
    ap.add_argument("--iterations", type=int, required=True)
    ap.add_argument("--csv")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    k = lambda r, *names: next(r[n] for n in names if n in r)   # noqa: E731
    ev = []
    for r in rows:
        ev.append((int(k(r, "Start_Timestamp", "start")), int(k(r, "End_Timestamp", "end")),
                   k(r, "Kernel_Name", "kernel_name").split("(")[0].replace("dfq::", "").replace("void ", ""),
                   int(k(r, "Grid_Size_X", "Grid_Size", "grid_size") or 0) //
                   max(1, int(k(r, "Workgroup_Size_X", "Workgroup_Size", "workgroup_size") or 1))))
    ev.sort()
    snaps = [i for i, e in enumerate(ev) if "cle_loop_snap" in e[2] or "cle_loop_init" in e[2]]
    if not snaps:
        print("no CLE loop in the trace")
        return
    run = [e for e in ev[snaps[-1]:] if "cle_loop" in e[2]]
    steps = [e for e in run if "cle_loop_step" in e[2]]
    L, N = a.launches, a.iterations
    it = [steps[i * L:(i + 1) * L] for i in range(N)]
    noop = steps[N * L:]
    print(f"CLE loop: {len(run)} dispatches ({len(steps)} step launches: {N} iterations x {L} + {len(noop)} no-op), "
          f"span {(run[-1][1] - run[0][0]) / 1e3:.1f} us")
    print(f"{'position':>8s} {'kernel':34s} {'grid_med':>8s} {'dur_med':>8s} {'dur_min':>8s} {'gap_med':>8s}")
    prev_end = {}
    for p in range(L):
        d = [(x[p][1] - x[p][0]) / 1e3 for x in it if len(x) == L]
        g = []
        for i, x in enumerate(it):
            if len(x) != L:
                continue
            before = x[p - 1][1] if p else (it[i - 1][-1][1] if i and len(it[i - 1]) == L else None)
            if before is not None:
                g.append((x[p][0] - before) / 1e3)
        grid = statistics.median([x[p][3] for x in it if len(x) == L])
        print(f"{p:8d} {it[0][p][2][:34]:34s} {grid:8.0f} {statistics.median(d):8.2f} {min(d):8.2f} "
              f"{statistics.median(g) if g else 0:8.2f}")
    span = [(x[-1][1] - x[0][0]) / 1e3 for x in it if len(x) == L]
    per = [(it[i][-1][1] - it[i - 1][-1][1]) / 1e3 for i in range(1, N) if len(it[i]) == L]
    print(f"per iteration: launches span median {statistics.median(span):.2f} us; end to end median "
          f"{statistics.median(per):.2f} us (min {min(per):.2f}, max {max(per):.2f})")
    if noop:
        print(f"no-op launches after convergence: {len(noop)}, {sum((e[1] - e[0]) for e in noop) / 1e3:.1f} us busy, "
              f"last ends {(noop[-1][1] - it[-1][-1][1]) / 1e3:.1f} us after the last iteration")
    if a.csv:
        with open(a.csv, "w") as f:
            w = csv.writer(f)
            w.writerow(["start_ns", "end_ns", "kernel", "grid"])
            t0 = run[0][0]
            for e in run:
                w.writerow([e[0] - t0, e[1] - t0, e[2], e[3]])


if __name__ == "__main__":
    main()
