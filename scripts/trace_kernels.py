"""Per-kernel summary of a rocprofv3 ``--kernel-trace --output-format csv`` run,
restricted to kernels whose name contains ``--match``: calls, mean / median
duration, and for the LAST stretch of matching dispatches (one stage: a stretch
ends where the gap to the next matching dispatch exceeds ``--split-us``) its
span, busy time and the gaps between its dispatches.

  python scripts/trace_kernels.py <kernel_trace.csv> --match bc_ [--split-us 200] [--csv out.csv]
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", required=True)
    ap.add_argument("--split-us", type=float, default=200.0)
    ap.add_argument("--csv")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    k = lambda r, *names: next(r[n] for n in names if n in r)   # noqa: E731
    ev = sorted((int(k(r, "Start_Timestamp", "start")), int(k(r, "End_Timestamp", "end")),
                 k(r, "Kernel_Name", "kernel_name").split("(")[0].replace("dfq::", "").replace("void ", ""))
                for r in rows)
    ev = [e for e in ev if a.match in e[2]]
    if not ev:
        print("no matching kernels")
        return
    by = {}
    for s, e, n in ev:
        by.setdefault(n, []).append((e - s) / 1e3)
    print(f"{'kernel':48s} {'calls':>6s} {'mean_us':>8s} {'med_us':>8s}")
    for n, d in sorted(by.items(), key=lambda x: -sum(x[1])):
        print(f"{n[:48]:48s} {len(d):6d} {statistics.mean(d):8.2f} {statistics.median(d):8.2f}")
    # the last stretch
    cut = len(ev) - 1
    while cut > 0 and (ev[cut][0] - ev[cut - 1][1]) / 1e3 <= a.split_us:
        cut -= 1
    st = ev[cut:]
    gaps = [(st[i][0] - st[i - 1][1]) / 1e3 for i in range(1, len(st))]
    busy = sum(e - s for s, e, _ in st) / 1e3
    print(f"last stretch: {len(st)} dispatches, span {(st[-1][1] - st[0][0]) / 1e3:.1f} us, busy {busy:.1f} us, "
          f"gap median {statistics.median(gaps) if gaps else 0:.2f} us, gaps total {sum(gaps):.1f} us")
    if a.csv:
        with open(a.csv, "w") as f:
            w = csv.writer(f)
            w.writerow(["start_ns", "end_ns", "kernel"])
            for s, e, n in st:
                w.writerow([s - st[0][0], e - st[0][0], n])


if __name__ == "__main__":
    main()
