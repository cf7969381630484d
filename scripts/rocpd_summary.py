"""Per-kernel summary (calls, total / average microseconds) of a rocprofv3 rocpd
database (the default output format of this image's rocprofv3)."""
import collections
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
names = {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
rows = list(c.execute("select kernel_id, start, end, grid_size_x, workgroup_size_x from rocpd_kernel_dispatch "
                      "order by start"))
agg = collections.defaultdict(lambda: [0, 0.0])
for kid, s, e, g, w in rows:
    a = agg[names.get(kid, kid)]
    a[0] += 1
    a[1] += (e - s) / 1e3
print(f"{'kernel':60s} {'calls':>7s} {'total_us':>10s} {'avg_us':>8s}")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{str(k)[:60]:60s} {n:7d} {t:10.1f} {t / n:8.2f}")
if len(sys.argv) > 2:   # timeline of the last N dispatches: start offset, duration, gap
    n = int(sys.argv[2])
    prev_end = None
    for kid, s, e, g, w in rows[-n:]:
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        print(f"{str(names.get(kid, kid))[:50]:50s} dur {(e - s) / 1e3:8.2f} gap {gap:8.2f} grid {g // max(w, 1)}")
        prev_end = e
