"""Per-kernel duration summary (avg / median / min / max, microseconds, launch count) from a
rocprofv3 rocpd SQLite database (the default output format of this image's rocprofv3), optionally
only the last N launches of each kernel.  Usage: rocpd_summary.py <run_results.db> [last_n]"""
import collections
import sqlite3
import statistics
import sys

db = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
c = sqlite3.connect(db)
rows = c.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
                 "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
by = collections.defaultdict(list)
for name, s, e in rows:
    by[name].append((e - s) / 1e3)
print(f"{'kernel':90s} {'n':>5s} {'avg':>8s} {'med':>8s} {'min':>8s} {'max':>8s}")
for name, ds in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    d = ds[-last:] if last else ds
    print(f"{name[:90]:90s} {len(d):5d} {statistics.mean(d):8.2f} {statistics.median(d):8.2f} {min(d):8.2f} {max(d):8.2f}")
