"""Per-kernel summary (ms/step, calls, avg us) from a rocprofv3 sqlite results db.
    python tools/kstats_db.py <results.db> <steps> [top]"""
import sqlite3
import sys

db, steps = sys.argv[1], int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = list(c.execute(f"select {name}, count(*), sum(end - start) from kernels group by {name}"))
tot = sum(r[2] for r in rows)
for n, k, t in sorted(rows, key=lambda r: -r[2])[:top]:
    print("%6.2f%% %8.3f ms/step %6d calls avg %8.1f us  %s" % (100 * t / tot, t / 1e6 / steps, k, t / k / 1e3, n[:100]))
print("total ms/step %.3f over %d kernels" % (tot / 1e6 / steps, len(rows)))
