"""Summarise a rocprofv3 kernel-trace database (per kernel: calls, avg/total time)."""
import sqlite3
import sys

db = sys.argv[1]
con = sqlite3.connect(db)
rows = con.execute("select name, count(*), avg(end-start), sum(end-start), min(end-start), max(end-start) "
                   "from kernels group by name order by sum(end-start) desc").fetchall()
tot = sum(r[3] for r in rows)
print(f"{'calls':>7} {'avg_us':>9} {'min_us':>8} {'max_us':>8} {'total%':>6}  kernel")
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{r[1]:7d} {r[2]/1e3:9.2f} {r[4]/1e3:8.2f} {r[5]/1e3:8.2f} {r[3]/tot*100:6.1f}  {r[0][:100]}")
print(f"total kernel time {tot/1e6:.2f} ms")
