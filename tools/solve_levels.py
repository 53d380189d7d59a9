"""Per-launch durations of the last global solve in a rocprofv3 kernel trace (NO_GRAPH runs).

    python tools/solve_levels.py run_kernel_trace.csv [3|6]
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
# optional argv[2]: right-hand sides of the solve to show (3 = one solve, 6 = the two-set solve)
want = sys.argv[2] if len(sys.argv) > 2 else None


def nr_of(n):
    m = re.search(r"k_[a-z_0-9]+<([^>]*)>", n)
    nr = [a.strip() for a in m.group(1).split(",") if a.strip() in ("3", "6")] if m else []
    return nr[0] if nr else None


idx = set(i for i, n in enumerate(names)
          if ("k_fwd" in n or "k_bwd" in n or "k_asm" in n) and (want is None or nr_of(n) == want))
end = max(idx)
start = end
while start - 1 in idx:
    start -= 1
tot = 0
for r in rows[start:end + 1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot += d
    m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", r["Kernel_Name"])
    nm = m.group(1) if m else r["Kernel_Name"][:20]
    print("  %-14s grid %8d wg %4s lds %6s vgpr %3s %7.2f us" % (nm, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]),
          r["Workgroup_Size_X"], r["LDS_Block_Size"], r["VGPR_Count"], d))
print(" kernels", end - start + 1, "sum %.1f us, wall %.1f us" % (tot, (int(rows[end]["End_Timestamp"]) - int(rows[start]["Start_Timestamp"])) / 1000))
