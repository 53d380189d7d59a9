#!/usr/bin/env python3
"""Per-kernel HBM traffic of one two-set (6 RHS) global solve against its algorithmic bytes.

    python tools/pmc_solve_table.py gpurun_out/pmc_r3_c4 gpurun_out/stats_c4.log [rhs_alg_bytes] > profiles/r3_c4_solve_pmc_table.txt

FETCH_SIZE x the k_copy calibration factor (tools/pmc_summary.py) + WRITE_SIZE per dispatch of
the last contiguous run of 6-RHS solve kernels, beside the factor bytes of the level each launch
streams (AA_SOLVE_STATS lines: fused subtrees, then per level forward, then backward in reverse).
Vector traffic (b, y, x, update vectors, tile partials) is not in the factor column.
"""
import csv
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import load, short   # noqa: E402

base, stats = sys.argv[1], sys.argv[2]
fetch = load(f"{base}_FETCH_SIZE/run_counter_collection.csv")
write = load(f"{base}_WRITE_SIZE/run_counter_collection.csv")
ids = sorted(set(fetch) & set(write))
copies = [(write[i][1], fetch[i][1]) for i in ids if "k_copy" in fetch[i][0] and fetch[i][1] > 0]
w_c, f_c = max(copies)
factor = w_c / f_c
names = [short(fetch[i][0]) for i in ids]


def nr(n):
    m = re.search(r"<([^>]*)>", n)
    return [a.strip() for a in m.group(1).split(",")] if m else []


is6 = [n.startswith(("k_fwd", "k_bwd")) and "6" in nr(n) for n in names]
end = max(j for j, v in enumerate(is6) if v)
start = end
while start - 1 >= 0 and is6[start - 1]:
    start -= 1
# level factor bytes from the stats log
sub_mb, lev = None, []
for line in open(stats):
    m = re.search(r"fused subtrees: \d+ .*?, ([\d.]+) MB/sweep", line)
    if m:
        sub_mb = float(m.group(1))
    m = re.search(r"\[solve\] level (\d+): .*?([\d.]+) MB/sweep, fwd tasks (\d+) .*?fwd tiles (\d+) .*?bwd tasks (\d+) .*?bwd tiles (\d+)", line)
    if m:
        lev.append(dict(mb=float(m.group(2)), ft=int(m.group(3)), ftl=int(m.group(4)), bt=int(m.group(5)), btl=int(m.group(6))))
alg = [("fused subtrees fwd", sub_mb)]
for k, L in enumerate(lev):
    if L["ft"]:
        alg.append((f"level {k} fwd rows", L["mb"]))
    if L["ftl"]:
        alg.append((f"level {k} fwd tiles", L["mb"]))
for k in range(len(lev) - 1, -1, -1):
    L = lev[k]
    if L["bt"]:
        alg.append((f"level {k} bwd rows", L["mb"]))
    if L["btl"]:
        alg.append((f"level {k} bwd tiles", L["mb"]))
alg.append(("fused subtrees bwd", sub_mb))
rows = list(range(start, end + 1))
print(f"# two-set solve, {len(rows)} kernels; FETCH_SIZE x {factor:.4f} (k_copy calibration) + WRITE_SIZE, MB per dispatch")
print(f"# {'kernel':28s} {'level':22s} {'factor MB':>10s} {'read MB':>9s} {'write MB':>9s} {'read/factor':>11s}")
tr = tw = ta = 0.0
for j, (lab, mb) in zip(rows, alg):
    i = ids[j]
    rd, wr = fetch[i][1] * factor / 1e6, write[i][1] / 1e6
    tr += rd; tw += wr; ta += mb or 0
    print(f"  {names[j]:28s} {lab:22s} {mb:10.2f} {rd:9.2f} {wr:9.2f} {rd / mb if mb else 0:11.3f}")
print(f"  {'total':28s} {'':22s} {ta:10.2f} {tr:9.2f} {tw:9.2f} {tr / ta:11.3f}")
rhs = [(fetch[i][1] * factor, write[i][1]) for i in ids if short(fetch[i][0]).startswith("k_rhs")]
if rhs:
    rd = sum(a for a, _ in rhs) / len(rhs) / 1e6
    wr = sum(b for _, b in rhs) / len(rhs) / 1e6
    alg_rhs = float(sys.argv[3]) / 1e6 if len(sys.argv) > 3 else None
    print(f"# k_rhs_slots: {len(rhs)} dispatches, read {rd:.2f} MB + write {wr:.2f} MB per dispatch" +
          (f" vs {alg_rhs:.2f} MB algorithmic (x{(rd + wr) / alg_rhs:.2f})" if alg_rhs else ""))
