"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; KB per dispatch).

    python tools/pmc_summary.py gpurun_out/pmc_r1_c4 [out.json]

Calibration (MI355X_MICROARCH.md, HBM): FETCH_SIZE is exact only for some access widths (it
reports half the bytes of 16-B/lane streaming reads on gfx950). Our kernels load 8 B per lane, so
the read factor is calibrated on our own k_copy dispatches (n doubles read + n written, n known
from the grid: the copy is grid-stride, so n is taken from the WRITE_SIZE, which the guide reports
exact for streaming stores): factor = WRITE_SIZE / FETCH_SIZE of the largest k_copy.
Groups: the global solve = the last contiguous run of k_fwd*/k_bwd*/k_asm dispatches of one width
(3 RHS: one solve; 6 RHS: the Z variant's two-set solve); the other
kernels are averaged per dispatch.
"""
import collections
import csv
import json
import re
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    out = {}
    for r in rows:
        out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0)
    return out


def short(name):
    m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", name)
    return m.group(1) if m else name.split("(")[0][-40:]


def main():
    base = sys.argv[1]
    fetch = load(f"{base}_FETCH_SIZE/run_counter_collection.csv")
    write = load(f"{base}_WRITE_SIZE/run_counter_collection.csv")
    ids = sorted(set(fetch) & set(write))
    # calibration on the largest k_copy
    copies = [(write[i][1], fetch[i][1]) for i in ids if "k_copy" in fetch[i][0] and fetch[i][1] > 0]
    w_c, f_c = max(copies) if copies else (1.0, 1.0)
    factor = w_c / f_c if f_c > 0 else 2.0
    per = collections.defaultdict(list)
    for i in ids:
        per[short(fetch[i][0])].append((fetch[i][1] * factor, write[i][1]))
    kern = {k: {"dispatches": len(v), "read_B": sum(a for a, _ in v) / len(v), "write_B": sum(b for _, b in v) / len(v)}
            for k, v in per.items()}
    names = [short(fetch[i][0]) for i in ids]
    is_solve = [n.startswith(("k_fwd", "k_bwd", "k_asm")) for n in names]

    def nsets(n):   # right-hand-side sets of a solve kernel: its template argument NR (3 or 6)
        m = re.search(r"<([^>]*)>", n)
        nr = [int(a) for a in m.group(1).split(",") if a.strip() in ("3", "6")] if m else []
        return nr[0] // 3 if nr else 0

    def last_run(sets):   # last contiguous run of solve kernels of one width
        idx = [j for j, n in enumerate(names) if is_solve[j] and nsets(n) == sets]
        if not idx:
            return None
        end = start = idx[-1]
        while start - 1 >= 0 and is_solve[start - 1] and nsets(names[start - 1]) == sets:
            start -= 1
        rd = sum(fetch[ids[j]][1] * factor for j in range(start, end + 1))
        wr = sum(write[ids[j]][1] for j in range(start, end + 1))
        return {"kernels": end - start + 1, "read_B": rd, "write_B": wr, "traffic_B": rd + wr}

    solve = last_run(1)    # one solve, 3 RHS
    solve2 = last_run(2)   # two-set solve, 6 RHS (Z variant: iteration solve + combined-residual solve)
    out = {"read_calibration": {"k_copy_write_B": w_c, "k_copy_fetch_B": f_c, "factor": factor},
           "solve_per_launch": solve, "solve2_per_launch": solve2, "per_kernel": kern}
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")
    print(json.dumps({"calibration": out["read_calibration"], "solve": solve, "solve2": solve2}, indent=1))
    for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["read_B"] * kv[1]["dispatches"])[:12]:
        print(f"  {k:28s} n={v['dispatches']:5d} read {v['read_B'] / 1e6:9.2f} MB write {v['write_B'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
