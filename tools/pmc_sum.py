"""Sum rocprofv3 --pmc counter CSVs per kernel (kernels whose name contains a filter string).

    python tools/pmc_sum.py DIR FILTER [OUT.json]

Prints and (optionally) merges into OUT.json: {kernel: {"dispatches": n, counter: total, ...}}.
Used by tools/gpu.sh's pmc step when PMC_KERNEL is set, so the raw per-dispatch CSVs can stay
on the box (they exceed gpurun's copy-back limit on the long configs).
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, filt = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if filt not in k:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    res = json.load(open(out)) if out and os.path.exists(out) else {}
    for k, v in tot.items():
        e = res.setdefault(k, {})
        e["dispatches"] = max(e.get("dispatches", 0), len(disp[k]))
        e.update(v)
        print(k[:80], len(disp[k]), dict(v))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
