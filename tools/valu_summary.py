"""Per-kernel VALU figures from the two SQ passes (tools/gpu.sh pmc, SQ counter groups).

    python tools/valu_summary.py gpurun_out/pmc_valu_c4 [out.json]

Counters are summed over every dispatch of a kernel (the short name k_...<...>), together with
the dispatches' wall time (End - Start). Derived per kernel:
  fp64_tflops    = 64 * SQ_INSTS_VALU_FLOPS_FP64 (+ _TRANS) / wall   (the counter counts the FLOPs of one
                   lane per wave instruction, FMA = 2: x 64 lanes = an upper bound, all lanes busy)
  valu_issue     = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES              share of wave time issuing VALU
  lane_util      = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)  active lanes per VALU cycle
                   (1.000 on a kernel without divergence, k_u_and_y)
The fp64 vector peak of MI355X: 256 CUs x 4 SIMDs x 16 fp64 FMA lanes/clk x 2 FLOP x 2.4 GHz
= 78.6 TFLOP/s (half the f32 vector rate, 157.3 TF in MI355X_MICROARCH.md).
"""
import collections
import csv
import json
import os
import re
import sys

PEAK_FP64_TF = 78.6


def short(name):
    m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def load(path, acc, wall):
    seen = set()
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        d = (path, r["Dispatch_Id"])
        if d not in seen:
            seen.add(d)
            wall[k][path] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            wall[k]["n:" + path] += 1


def main():
    base = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    wall = collections.defaultdict(lambda: collections.defaultdict(float))
    paths = []
    for i in (1, 2):
        p = os.path.join(base + "_%d" % i, "run_counter_collection.csv")
        if os.path.exists(p):
            load(p, acc, wall)
            paths.append(p)
    out = {}
    for k, c in acc.items():
        w = wall[k].get(paths[0], 0.0)
        n = int(wall[k].get("n:" + paths[0], 0))
        flops = 64 * (c.get("SQ_INSTS_VALU_FLOPS_FP64", 0) + c.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0))
        wc = c.get("SQ_WAVE_CYCLES", 0)
        av = c.get("SQ_ACTIVE_INST_VALU", 0)
        row = {
            "dispatches": n,
            "wall_ms_total": round(w * 1e3, 4),
            "fp64_flops_per_dispatch": flops / n if n else 0,
            "fp64_tflops": flops / w / 1e12 if w else 0,
            "frac_fp64_peak": flops / w / 1e12 / PEAK_FP64_TF if w else 0,
            "valu_insts_per_dispatch": c.get("SQ_INSTS_VALU", 0) / n if n else 0,
            "valu_issue_frac_of_wave_cycles": av / wc if wc else 0,
            "lane_util": c.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * av) if av else 0,
        }
        for extra in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                      "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD"):
            n2 = int(wall[k].get("n:" + paths[-1], 0))
            if extra in c and n2:
                row[extra.lower()[3:] + "_per_dispatch"] = c[extra] / n2
        if c.get("SQ_WAVES"):   # per-wave figures (SQ_WAVES counted in the first pass)
            nw = c["SQ_WAVES"]
            row["wave_cycles_per_wave"] = wc / nw
            row["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0) / nw
            if n and int(wall[k].get("n:" + paths[-1], 0)):
                nw2 = nw / n * int(wall[k].get("n:" + paths[-1], 0))   # waves of the second pass
                for extra in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"):
                    if extra in c:
                        row[extra.lower()[3:] + "_per_wave"] = c[extra] / nw2
        if "SQ_ACTIVE_INST_ANY" in c and "SQ_WAIT_INST_ANY" in c:
            tot = c["SQ_ACTIVE_INST_ANY"] + c["SQ_WAIT_INST_ANY"]
            row["issue_stall_share"] = c["SQ_WAIT_INST_ANY"] / tot if tot else 0
        out[k] = row
    ranked = sorted(out.items(), key=lambda kv: -kv[1]["wall_ms_total"])
    for k, r in ranked[:12]:
        print("%-34s n=%4d wall=%8.3f ms  %6.2f TF fp64 (%.3f of peak)  valu-issue %.3f  lanes %.3f"
              % (k[:34], r["dispatches"], r["wall_ms_total"], r["fp64_tflops"], r["frac_fp64_peak"],
                 r["valu_issue_frac_of_wave_cycles"], r["lane_util"]))
    if len(sys.argv) > 2:
        json.dump({"source": paths, "peak_fp64_tflops": PEAK_FP64_TF, "kernels": dict(ranked)},
                  open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
