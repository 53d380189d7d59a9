#!/usr/bin/env python3
"""Static instruction histogram of one kernel in a device assembly file (hipcc --cuda-device-only
-S). Groups: fp64 arithmetic, division sequences (v_div_scale/fmas/fixup, v_rcp), moves (v_mov,
v_accvgpr_*), memory, scalar, branches. Used for the local-step instruction diet.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -o ek.s csrc/elastic_kernels.hip
    python tools/isa_hist.py ek.s k_local_z_hqILi4ELb0E [--json out.json]
"""
import collections
import json
import re
import sys


def kernel_body(text, needle):
    lines = text.splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(needle) + r"\S*:\s*(;.*)?$", l))
    name = lines[start].split(":")[0]
    body = []
    for l in lines[start + 1:]:
        if l.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", l):
            break
        t = l.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        body.append(t.split()[0])
    return name, body


def group(op):
    if op.startswith("v_accvgpr"):
        return "agpr moves (v_accvgpr_*)"
    if op.startswith(("v_mov", "v_pk_mov", "v_cndmask")):
        return "vgpr moves / selects"
    if op.startswith(("v_div_scale_f64", "v_div_fmas_f64", "v_div_fixup_f64", "v_rcp_f64", "v_rsq_f64")):
        return "fp64 division / rcp / rsq sequence"
    if op.endswith("_f64") or op.startswith("v_fma_f64"):
        return "fp64 arithmetic"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vector memory"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branches"
    if op.startswith("s_"):
        return "scalar"
    if op.startswith("v_"):
        return "other valu (int / f32 / cmp)"
    return "other"


def main():
    text = open(sys.argv[1]).read()
    name, body = kernel_body(text, sys.argv[2])
    ops = collections.Counter(body)
    groups = collections.Counter()
    for op, c in ops.items():
        groups[group(op)] += c
    out = {"kernel": name, "static_instructions": len(body), "groups": dict(groups.most_common()),
           "top_ops": dict(ops.most_common(40))}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4 and sys.argv[3] == "--json":
        json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
