#!/usr/bin/env python3
"""Run-to-epsilon statistics of the C4 recipe (NeoHookean block drop, z-AA m=6) per time step,
from the reference (--ref: oracle/_ref/ref_elastic_x, container only) or from the GPU solver
(--gpu), on the same scene with the reference's default cap of 500 ADMM iterations per step and
no early stop, so both record whole curves. Per step: the first iteration reaching
comb <= r comb_0 (r = 1e-4, 1e-6, 1e-8) and the minimum of comb / comb_0. Shows whether the
time steps that miss epsilon within 500 iterations miss it in the reference too.

    python tools/elastic_eps_curves.py --ref --tets 20,8,10 --steps 20 --out profiles/r3_eps_ref_drop20.json
"""
import argparse
import importlib
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

ap = argparse.ArgumentParser()
g = ap.add_mutually_exclusive_group(required=True)
g.add_argument("--ref", action="store_true")
g.add_argument("--gpu", action="store_true")
ap.add_argument("--tets", default="20,8,10")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--cap", type=int, default=500)
ap.add_argument("--out", required=True)
a = ap.parse_args()
scenes = importlib.import_module("aa-admm_amd.scenes")
cx, cy, cz = (int(v) for v in a.tets.split(","))
sc = scenes.tet_drop(cx, cy, cz, iters=a.cap, n_steps=a.steps)


def stats(comb):
    comb = np.asarray(comb)
    out = {"iters": int(len(comb)), "min_over_comb0": float(comb.min() / comb[0]),
           "final_over_comb0": float(comb[-1] / comb[0])}
    for r in (1e-4, 1e-6, 1e-8):
        h = np.nonzero(comb <= r * comb[0])[0]
        out[f"{r:g}"] = int(h[0]) + 1 if len(h) else None
    return out


t0 = time.time()
if a.ref:
    import subprocess
    import refio
    with tempfile.TemporaryDirectory() as tmp:
        refio.write_scene(sc, os.path.join(tmp, "s.bin"))
        r = subprocess.run([os.path.join(REPO, "oracle", "_ref", "ref_elastic_x"), "s.bin", "o.bin"], cwd=tmp,
                           capture_output=True, text=True)
        if r.returncode:
            sys.exit(r.stderr[-2000:])
        steps = refio.read_ref_result(os.path.join(tmp, "o.bin"), sc.n_nodes)
    per = [stats(s["comb"]) for s in steps]
    src = "reference (oracle/_ref/ref_elastic_x, compiled from admm_anderson_xzu's own sources), this container's CPU"
else:
    pkg = importlib.import_module("aa-admm_amd")
    ctx = pkg.capi.Context(0)
    s = pkg.capi.solver_from_scene(ctx, sc)
    s.initialize(pkg.capi.settings_from_scene(sc))
    per = []
    for _ in range(a.steps):
        s.step()
        per.append(stats(s.history()["comb"]))
        print(f"[eps] step {len(per)}: {per[-1]}", file=sys.stderr, flush=True)
    s.close()
    ctx.close()
    src = "GPU solver (libaa_admm.so), MI355X"
summary = {k: sum(1 for p in per if p[k] is not None) for k in ("0.0001", "1e-06", "1e-08")}
json.dump({"scene": sc.name, "tets": sc.n_elements(), "nodes": sc.n_nodes, "cap": a.cap, "steps": a.steps,
           "reached": summary, "per_step": per, "source": src, "wall_s": round(time.time() - t0, 1)},
          open(a.out, "w"), indent=1)
print(json.dumps({"reached": summary, "wall_s": round(time.time() - t0, 1)}))
