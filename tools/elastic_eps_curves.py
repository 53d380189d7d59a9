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
ap.add_argument("--npz", default=None, help="also store the per-step curves (prim, comb, reject) here")
ap.add_argument("--threads", type=int, default=0, help="OMP_NUM_THREADS for --ref (0: inherit)")
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
abort = None
curves = []
if a.ref:
    import subprocess
    import refio
    with tempfile.TemporaryDirectory() as tmp:
        refio.write_scene(sc, os.path.join(tmp, "s.bin"))
        env = dict(os.environ)
        if a.threads:
            env["OMP_NUM_THREADS"] = str(a.threads)
        r = subprocess.run([os.path.join(REPO, "oracle", "_ref", "ref_elastic_x"), "s.bin", "o.bin"], cwd=tmp,
                           capture_output=True, text=True, env=env)
        if r.returncode == 3 or "line search" in r.stderr:   # the reference threw inside step() (exit 3, or
            # std::terminate when the throw leaves an OpenMP region): keep the finished steps, record why
            abort = f"reference aborted (rc {r.returncode}) in step {{}}: " + r.stderr.strip().splitlines()[-1]
        elif r.returncode:
            sys.exit(r.stderr[-2000:])
        steps = refio.read_ref_result(os.path.join(tmp, "o.bin"), sc.n_nodes)
    curves = [(s["prim"], s["comb"], s["reject"]) for s in steps]
    if abort:
        abort = abort.format(len(steps) + 1)
    per = [stats(s["comb"]) for s in steps]
    src = "reference (oracle/_ref/ref_elastic_x, compiled from admm_anderson_xzu's own sources), this container's CPU"
else:
    pkg = importlib.import_module("aa-admm_amd")
    ctx = pkg.capi.Context(0)
    s = pkg.capi.solver_from_scene(ctx, sc)
    s.initialize(pkg.capi.settings_from_scene(sc))
    per = []
    for k in range(a.steps):
        try:
            s.step()
        except Exception as e:   # aa::Error ERR_NUMERIC: the same abort the reference raises
            abort = f"GPU_ABORT step {k + 1}: {e}"
            break
        h = s.history()
        curves.append((np.asarray(h["prim"]), np.asarray(h["comb"]), np.asarray(h["reject"])))
        per.append(stats(h["comb"]))
        print(f"[eps] step {len(per)}: {per[-1]}", file=sys.stderr, flush=True)
    s.close()
    ctx.close()
    src = "GPU solver (libaa_admm.so), MI355X"
summary = {k: sum(1 for p in per if p[k] is not None) for k in ("0.0001", "1e-06", "1e-08")}
json.dump({"scene": sc.name, "tets": sc.n_elements(), "nodes": sc.n_nodes, "cap": a.cap, "steps": a.steps,
           "steps_done": len(per), "abort": abort,
           "reached": summary, "per_step": per, "source": src, "wall_s": round(time.time() - t0, 1)},
          open(a.out, "w"), indent=1)
if a.npz:
    np.savez_compressed(a.npz, nrec=np.array([len(c[1]) for c in curves], np.int32),
                        prim=np.concatenate([c[0] for c in curves]) if curves else np.zeros(0),
                        comb=np.concatenate([c[1] for c in curves]) if curves else np.zeros(0),
                        reject=np.concatenate([c[2] for c in curves]).astype(np.int32) if curves else np.zeros(0, np.int32),
                        tets=np.array(a.tets), cap=a.cap, abort=np.array(abort or ""))
print(json.dumps({"reached": summary, "wall_s": round(time.time() - t0, 1)}))
