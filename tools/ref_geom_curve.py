#!/usr/bin/env python3
"""Reference convergence curve of a geometry config (container only: runs oracle/_ref/ref_geom,
the reference's ALMGeometrySolver compiled from /root/reference): comb per accepted iteration
against the reference's residual_eps (ALMGeometrySolver.h:172), to show whether the reference
itself reaches it. Writes profiles/<tag>.json.

    python tools/ref_geom_curve.py --config c3 --iters 1000 --tag r3_c3_ref_curve
"""
import argparse
import importlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import refio  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3", choices=["c3", "c5"])
ap.add_argument("--iters", type=int, default=1000)
ap.add_argument("--nx", type=int, default=0)
ap.add_argument("--tag", default="r3_c3_ref_curve")
ap.add_argument("--gpu", action="store_true", help="the GPU solver's curve of the same scene (libaa_admm.so)")
ap.add_argument("--out", default=None, help="output path (default profiles/<tag>.json)")
ap.add_argument("--perturb", type=float, default=0.0,
                help="relative random perturbation of the start positions (seeded): how sensitive the curve's "
                     "late tail is to rounding-level differences")
a = ap.parse_args()
gs = importlib.import_module("aa-admm_amd.geom_scenes")
if a.config == "c3":
    n = a.nx or 317
    sc = gs.pq_heightfield(n, n, iters=a.iters, aa_m=10, noise=0.3)
else:
    n = a.nx or 707
    sc = gs.wire_grid(n, n, iters=a.iters, aa_m=20)
eps = 2.0 * (1e-8 * sc.avg_edge_length() * sc.hard_cols()) ** 2   # before any perturbation
if a.perturb:
    sc.x0 = sc.x0 * (1.0 + a.perturb * np.random.default_rng(7).standard_normal(sc.x0.shape))
if a.gpu:   # same scene, same cap, no early stop (the reference's stop is commented out too)
    pkg = importlib.import_module("aa-admm_amd")
    ctx = pkg.capi.Context(0)
    t0 = time.time()
    h, g = pkg.capi.run_geom(ctx, sc)
    wall = time.time() - t0
    res = {"comb": h["comb"], "loop_s": float(h["time_s"][-1]) if len(h["time_s"]) else None, "setup_s": None}
    g.close()
    ctx.close()
else:
    with tempfile.TemporaryDirectory() as tmp:
        refio.write_geom_scene(sc, os.path.join(tmp, "s.bin"))
        t0 = time.time()
        r = subprocess.run([os.path.join(REPO, "oracle", "_ref", "ref_geom"), "s.bin", "o.bin"], cwd=tmp,
                           capture_output=True, text=True)
        wall = time.time() - t0
        if r.returncode:
            sys.exit(r.stderr[-2000:])
        res = refio.read_geom_result(os.path.join(tmp, "o.bin"), sc.n_points)
comb = np.asarray(res["comb"])
idx = sorted(set([0, 1, 2, 4, 9, 19, 49, 99, 199, 299, 499, 699, 999, 1499, 1999, len(comb) - 1]) & set(range(len(comb))))
out = {"config": a.config, "scene": sc.name, "points": sc.n_points, "hard_cols": sc.hard_cols(), "anderson_m": sc.aa_m,
       "accepted_iters": int(len(comb)), "eps_abs": eps, "perturb": a.perturb,
       "first_iter_below_eps_abs": (int(np.nonzero(comb < eps)[0][0]) + 1 if (comb < eps).any() else None), "comb0": float(comb[0]),
       "min_comb": float(comb.min()), "min_comb_over_eps": float(comb.min() / eps),
       "reached_eps_abs": bool((comb < eps).any()),
       "first_iter_below": {f"{r:g}": (int(np.nonzero(comb <= r * comb[0])[0][0]) + 1 if (comb <= r * comb[0]).any() else None)
                            for r in (1e-2, 1e-4, 1e-6, 1e-8)},
       "curve": {str(i + 1): float(comb[i]) for i in idx},
       "loop_s": res["loop_s"], "setup_s": res["setup_s"], "wall_s": round(wall, 1),
       "omp_threads": os.environ.get("OMP_NUM_THREADS", str(os.cpu_count())),
       "source": ("GPU solver (libaa_admm.so), MI355X" if a.gpu else
                  "oracle/_ref/ref_geom (reference ALMGeometrySolver compiled from its own sources), this container's CPU"),
       "comb_all": [float(c) for c in comb]}
json.dump(out, open(a.out or os.path.join(REPO, "profiles", a.tag + ".json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k not in ("curve", "comb_all")}))
