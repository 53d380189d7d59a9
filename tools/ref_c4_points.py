#!/usr/bin/env python3
"""Measured reference CPU points of the C4 recipe (container only: runs oracle/_ref/ref_elastic_x,
the reference's admm_anderson_xzu Solver compiled from its own sources; Solver.cpp:373-498 setup,
:122-251 loop). bench.py's C4 cpu_baseline extrapolates the reference's per-iteration time to 1M
tets from two samples (64k, 202k tets) as t ~ tets^b; this measures the same two samples plus a
larger one on the same host, so the fit's prediction at the large point can be checked against a
measurement. Writes profiles/<tag>.json.

    python tools/ref_c4_points.py --dims 40,16,20 60,24,28 80,32,40 --tag r5_c4_ref_points
"""
import argparse
import json
import math
import os
import statistics
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import importlib  # noqa: E402

import refio  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dims", nargs="+", default=["40,16,20", "60,24,28", "80,32,40"])
ap.add_argument("--tag", default="r5_c4_ref_points")
a = ap.parse_args()
scenes = importlib.import_module("aa-admm_amd.scenes")
drv = os.path.join(REPO, "oracle", "_ref", "ref_elastic_x")
threads = int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1)))
pts = []
for d in a.dims:
    dims = tuple(int(v) for v in d.split(","))
    sc = scenes.tet_drop(*dims, iters=10, n_steps=3)
    with tempfile.TemporaryDirectory() as tmp:
        refio.write_scene(sc, os.path.join(tmp, "s.bin"))
        t0 = time.time()
        r = subprocess.run([drv, "s.bin", "o.bin"], cwd=tmp, capture_output=True, text=True,
                           env=dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES="cores"))
        wall = time.time() - t0
        if r.returncode:
            sys.exit(r.stderr[-2000:])
        steps = refio.read_ref_result(os.path.join(tmp, "o.bin"), sc.n_nodes)
    per = [len(s["prim"]) / (s["step_ms"] / 1000.0) for s in steps[1:]]
    loop_s = sum(s["step_ms"] for s in steps) / 1000.0
    p = {"sample": sc.name, "tets": sc.n_elements(), "nodes": sc.n_nodes, "iters_per_s": round(statistics.median(per), 4),
         "ms_per_iter": round(1000.0 / statistics.median(per), 2), "wall_s": round(wall, 1),
         "setup_s_approx": round(wall - loop_s, 1)}
    print(json.dumps(p), flush=True)
    pts.append(p)
out = {"what": "reference X-order solver (oracle/_ref/ref_elastic_x) on make_tet_blocks drops, NeoHookean, z-AA m=6, "
               "3 time steps x 10 ADMM iters, median iters/s of steps 2-3; setup = wall - loop",
       "host": {"cpus": os.cpu_count(), "OMP_NUM_THREADS": threads}, "points": pts}
if len(pts) >= 3:
    p0, p1, p2 = pts[0], pts[1], pts[-1]
    b = math.log(p0["iters_per_s"] / p1["iters_per_s"]) / math.log(p1["tets"] / p0["tets"])
    pred = p1["iters_per_s"] * (p1["tets"] / p2["tets"]) ** b
    b_all = math.log(p0["iters_per_s"] / p2["iters_per_s"]) / math.log(p2["tets"] / p0["tets"])
    out["fit_check"] = {"exponent_two_small": round(b, 4), "predicted_iters_per_s": round(pred, 4),
                        "measured_iters_per_s": p2["iters_per_s"], "measured_over_predicted": round(p2["iters_per_s"] / pred, 4),
                        "exponent_smallest_to_largest": round(b_all, 4)}
    print(json.dumps(out["fit_check"]))
json.dump(out, open(os.path.join(REPO, "profiles", a.tag + ".json"), "w"), indent=1)
