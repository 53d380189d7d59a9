#!/usr/bin/env python3
"""Turn a reference run-to-epsilon curve written by tools/ref_geom_curve.py (profiles/<tag>.json,
oracle/_ref/ref_geom = the reference's ALMGeometrySolver compiled from its own sources) into a
golden fixture for the -m gpu tests: the per-iteration comb, the reference's residual_eps
(ALMGeometrySolver.h:172) and the scene digest (so the test can prove it regenerated the same
scene). Data only: no reference source travels.

    python tools/eps_fixture.py profiles/r5_c3_ref_curve1500.json tests/golden/eps_pq317_ref.npz \
        [profiles/r5_c3_ref_curve1500_p13.json]

An optional second curve is the reference on the same scene with its start positions perturbed
(tools/ref_geom_curve.py --perturb): where the late tail branches on rounding-level differences,
both of the reference's branches go into the fixture (comb_alt, perturb_alt).
"""
import importlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main(src, dst, alt=None):
    d = json.load(open(src))
    if d.get("perturb"):
        sys.exit("refusing a perturbed curve as a fixture")
    gs = importlib.import_module("aa-admm_amd.geom_scenes")
    from make_golden_geom import scene_digest
    n = int(d["points"] ** 0.5 + 0.5) - 1 if d["config"] == "c3" else None
    if d["config"] == "c3":
        sc = gs.pq_heightfield(n, n, iters=len(d["comb_all"]), aa_m=10, noise=0.3)
    else:
        n = int(d["scene"].split("x")[-1]) if "x" in d["scene"] else 707
        sc = gs.wire_grid(n, n, iters=len(d["comb_all"]), aa_m=20)
    assert sc.n_points == d["points"], (sc.n_points, d["points"])
    extra = {}
    if alt:
        da = json.load(open(alt))
        assert da["points"] == d["points"] and len(da["comb_all"]) == len(d["comb_all"]) and da["perturb"] > 0
        extra = {"comb_alt": np.asarray(da["comb_all"], np.float64), "perturb_alt": np.float64(da["perturb"])}
    np.savez(dst, comb=np.asarray(d["comb_all"], np.float64), eps_abs=np.float64(d["eps_abs"]),
             digest=scene_digest(sc), **extra,
             generator=np.str_(f"tools/ref_geom_curve.py --config {d['config']} --iters {len(d['comb_all'])} "
                               f"(oracle/_ref/ref_geom, OMP_NUM_THREADS={d.get('omp_threads')}) -> tools/eps_fixture.py"))
    print(dst, len(d["comb_all"]), "iterations, eps_abs", d["eps_abs"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
