"""Fixture of the geometry applications' before/after quality reports, from the REFERENCE itself:
the unmodified PlanarityOpt (airport3k, 100 iterations, m = 10 -- the geom_airport3k_aa10 scene)
and WireMeshOpt (costa2k, 60 iterations, m = 5 -- the geom_costa2k_wire_aa5 scene) built by
`make -C oracle ref`, run on the reference's own data files. Stores the values of every error
file they write (result/planarityErrBefore.txt, result/planatityErrAfter.txt,
result/{edge,angle,ref}_wiremeshErr{Before,After}.txt) and the report lines they print.

    make -C oracle ref && python tests/golden/make_golden_quality.py
"""
from __future__ import annotations

import os
import subprocess
import tempfile

import numpy as np

import importlib
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
gs = importlib.import_module("aa-admm_amd.geom_scenes")

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(os.path.dirname(HERE), "..", "oracle", "_ref")
DATA = "/root/reference/Geometry/Geometry_model/PQMeshData"

RUNS = {
    "pq_airport3k": ("PlanarityOpt", "airport3k", 100, 10, ["planarityErrBefore", "planatityErrAfter"]),
    "wire_costa2k": ("WireMeshOpt", "costa2k", 60, 5,
                     [f"{t}_wiremeshErr{w}" for t in ("edge", "angle", "ref") for w in ("Before", "After")]),
}
REPORT_KEYS = ("Before optimization", "After optimization", "Diagonal error", "Planarity error",
               "Reference surface distance", "Normalized edge length error", "Angle error")


def main():
    out = {}
    for key, (app, mesh, iters, m, files) in RUNS.items():
        with tempfile.TemporaryDirectory() as tmp:
            os.makedirs(os.path.join(tmp, "result"))
            with open(os.path.join(tmp, "opt.txt"), "w") as f:
                f.write(f"Iterations {iters}\nAndersonM {m}\n")
            r = subprocess.run([os.path.join(REF, app), os.path.join(DATA, "polymesh", f"{mesh}_poly.obj"),
                                os.path.join(DATA, "trimesh", f"{mesh}_tri.obj"), "opt.txt", "out.obj"],
                               cwd=tmp, capture_output=True, text=True, check=True)
            for name in files:
                out[f"{key}__{name}"] = np.loadtxt(os.path.join(tmp, "result", name + ".txt"))
            out[f"{key}__stdout"] = np.array([ln for ln in r.stdout.splitlines() if ln.startswith(REPORT_KEYS)])
        _, F = gs.read_obj(os.path.join(DATA, "polymesh", f"{mesh}_poly.obj"))   # the app's face order
        out[f"{key}__face_sizes"] = np.array([len(f) for f in F], np.int32)
        out[f"{key}__face_idx"] = np.array([v for f in F for v in f], np.int32)
        print(key, {k: v.shape for k, v in out.items() if k.startswith(key)})
    np.savez_compressed(os.path.join(HERE, "quality_reports.npz"), **out)


if __name__ == "__main__":
    main()
