"""Generates the Geometry (ALM) golden fixtures under tests/golden/ from the REFERENCE itself.

oracle/Makefile (`make -C oracle ref`) compiles, from the reference's own sources under
/root/reference/Geometry: ref_geom (ALMGeometrySolver<3> fed from an AAGEOM01 scene file),
ref_geom_element (Constraint<3>::project per constraint type) and the unmodified PlanarityOpt
application. This script writes the scenes below, runs them, and stores inputs + outputs as .npz
(data only). The airport3k case also carries the residual curve of the reference's own
PlanarityOpt run on its own data files (Geometry/Geometry_model/PQMeshData), which pins the
scene recipe of geom_scenes.planarity_from_mesh. Run in the build container:

    make -C oracle ref && python tests/golden/make_golden_geom.py [--full]
"""
from __future__ import annotations

import importlib
import math
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import refio  # noqa: E402
gs = importlib.import_module("aa-admm_amd.geom_scenes")
from golden_io import save_geom_case  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref")
DATA = "/root/reference/Geometry/Geometry_model/PQMeshData"


def mixed_scene(n=8, aa_m=6, iters=50):
    """Every constraint type, hard and soft, plus all three regularisation row kinds."""
    V, Q = gs.quad_grid(n, n, shear=0.9)
    rng = np.random.default_rng(7)
    V = V + 0.01 * rng.standard_normal(V.shape)
    RV, RF = gs.field_trimesh(2 * n, 2 * n, shear=0.9)
    faces = [list(q) for q in Q]
    edges, _ = gs.edges_of(faces)
    npts = len(V)
    G = gs.ConstraintGroup
    groups = [
        G(gs.PLANE, Q.astype(np.int32), 1.0, True),
        G(gs.ANGLE, np.array([[f[0], f[1], f[3]] for f in faces], np.int32), 1.0, True,
          np.tile([math.pi / 3, 2 * math.pi / 3], (len(faces), 1))),
        G(gs.EDGE, np.array(edges[::2], np.int32), 1.0, True, np.full((len(edges[::2]), 1), 1.0 / n)),
        G(gs.CLOSENESS, np.arange(0, npts, 7, dtype=np.int32)[:, None], 1.0, True,
          V[::7] + 0.05),
        G(gs.POINT_TO_REF, np.arange(0, npts, 2, dtype=np.int32)[:, None], 2.0, False,
          np.zeros(((npts + 1) // 2, 1))),
        G(gs.EDGE, np.array(edges[1::2], np.int32), 0.5, False, np.full((len(edges[1::2]), 1), 1.1 / n)),
        G(gs.CLOSENESS, np.arange(1, npts, 5, dtype=np.int32)[:, None], 3.0, False, V[1::5]),
    ]
    reg = gs.RegBuilder()
    rings, bnd = gs.one_rings(npts, faces)
    for v in range(npts):
        if rings[v] is not None and len(rings[v]) == 4:
            r = rings[v]
            reg.laplacian([v, r[0], r[2]], [2.0, -1.0, -1.0], 0.3)
            reg.uniform_laplacian([v, r[1], r[3]], 0.2, relative=True)
    for v in range(0, npts, 11):
        reg.closeness(v, 5.0, V[v] + [0.0, 0.0, 0.02])
    sc = gs.GeomScene(x0=V, groups=groups, ref_points=V.copy(), surfaces=[(RV, RF)], penalty=50.0, iters=iters,
                      aa_m=aa_m, name="mixed", **reg.arrays())
    sc._avg_edge = gs.average_edge_length(V, faces)
    return sc


def bigplane_scene(n=10, aa_m=6, iters=40, solver="alm"):
    """Plane constraints of valence 4, 9 and 12 (vertex patches of a noisy quad grid) -- PlaneConstraint
    takes any number of points (Constraint.h:396-414; PlanarityOpt.cpp:235-246 adds one per face of
    any valence) -- hard and soft, with closeness + Laplacian regularisation."""
    V, Q = gs.quad_grid(n, n, shear=0.7)
    rng = np.random.default_rng(11)
    V = V + 0.02 * rng.standard_normal(V.shape)
    npts = len(V)
    grid = np.arange(npts).reshape(n + 1, n + 1)
    p12 = np.array([grid[i:i + 3, j:j + 4].ravel() for i in range(0, n - 1, 2) for j in range(0, n - 2, 3)], np.int32)
    p9 = np.array([grid[i:i + 3, j:j + 3].ravel() for i in range(1, n - 1, 3) for j in range(1, n - 1, 2)], np.int32)
    G = gs.ConstraintGroup
    groups = [G(gs.PLANE, Q.astype(np.int32), 1.0, True), G(gs.PLANE, p12, 1.0, True), G(gs.PLANE, p9, 2.0, False)]
    reg = gs.RegBuilder()
    faces = [list(q) for q in Q]
    rings, _ = gs.one_rings(npts, faces)
    for v in range(npts):
        reg.closeness(v, 1.0, V[v])
        if rings[v] is not None and len(rings[v]) == 4:
            reg.uniform_laplacian([v] + list(rings[v]), 0.1, relative=True)
    sc = gs.GeomScene(x0=V, groups=groups, ref_points=V.copy(), surfaces=[], penalty=20.0, iters=iters, aa_m=aa_m,
                      name="bigplane", solver=solver, **reg.arrays())
    sc._avg_edge = gs.average_edge_length(V, faces)
    return sc


def plain(sc, penalty=10.0):
    """The same scene driven through GeometrySolver<3> (Geometry/GeometrySolver.h)."""
    sc.solver = "plain"
    sc.penalty = penalty
    return sc


def airport(iters=100, aa_m=10):
    V, F = gs.read_obj(os.path.join(DATA, "polymesh", "airport3k_poly.obj"))
    RV, RF = gs.read_obj(os.path.join(DATA, "trimesh", "airport3k_tri.obj"))
    return gs.planarity_from_mesh(V, F, RV, np.array(RF, np.int32), iters=iters, aa_m=aa_m, name="airport3k")


def costa_wire(iters=60, aa_m=5):
    """WireMeshOpt's main on the reference's costa2k files: subdivide_and_smooth, half the
    average edge length, the optimize_mesh recipe (geom_scenes.wire_from_polymesh)."""
    V, F = gs.read_obj(os.path.join(DATA, "polymesh", "costa2k_poly.obj"))
    RV, RF = gs.read_obj(os.path.join(DATA, "trimesh", "costa2k_tri.obj"))
    return gs.wire_from_polymesh(V, F, RV, np.array(RF, np.int32), iters=iters, aa_m=aa_m, name="costa2k_wire")


def cases():
    return {
        "geom_costa2k_wire_aa5": costa_wire(),
        "geom_pq12_aa10": gs.pq_heightfield(12, 12, iters=60, aa_m=10),
        "geom_pq12_noaa": gs.pq_heightfield(12, 12, iters=40, aa_m=0),
        "geom_wire12_aa20": gs.wire_grid(12, 12, iters=60, aa_m=20),
        "geom_wire10_aa5": gs.wire_grid(10, 10, iters=40, aa_m=5),
        "geom_mixed_aa6": mixed_scene(),
        "geom_mixed_noaa": mixed_scene(aa_m=0, iters=30),
        "geom_airport3k_aa10": airport(),
        "geom_airport3k_noaa": airport(iters=40, aa_m=0),
        "geom_bigplane_aa6": bigplane_scene(),
        # GeometrySolver<3> (project_and_combine, Anderson on (u, x) with replace)
        "geom_plain_mixed_aa6": plain(mixed_scene(iters=40)),
        "geom_plain_mixed_noaa": plain(mixed_scene(aa_m=0, iters=30)),
        "geom_plain_bigplane_aa6": plain(bigplane_scene(), penalty=20.0),
        "geom_plain_pq12_aa10": plain(gs.pq_heightfield(12, 12, iters=50, aa_m=10), penalty=1e3),
    }


def run_ref(sc, tmp):
    pin, pout = os.path.join(tmp, "g.bin"), os.path.join(tmp, "g.out")
    refio.write_geom_scene(sc, pin)
    drv = "ref_geom_plain" if sc.solver == "plain" else "ref_geom"
    r = subprocess.run([os.path.join(REF, drv), pin, pout], cwd=tmp, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return refio.read_geom_result(pout, sc.n_points)


def run_planarity_app(tmp, iters, m):
    """The reference's own PlanarityOpt on its own airport3k files; returns the residual curve."""
    os.makedirs(os.path.join(tmp, "result"), exist_ok=True)
    with open(os.path.join(tmp, "opt.txt"), "w") as f:
        f.write(f"Iterations {iters}\nAndersonM {max(m, 1)}\n")
    if m == 0:
        return None   # the option file cannot express m = 0 (Parameters.h valid_parameters)
    r = subprocess.run([os.path.join(REF, "PlanarityOpt"), os.path.join(DATA, "polymesh", "airport3k_poly.obj"),
                        os.path.join(DATA, "trimesh", "airport3k_tri.obj"), "opt.txt", "out.obj"], cwd=tmp,
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return np.loadtxt(os.path.join(tmp, "result", f"residual-{m}.txt"))[:, 1]


def run_wire_app(tmp, iters, m):
    """The reference's own WireMeshOpt on its own costa2k files; returns the residual curve."""
    os.makedirs(os.path.join(tmp, "result"), exist_ok=True)
    with open(os.path.join(tmp, "opt.txt"), "w") as f:
        f.write(f"Iterations {iters}\nAndersonM {max(m, 1)}\n")
    r = subprocess.run([os.path.join(REF, "WireMeshOpt"), os.path.join(DATA, "polymesh", "costa2k_poly.obj"),
                        os.path.join(DATA, "trimesh", "costa2k_tri.obj"), "opt.txt", "out.obj"], cwd=tmp,
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return np.loadtxt(os.path.join(tmp, "result", f"residual-{m}.txt"))[:, 1]


def subdiv_fixture(tmp):
    """subdivide_and_smooth_mesh (MeshTypes.h:214-342) + average_edge_length of the reference on
    costa2k_poly (oracle/_ref/ref_subdiv): output positions, faces and the edge length."""
    out = os.path.join(tmp, "sub.bin")
    r = subprocess.run([os.path.join(REF, "ref_subdiv"), os.path.join(DATA, "polymesh", "costa2k_poly.obj"), out],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    d = open(out, "rb").read()
    nv, nf = struct.unpack("<ii", d[:8])
    el = struct.unpack("<d", d[8:16])[0]
    X = np.frombuffer(d[16:16 + 24 * nv], "<f8").reshape(-1, 3)
    off, sizes, idx = 16 + 24 * nv, [], []
    for _ in range(nf):
        k = struct.unpack("<i", d[off:off + 4])[0]
        off += 4
        sizes.append(k)
        idx += list(struct.unpack(f"<{k}i", d[off:off + 4 * k]))
        off += 4 * k
    V, F = gs.read_obj(os.path.join(DATA, "polymesh", "costa2k_poly.obj"))   # the input, as OpenMesh reads it
    np.savez_compressed(os.path.join(HERE, "mesh_wire_subdiv_costa2k.npz"), x=X, face_sizes=np.array(sizes, np.int32),
                        face_idx=np.array(idx, np.int32), edge_length=np.array(el), in_x=V,
                        in_face_sizes=np.array([len(f) for f in F], np.int32),
                        in_face_idx=np.array([v for f in F for v in f], np.int32))
    print("mesh_wire_subdiv_costa2k", nv, nf, el)


def element_tables(tmp):
    rng = np.random.default_rng(20191015)
    out = {}

    def run(op, cases, surface=None):
        buf = struct.pack("<ii", op, len(cases))
        if surface is not None:
            V, F = surface
            buf += struct.pack("<ii", len(V), len(F)) + V.astype("<f8").tobytes() + F.astype("<i4").tobytes()
        for k, prm, x in cases:
            buf += struct.pack("<i3d", k, *prm) + np.ascontiguousarray(x, "<f8").tobytes()
        pin, pout = os.path.join(tmp, "e.bin"), os.path.join(tmp, "e.out")
        with open(pin, "wb") as f:
            f.write(buf)
        r = subprocess.run([os.path.join(REF, "ref_geom_element"), pin, pout], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr)
        return np.fromfile(pout, "<f8")

    # planes: k = 3..8 mean-centred point sets, from near-planar to strongly warped
    for k in (3, 4, 5, 6, 8):
        cs = []
        for i in range(24):
            P = rng.standard_normal((k, 3)) * [1.0, 1.0, 10.0 ** rng.uniform(-8, 0)]
            P -= P.mean(0)
            cs.append((k, (0, 0, 0), P))
        out[f"plane{k}"] = (np.stack([c[2] for c in cs]), run(0, cs).reshape(len(cs), k, 3))
    # angles: random pairs across the range, colinear and degenerate cases
    cs, prms = [], []
    for i in range(64):
        v1, v2 = rng.standard_normal(3), rng.standard_normal(3)
        if i % 16 == 0:
            v2 = 2.0 * v1
        lo, hi = sorted(rng.uniform(0, math.pi, 2))
        if i % 4 == 0:
            lo, hi = math.pi / 4, 3 * math.pi / 4
        cs.append((3, (lo, hi, 0), np.stack([v1, v2])))
        prms.append((lo, hi))
    out["angle"] = (np.stack([c[2] for c in cs]), run(1, cs).reshape(len(cs), 2, 3), np.array(prms))
    # edges (incl. a zero vector: Eigen normalized() leaves it unchanged)
    cs = [(2, (0.7, 0, 0), rng.standard_normal((1, 3)) * (0 if i == 5 else 1)) for i in range(32)]
    out["edge"] = (np.stack([c[2] for c in cs]), run(2, cs).reshape(len(cs), 1, 3), np.full(32, 0.7))
    # closest points on a small height-field surface, from above/below/outside the footprint
    RV, RF = gs.field_trimesh(10, 10, shear=0.5)
    P = np.stack([rng.uniform(-0.3, 1.8, 200), rng.uniform(-0.3, 1.3, 200), rng.uniform(-0.5, 0.5, 200)], 1)
    cs = [(1, (0, 0, 0), p[None]) for p in P]
    out["closest"] = (P, run(3, cs, (RV, RF)).reshape(-1, 3), RV, RF)
    return out


def scene_digest(sc):
    """sha256 over the scene arrays: the full-size fixture stores outputs only (the scene is
    regenerated by geom_scenes) and this digest proves the regenerated scene is the same."""
    import hashlib
    h = hashlib.sha256()
    for a in [sc.x0, sc.reg_idx, sc.reg_coef] + [g.idx for g in sc.groups] + [V for V, F in sc.surfaces] + \
             [F for V, F in sc.surfaces]:
        h.update(np.ascontiguousarray(a).tobytes())
    return np.frombuffer(h.digest(), np.uint8)


def full_size_c3(tmp):
    """BASELINE configs[2] at full size (317 x 317 quads): the reference's residual curve and
    sampled solution points (the 2.4 MB solution itself is not stored)."""
    sc = gs.pq_heightfield(317, 317, iters=100, aa_m=10, noise=0.3)
    res = run_ref(sc, tmp)
    rng = np.random.default_rng(3)
    sample = np.sort(rng.choice(sc.n_points, 256, replace=False)).astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "full_c3_pq317.npz"), comb=res["comb"], sample=sample,
                        x_sample=res["x"][sample], x_sum=res["x"].sum(0), x_norm=np.linalg.norm(res["x"]),
                        digest=scene_digest(sc), ref_loop_s=res["loop_s"], ref_setup_s=res["setup_s"])
    print("full_c3_pq317", len(res["comb"]), res["loop_s"])


def full_size_c5(tmp):
    """BASELINE configs[4] at full size (707 x 707 wire mesh, 501 264 points, m = 20), 10 accepted
    iterations of the reference (its iterations cost ~0.5 s each here): the residual curve and
    sampled solution points."""
    sc = gs.wire_grid(707, 707, iters=10, aa_m=20)
    res = run_ref(sc, tmp)
    rng = np.random.default_rng(5)
    sample = np.sort(rng.choice(sc.n_points, 512, replace=False)).astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "full_c5_wire707.npz"), comb=res["comb"], sample=sample,
                        x_sample=res["x"][sample], x_sum=res["x"].sum(0), x_norm=np.linalg.norm(res["x"]),
                        digest=scene_digest(sc), ref_loop_s=res["loop_s"], ref_setup_s=res["setup_s"])
    print("full_c5_wire707", len(res["comb"]), res["loop_s"])


def main():
    only = [a for a in sys.argv[1:] if not a.startswith("--")]
    if only:   # regenerate only these trajectory fixtures
        with tempfile.TemporaryDirectory() as tmp:
            for name, sc in cases().items():
                if name in only:
                    res = run_ref(sc, tmp)
                    outputs = dict(comb=res["comb"], x=res["x"])
                    if name.startswith("geom_costa2k_wire"):
                        outputs["app_comb"] = run_wire_app(tmp, sc.iters, sc.aa_m)
                    save_geom_case(os.path.join(HERE, name + ".npz"), sc, outputs)
                    print(name, sc.n_points, len(res["comb"]), f"comb {res['comb'][0]:.4e} -> {res['comb'][-1]:.4e}")
        return
    if "--subdiv" in sys.argv:
        with tempfile.TemporaryDirectory() as tmp:
            subdiv_fixture(tmp)
        return
    if "--full" in sys.argv:
        with tempfile.TemporaryDirectory() as tmp:
            full_size_c3(tmp)
        return
    if "--full-c5" in sys.argv:
        with tempfile.TemporaryDirectory() as tmp:
            full_size_c5(tmp)
        return
    with tempfile.TemporaryDirectory() as tmp:
        for name, sc in cases().items():
            res = run_ref(sc, tmp)
            outputs = dict(comb=res["comb"], x=res["x"])
            if name.startswith("geom_airport3k"):
                app = run_planarity_app(tmp, sc.iters, sc.aa_m)
                if app is not None:
                    outputs["app_comb"] = app
            if name.startswith("geom_costa2k_wire"):
                outputs["app_comb"] = run_wire_app(tmp, sc.iters, sc.aa_m)
            save_geom_case(os.path.join(HERE, name + ".npz"), sc, outputs)
            print(name, sc.n_points, len(res["comb"]), f"comb {res['comb'][0]:.4e} -> {res['comb'][-1]:.4e}")
        et = element_tables(tmp)
        arrays = {}
        for k, v in et.items():
            if k.startswith("plane"):
                arrays[k + "_in"], arrays[k + "_out"] = v
            elif k in ("angle", "edge"):
                arrays[k + "_in"], arrays[k + "_out"], arrays[k + "_prm"] = v
            else:
                arrays["closest_in"], arrays["closest_out"], arrays["closest_V"], arrays["closest_F"] = v
        np.savez_compressed(os.path.join(HERE, "geom_elements.npz"), **arrays)
        print("geom_elements", sorted(arrays))


if __name__ == "__main__":
    main()
