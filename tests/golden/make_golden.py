"""Generates the golden fixtures under tests/golden/ from the REFERENCE itself.

The reference (bldeng/AA-ADMM) is compiled from its own sources under /root/reference by
oracle/Makefile (`make -C oracle ref`) into oracle/_ref/ -- headless drivers replace the GUI
sample loops (oracle/ref_drivers/*.cpp). This script feeds them the scenes below and stores
inputs + outputs as .npz (data only, no code). Run in the build container:

    make -C oracle ref && python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib
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
scenes = importlib.import_module("aa-admm_amd.scenes")
from golden_io import save_case  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref")


def cases():
    S = scenes
    return {
        "cloth12_ux_aa6": S.cloth(12, 12, iters=40, n_steps=3),
        "cloth12_ux_noaa": S.cloth(12, 12, iters=40, n_steps=2, accel=0),
        "cloth12_z_noaa": S.cloth(12, 12, iters=30, n_steps=2, accel=0, variant=S.VARIANT_X),
        "cantilever_z_nh_aa6": S.cantilever(20, 4, 5, S.NEOHOOKEAN, iters=50, n_steps=1),   # BASELINE configs[0]
        "cant8_z_lin_aa6": S.cantilever(8, 2, 2, S.LINEAR, iters=30, n_steps=2),
        "cant8_ux_lin_aa6": S.cantilever(8, 2, 2, S.LINEAR, iters=30, n_steps=2, variant=S.VARIANT_H),
        "cant8_z_stvk_noaa": S.cantilever(8, 2, 2, S.STVK, iters=30, n_steps=2, accel=0),
        "beams2_z_aa6": S.beams(2, iters=40, n_steps=2),
        "beams2_ux_aa6": S.beams(2, iters=40, n_steps=2, variant=S.VARIANT_H),
        "cloth12_ux_aa1": S.cloth(12, 12, iters=30, n_steps=2, aa_m=1),
        "cant8_ux_lin_aa3_pen": _with(S.cantilever(8, 2, 2, S.LINEAR, iters=30, n_steps=1, variant=S.VARIANT_H, aa_m=3),
                                      penalty=4.0),
        # C4 recipe at small size: NeoHookean block free fall from a squashed pose (rest != initial)
        "drop6_z_nh_aa6": S.tet_drop(6, 2, 3, iters=40, n_steps=2),
        # ... at 8 000 tets and 100 iterations a step: the Z variant's Anderson rejects (the
        # re-solve from the defaults, Solver.cpp:159-181) happen -- the small goldens have none
        "drop20_z_nh_aa6_rej": S.tet_drop(20, 8, 10, iters=100, n_steps=2),
        # collision terms + obstacles (the plinko samples' horse759 mesh) and wind (windyflag)
        "plinkohit_ux_noaa": S.plinko_hit(*horse(), n_steps=20),
        "plinkohit_ux_aa2": S.plinko_hit(*horse(), n_steps=16, accel=1, aa_m=2),
        "obstacles_ux_aa5": S.obstacle_course(*horse()),
        "windycloth12_ux_aa6": S.windy_cloth(12, 12),
        "windycloth12_z_noaa": _with(S.windy_cloth(12, 12, accel=0, iters=30), variant=S.VARIANT_X),
    }


HORSE = "/root/reference/admm_anderson_hard_zxu/samples/data/horse759"


def horse():
    """The plinko samples' tet mesh (samples/data/horse759.{ele,node}, read with the
    load_elenode restatement) -- kept as input data in mesh_horse759.npz, so the GPU tests do
    not need the reference tree. The same file pins the loader and binding::add_tetmesh's
    masses: the node coordinates as parsed (float64), and the reference's own mcl loader +
    apply_xform + TetMesh::weighted_masses output (oracle/_ref/ref_tetmesh) for the plinkohit
    transform."""
    path = os.path.join(HERE, "mesh_horse759.npz")
    if os.path.exists(HORSE + ".ele"):
        v, t = scenes.load_elenode(HORSE)
        with open(HORSE + ".node") as f:
            rows = [ln.split() for ln in f if ln.split() and not ln.lstrip().startswith("#")][1:]
        nodes64 = np.array([[float(r[1]), float(r[2]), float(r[3])] for r in rows[:len(v)]], np.float64)
        xf = np.array([13.0, 13.0, 13.0, 0.25, -1.0, 0.0])
        with tempfile.TemporaryDirectory() as tmp:
            out = os.path.join(tmp, "m.bin")
            subprocess.run([os.path.join(REF, "ref_tetmesh"), HORSE] + [repr(float(a)) for a in xf] + [out], check=True)
            d = open(out, "rb").read()
        nv, nt = np.frombuffer(d, "<i4", 2)
        o = 8
        rv = np.frombuffer(d, "<f4", nv * 3, o).reshape(-1, 3); o += nv * 12
        rt = np.frombuffer(d, "<i4", nt * 4, o).reshape(-1, 4); o += nt * 16
        rm = np.frombuffer(d, "<f4", nv, o)
        np.savez_compressed(path, verts=v, tets=t, nodes64=nodes64, xform=xf, ref_verts_xf=rv, ref_tets=rt,
                            ref_masses_xf=rm)
    d = np.load(path)
    return d["verts"], d["tets"]


def _with(scene, **kw):
    for k, v in kw.items():
        setattr(scene, k, v)
    return scene


def run_ref(scene, tmp):
    path_in = os.path.join(tmp, "scene.bin")
    path_out = os.path.join(tmp, "out.bin")
    refio.write_scene(scene, path_in)
    drv = os.path.join(REF, "ref_elastic_h" if scene.variant == scenes.VARIANT_H else "ref_elastic_x")
    env = dict(os.environ)
    if getattr(scene, "winds", None):   # WindForce::project updates v in place inside an OpenMP loop:
        env["OMP_NUM_THREADS"] = "1"     # one thread = its sequential (reproducible) order
    r = subprocess.run([drv, path_in, path_out], cwd=tmp, capture_output=True, text=True, env=env)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    steps = refio.read_ref_result(path_out, scene.n_nodes)
    if scene.variant != scenes.VARIANT_H and scene.accel:
        z_reject_flags(steps, r.stdout)
    return steps


def z_reject_flags(steps, stdout):
    """The z-AA reference (admm_anderson_xzu) writes no reject column to its residual file
    (Solver.hpp:142-144: time, prim, comb), so the driver's flags read 0; it prints each step's
    reject count instead ("reset number = N", Solver.cpp:253). A reject at iteration k happens iff
    the fresh prim exceeds the previous recorded one (Solver.cpp:159); without one the recorded prim
    is that fresh value, so every recorded rise prim_k > prim_{k-1} is a reject. Those flags are
    the reference's flags exactly when their count equals the printed count (then `reject_exact`
    is 1 for the step); otherwise they are a lower bound. Each step also keeps the printed count."""
    counts = [int(ln.split("=")[1]) for ln in stdout.splitlines() if ln.strip().startswith("reset number")]
    for k, st in enumerate(steps):
        p = np.asarray(st["prim"])
        flags = np.zeros(len(p), np.int32)
        flags[1:] = p[1:] > p[:-1]
        st["reject"] = flags
        st["resets"] = counts[k] if k < len(counts) else -1
        st["reject_exact"] = int(st["resets"] == int(flags.sum()))


def element_tables(tmp):
    rng = np.random.default_rng(20191015)
    out = {}
    # tets: F = I + 0.3 N, some inverted (flip a column), some near-singular
    n = 64
    F = np.eye(3)[None] + 0.3 * rng.standard_normal((n, 3, 3))
    F[::5, :, 0] *= -1.0                 # inverted
    F[3::7, :, 2] = F[3::7, :, 1] * 0.5  # rank-deficient
    Fv = np.transpose(F, (0, 2, 1)).reshape(n, 9)  # column-major vec(F)
    for op, name, prm in [(0, "tet_linear", (1e7, 0.399, 1.0, 0.0)), (1, "tet_nh", (1e7, 0.399, 0.1, 0.0)),
                          (2, "tet_stvk", (1e7, 0.399, 0.1, 0.0))]:
        X = Fv if op == 0 else Fv[1::5].copy()   # hyperelastic: skip inverted inputs (log J of J < 0)
        if op != 0:
            X = np.concatenate([np.eye(3).reshape(1, 9) + 0.2 * rng.standard_normal((24, 9))])
            X = X[np.linalg.det(X.reshape(-1, 3, 3)) > 0.2]
        buf = struct.pack("<ii", op, len(X)) + b"".join(struct.pack("<4d", *prm) + x.astype("<f8").tobytes() for x in X)
        out[name] = (X, prm, _run_elem(buf, tmp, 9, len(X)))
    # tris (H prox) with and without strain limits
    T = np.concatenate([np.eye(3)[:, :2].T.reshape(1, 6).repeat(32, 0)]) + 0.3 * rng.standard_normal((32, 6))
    for name, prm in [("tri_h_limits", (50.0, 0.1, 0.95, 1.05)), ("tri_h_free", (50.0, 0.1, -100.0, 100.0))]:
        buf = struct.pack("<ii", 3, len(T)) + b"".join(struct.pack("<4d", *prm) + t.astype("<f8").tobytes() for t in T)
        out[name] = (T, prm, _run_elem(buf, tmp, 6, len(T)))
    # COD solves: SPD, near-singular and rank-deficient normal-equation matrices
    mats = []
    for k in (1, 2, 3, 6, 10):
        for kind in range(3):
            A = rng.standard_normal((40, k))
            if kind == 1 and k > 1:
                A[:, -1] = A[:, 0] + 1e-9 * rng.standard_normal(40)
            if kind == 2 and k > 2:
                A[:, 1] = A[:, 0]
            A /= np.linalg.norm(A, axis=0)
            M = A.T @ A
            b = A.T @ rng.standard_normal(40)
            mats.append((k, M, b))
    res = []
    for k, M, b in mats:
        buf = struct.pack("<ii", 4, 1) + struct.pack("<4d", k, 0, 0, 0) + M.astype("<f8").ravel(order="F").tobytes() + b.astype("<f8").tobytes()
        res.append(_run_elem(buf, tmp, k, 1)[0])
    out["cod"] = mats, res
    return out


def _run_elem(buf, tmp, width, count):
    pin = os.path.join(tmp, "elem.bin")
    pout = os.path.join(tmp, "elem.out")
    with open(pin, "wb") as f:
        f.write(buf)
    r = subprocess.run([os.path.join(REF, "ref_element"), pin, pout], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return np.fromfile(pout, dtype="<f8").reshape(count, width)


def scene_digest(sc):
    """sha256 over the scene arrays: full-size fixtures store outputs only (the scene is
    regenerated by scenes.tet_drop) and this digest proves the regenerated scene is the same."""
    import hashlib
    h = hashlib.sha256()
    for a in [sc.x, sc.masses] + ([sc.rest] if sc.rest is not None else []) + [g.idx for g in sc.groups]:
        h.update(np.ascontiguousarray(a).tobytes())
    return np.frombuffer(h.digest(), np.uint8)


def full_drop40(tmp):
    """The C4 recipe at the CPU-baseline sample size (make_tet_blocks(40,16,20) = 64 000
    NeoHookean tets, z-AA m=6, 3 time steps x 10 iterations -- the scene bench.py times the
    reference on): the reference's per-iteration residuals, and positions / velocities on 512
    sampled nodes plus their column sums per step (the 350 kB state itself is not stored)."""
    sc = scenes.tet_drop(40, 16, 20, iters=10, n_steps=3)
    steps = run_ref(sc, tmp)
    rng = np.random.default_rng(4)
    sample = np.sort(rng.choice(sc.n_nodes, 512, replace=False)).astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "full_drop40_z_nh_aa6.npz"), digest=scene_digest(sc), sample=sample,
                        ref_resets=np.array([s["resets"] for s in steps]),
                        nrec=np.array([len(s["prim"]) for s in steps]),
                        prim=np.concatenate([s["prim"] for s in steps]), comb=np.concatenate([s["comb"] for s in steps]),
                        reject=np.concatenate([s["reject"] for s in steps]),
                        x_sample=np.stack([s["x"][sample] for s in steps]),
                        v_sample=np.stack([s["v"][sample] for s in steps]),
                        x_sum=np.stack([s["x"].sum(0) for s in steps]), v_sum=np.stack([s["v"].sum(0) for s in steps]))
    print("full_drop40_z_nh_aa6", [len(s["prim"]) for s in steps])


def full_bunny40(tmp):
    """The C4 recipe on the voxelised bunny BASELINE configs[3] names, at the golden size
    (scenes.bunny_drop(40) = 64 150 NeoHookean tets, 15 724 nodes on an irregular, boundary-heavy
    mesh; z-AA m=6, 3 time steps x 10 iterations): the reference's per-iteration residuals and
    positions / velocities on 512 sampled nodes plus their column sums per step."""
    sc = scenes.bunny_drop(40, iters=10, n_steps=3)
    steps = run_ref(sc, tmp)
    rng = np.random.default_rng(5)
    sample = np.sort(rng.choice(sc.n_nodes, 512, replace=False)).astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "full_bunny40_z_nh_aa6.npz"), digest=scene_digest(sc), sample=sample,
                        ref_resets=np.array([s["resets"] for s in steps]),
                        nrec=np.array([len(s["prim"]) for s in steps]),
                        prim=np.concatenate([s["prim"] for s in steps]), comb=np.concatenate([s["comb"] for s in steps]),
                        reject=np.concatenate([s["reject"] for s in steps]),
                        x_sample=np.stack([s["x"][sample] for s in steps]),
                        v_sample=np.stack([s["v"][sample] for s in steps]),
                        x_sum=np.stack([s["x"].sum(0) for s in steps]), v_sum=np.stack([s["v"].sum(0) for s in steps]))
    print("full_bunny40_z_nh_aa6", [len(s["prim"]) for s in steps])


def full_c4(tmp):
    """BASELINE configs[3] at full size (make_tet_blocks(100,40,50) = 1 000 000 NeoHookean tets,
    211 191 nodes, z-AA m=6): ONE time step of 10 iterations of the reference itself (its setup
    factors the 633 k-dof system with Eigen's SimplicialLDLT: about three hours here), the
    per-iteration residuals and positions / velocities on 512 sampled nodes plus their column sums."""
    sc = scenes.tet_drop(100, 40, 50, iters=10, n_steps=1)
    steps = run_ref(sc, tmp)
    rng = np.random.default_rng(6)
    sample = np.sort(rng.choice(sc.n_nodes, 512, replace=False)).astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "full_c4_block_z_nh_aa6.npz"), digest=scene_digest(sc), sample=sample,
                        nrec=np.array([len(s["prim"]) for s in steps]),
                        prim=np.concatenate([s["prim"] for s in steps]), comb=np.concatenate([s["comb"] for s in steps]),
                        reject=np.concatenate([s["reject"] for s in steps]),
                        x_sample=np.stack([s["x"][sample] for s in steps]),
                        v_sample=np.stack([s["v"][sample] for s in steps]),
                        x_sum=np.stack([s["x"].sum(0) for s in steps]), v_sum=np.stack([s["v"].sum(0) for s in steps]),
                        step_ms=np.array([s["step_ms"] for s in steps]))
    print("full_c4_block_z_nh_aa6", [len(s["prim"]) for s in steps])


def full_c4_2steps(tmp):
    """full_c4 over TWO time steps of 10 iterations (the second starts from the reference's own
    first-step state: velocity update, pins, the Anderson restart between steps) --
    full_c4_block_z_nh_aa6_2steps.npz. About three hours of the reference's serial setup here."""
    sc = scenes.tet_drop(100, 40, 50, iters=10, n_steps=2)
    steps = run_ref(sc, tmp)
    rng = np.random.default_rng(6)
    sample = np.sort(rng.choice(sc.n_nodes, 512, replace=False)).astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "full_c4_block_z_nh_aa6_2steps.npz"), digest=scene_digest(sc), sample=sample,
                        nrec=np.array([len(s["prim"]) for s in steps]),
                        prim=np.concatenate([s["prim"] for s in steps]), comb=np.concatenate([s["comb"] for s in steps]),
                        reject=np.concatenate([s["reject"] for s in steps]),
                        x_sample=np.stack([s["x"][sample] for s in steps]),
                        v_sample=np.stack([s["v"][sample] for s in steps]),
                        x_sum=np.stack([s["x"].sum(0) for s in steps]), v_sum=np.stack([s["v"].sum(0) for s in steps]),
                        step_ms=np.array([s["step_ms"] for s in steps]))
    print("full_c4_block_z_nh_aa6_2steps", [len(s["prim"]) for s in steps])


def residual_files(tmp):
    """The reference's own Solver::save() output (Solver.hpp:130-155: result/residual-<m>.txt,
    written by every step()) for one (u,x)-variant and one z-variant scene, kept verbatim as data
    (the last step's rows) -- pins the format of Solver.save()."""
    for name, sc, out in (("cant8_ux_lin_aa6", cases()["cant8_ux_lin_aa6"], "ref_residual_h.txt"),
                          ("cloth12_z_noaa", cases()["cloth12_z_noaa"], "ref_residual_x.txt")):
        res = os.path.join(tmp, "result")
        if os.path.isdir(res):
            for f in os.listdir(res):
                os.remove(os.path.join(res, f))
        run_ref(sc, tmp)
        (f,) = os.listdir(res)
        with open(os.path.join(res, f)) as src, open(os.path.join(HERE, out), "w") as dst:
            dst.write("# " + name + " " + f + "\n" + src.read())
        print(out, f)


def main(only=None):
    if only == ["--residual-files"]:
        with tempfile.TemporaryDirectory() as tmp:
            residual_files(tmp)
        return
    if only == ["--full"]:
        with tempfile.TemporaryDirectory() as tmp:
            full_drop40(tmp)
        return
    if only == ["--full-c4-2steps"]:
        with tempfile.TemporaryDirectory() as tmp:
            full_c4_2steps(tmp)
        return
    if only == ["--full-c4"]:
        with tempfile.TemporaryDirectory() as tmp:
            full_c4(tmp)
        return
    if only == ["--bunny"]:
        with tempfile.TemporaryDirectory() as tmp:
            full_bunny40(tmp)
        return
    with tempfile.TemporaryDirectory() as tmp:
        for name, sc in cases().items():
            if only and name not in only:
                continue
            steps = run_ref(sc, tmp)
            save_case(os.path.join(HERE, name + ".npz"), sc, steps)
            print(name, [len(s["prim"]) for s in steps])
        if only:
            return
        et = element_tables(tmp)
        arrays = {}
        for name in ("tet_linear", "tet_nh", "tet_stvk", "tri_h_limits", "tri_h_free"):
            X, prm, Y = et[name]
            arrays[name + "_in"], arrays[name + "_prm"], arrays[name + "_out"] = X, np.array(prm), Y
        mats, res = et["cod"]
        for i, ((k, M, b), th) in enumerate(zip(mats, res)):
            arrays[f"cod{i}_M"], arrays[f"cod{i}_b"], arrays[f"cod{i}_theta"] = M, b, th
        np.savez_compressed(os.path.join(HERE, "elements.npz"), **arrays)
        print("elements", sorted(k for k in arrays if k.endswith("_out")))


if __name__ == "__main__":
    main(sys.argv[1:])   # optional case names: regenerate only those trajectory fixtures
