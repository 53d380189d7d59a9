"""Golden-fixture (de)serialisation: scene arrays + reference outputs as .npz (data only)."""
from __future__ import annotations

import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
scenes = importlib.import_module("aa-admm_amd.scenes")
GOLDEN = os.path.join(REPO, "tests", "golden")


def save_case(path, sc, steps):
    d = dict(
        x=sc.x, masses=sc.masses, pin_idx=sc.pin_idx, pin_pts=sc.pin_pts, pin_vel=sc.pin_vel,
        g_kind=np.array([g.kind for g in sc.groups]), g_mat=np.array([g.material for g in sc.groups]),
        g_E=np.array([g.E for g in sc.groups]), g_nu=np.array([g.nu for g in sc.groups]),
        g_lmin=np.array([g.limit_min for g in sc.groups]), g_lmax=np.array([g.limit_max for g in sc.groups]),
        settings=np.array([sc.variant, sc.dt, sc.gravity, sc.penalty, sc.iters, sc.accel, sc.aa_m, sc.n_steps]),
        nrec=np.array([len(s["prim"]) for s in steps]),
        prim=np.concatenate([s["prim"] for s in steps]), comb=np.concatenate([s["comb"] for s in steps]),
        reject=np.concatenate([s["reject"] for s in steps]),
        xs=np.stack([s["x"] for s in steps]), vs=np.stack([s["v"] for s in steps]),
    )
    for i, g in enumerate(sc.groups):
        d[f"g{i}_idx"] = g.idx
    np.savez_compressed(path, **d)


def load_case(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    st = d["settings"]
    groups = [scenes.ElementGroup(int(d["g_kind"][i]), int(d["g_mat"][i]), float(d["g_E"][i]), float(d["g_nu"][i]),
                                  d[f"g{i}_idx"].astype(np.int32), float(d["g_lmin"][i]), float(d["g_lmax"][i]))
              for i in range(len(d["g_kind"]))]
    sc = scenes.Scene(x=d["x"], masses=d["masses"], groups=groups, pin_idx=d["pin_idx"].astype(np.int32),
                      pin_pts=d["pin_pts"], pin_vel=d["pin_vel"], variant=int(st[0]), dt=float(st[1]),
                      gravity=float(st[2]), penalty=float(st[3]), iters=int(st[4]), accel=int(st[5]),
                      aa_m=int(st[6]), n_steps=int(st[7]), name=name)
    steps, o = [], 0
    for k, n in enumerate(d["nrec"]):
        steps.append(dict(prim=d["prim"][o:o + n], comb=d["comb"][o:o + n], reject=d["reject"][o:o + n],
                          x=d["xs"][k], v=d["vs"][k]))
        o += n
    return sc, steps


def case_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f != "elements.npz")


def compare(ref_steps, got_steps, tol_comb, tol_x, n_check=None):
    """Per-iteration residual parity judged relative to comb_0 / prim_0 of each time step
    (SURVEY.md §8c, Appendix B.12), plus final positions. Returns a list of failures."""
    fails = []
    for k, (r, g) in enumerate(zip(ref_steps, got_steps)):
        n = min(len(r["comb"]), len(g["comb"]))
        if n_check is not None:
            n = min(n, n_check)
        if n == 0:
            continue
        c0, p0 = r["comb"][0], r["prim"][0]
        dc = np.max(np.abs(r["comb"][:n] - g["comb"][:n])) / c0
        dp = np.max(np.abs(r["prim"][:n] - g["prim"][:n])) / p0
        if not (dc <= tol_comb and dp <= tol_comb * 10):
            fails.append(f"step {k}: comb dev {dc:.3e} prim dev {dp:.3e} (tol {tol_comb:g})")
        nr = min(n, 20)
        if np.any(r["reject"][:nr] != g["reject"][:nr]):
            fails.append(f"step {k}: reject flags differ in the first {nr} iterations")
    xr, xg = ref_steps[-1]["x"], got_steps[-1]["x"]
    dx = np.linalg.norm(xr - xg) / np.linalg.norm(xr)
    if not dx <= tol_x:
        fails.append(f"final x rel err {dx:.3e} (tol {tol_x:g})")
    return fails
