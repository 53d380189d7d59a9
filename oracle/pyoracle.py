"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker. The product path (aa-admm_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import refio  # noqa: E402  (same directory; test infrastructure)

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class Settings(C.Structure):
    _fields_ = [("variant", C.c_int), ("dt", C.c_double), ("gravity", C.c_double), ("penalty", C.c_double),
                ("iters", C.c_int), ("accel", C.c_int), ("aa_m", C.c_int)]


def build():
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        _LIB = C.CDLL(path)
    return _LIB


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


def run_elastic(scene, n_steps=None, cap=None):
    """Runs the oracle on a scenes.Scene; returns per-step dicts like scenes.read_ref_result."""
    L = lib()
    n_steps = scene.n_steps if n_steps is None else n_steps
    cap = scene.iters if cap is None else cap
    groups = scene.groups
    kind = np.array([g.kind for g in groups], np.int32)
    mat = np.array([g.material for g in groups], np.int32)
    E = np.array([g.E for g in groups], np.float64)
    nu = np.array([g.nu for g in groups], np.float64)
    lmin = np.array([g.limit_min for g in groups], np.float64)
    lmax = np.array([g.limit_max for g in groups], np.float64)
    cnt = np.array([len(g.idx) for g in groups], np.int32)
    idx = np.concatenate([np.ascontiguousarray(g.idx, np.int32).ravel() for g in groups]).astype(np.int32)
    off = np.zeros(len(groups), np.int32)
    acc = 0
    for i, g in enumerate(groups):
        off[i] = acc
        acc += g.idx.size
    x = np.ascontiguousarray(scene.x, np.float64)
    rest = None if getattr(scene, "rest", None) is None else np.ascontiguousarray(scene.rest, np.float64)
    m = np.ascontiguousarray(scene.masses, np.float64)
    pins = np.ascontiguousarray(scene.pin_idx, np.int32)
    pts = np.ascontiguousarray(scene.pin_pts, np.float64)
    vel = np.ascontiguousarray(scene.pin_vel, np.float64)
    st = Settings(scene.variant, scene.dt, scene.gravity, scene.penalty, scene.iters, scene.accel, scene.aa_m)
    nrec = np.zeros(n_steps, np.int32)
    prim = np.zeros(n_steps * cap)
    comb = np.zeros(n_steps * cap)
    rej = np.zeros(n_steps * cap, np.int32)
    ox = np.zeros_like(x)
    ov = np.zeros_like(x)
    ms = np.zeros(n_steps)
    err = C.create_string_buffer(512)
    rc = L.oracle_elastic_run(
        C.c_int(scene.n_nodes), _p(x, C.c_double), None if rest is None else _p(rest, C.c_double), _p(m, C.c_double), C.c_int(len(groups)), _p(kind, C.c_int),
        _p(mat, C.c_int), _p(E, C.c_double), _p(nu, C.c_double), _p(lmin, C.c_double), _p(lmax, C.c_double),
        _p(cnt, C.c_int), _p(off, C.c_int), _p(idx, C.c_int), C.c_int(len(pins)), _p(pins, C.c_int),
        _p(pts, C.c_double), _p(vel, C.c_double), C.byref(st), C.c_int(n_steps), C.c_int(cap), _p(nrec, C.c_int),
        _p(prim, C.c_double), _p(comb, C.c_double), _p(rej, C.c_int), _p(ox, C.c_double), _p(ov, C.c_double),
        _p(ms, C.c_double), err, C.c_int(512))
    if rc != 0:
        raise RuntimeError("oracle: " + err.value.decode())
    steps = []
    for k in range(n_steps):
        n = min(int(nrec[k]), cap)
        sl = slice(k * cap, k * cap + n)
        steps.append(dict(prim=prim[sl].copy(), comb=comb[sl].copy(), reject=rej[sl].copy(), step_ms=float(ms[k])))
    steps[-1]["x"] = ox
    steps[-1]["v"] = ov
    return steps


def _vec(fn, *args):
    return fn(*args)


def tri_prox(z6, lmin=-100.0, lmax=100.0, variant=1):
    L = lib()
    z = np.ascontiguousarray(z6, np.float64)
    out = np.zeros(6)
    f = L.oracle_tri_prox_h if variant == 1 else L.oracle_tri_prox_x
    f(_p(z, C.c_double), C.c_double(lmin), C.c_double(lmax), _p(out, C.c_double))
    return out


def tet_prox_linear(z9):
    L = lib()
    z = np.ascontiguousarray(z9, np.float64)
    out = np.zeros(9)
    L.oracle_tet_prox_linear(_p(z, C.c_double), _p(out, C.c_double))
    return out


def tet_prox_hyper(material, mu, lam, k, vol, v9):
    L = lib()
    v = np.ascontiguousarray(v9, np.float64)
    out = np.zeros(9)
    it = L.oracle_tet_prox_hyper(C.c_int(material), C.c_double(mu), C.c_double(lam), C.c_double(k), C.c_double(vol),
                                 _p(v, C.c_double), _p(out, C.c_double))
    return out, it


def svd3(F9):
    L = lib()
    F = np.ascontiguousarray(F9, np.float64)
    U, S, V = np.zeros(9), np.zeros(3), np.zeros(9)
    L.oracle_svd3(_p(F, C.c_double), _p(U, C.c_double), _p(S, C.c_double), _p(V, C.c_double))
    return U.reshape(3, 3).T, S, V.reshape(3, 3).T


def cod_solve(M, b):
    L = lib()
    Mc = np.asfortranarray(M, np.float64).ravel(order="F").copy()
    bb = np.ascontiguousarray(b, np.float64)
    th = np.zeros(len(bb))
    L.oracle_cod_solve(C.c_int(len(bb)), _p(Mc, C.c_double), _p(bb, C.c_double), _p(th, C.c_double))
    return th


def run_geom(scene):
    """Runs the oracle's ALM (or, scene.solver == "plain", GeometrySolver) restatement on a geom_scenes.GeomScene; dict like read_geom_result
    (`faces_added` carries the number of x-updates, i.e. accepted + rejected iterations)."""
    import importlib
    import sys
    import tempfile
    sys.path.insert(0, os.path.dirname(HERE))
    gs = importlib.import_module("aa-admm_amd.geom_scenes")
    L = lib()
    with tempfile.TemporaryDirectory() as tmp:
        sp, op = os.path.join(tmp, "s.bin"), os.path.join(tmp, "o.bin")
        refio.write_geom_scene(scene, sp)
        err = C.create_string_buffer(512)
        rc = L.oracle_geom_run_file_mode(sp.encode(), op.encode(), C.c_int(1 if scene.solver == "plain" else 0), err,
                                         C.c_int(512))
        if rc != 0:
            raise RuntimeError("oracle: " + err.value.decode())
        res = refio.read_geom_result(op, scene.n_points)
    res["x_updates"] = res.pop("faces_added")
    return res


def closest_point(V, F, P):
    L = lib()
    V = np.ascontiguousarray(V, np.float64)
    F = np.ascontiguousarray(F, np.int32)
    P = np.ascontiguousarray(P, np.float64)
    out = np.zeros_like(P)
    L.oracle_closest_point(_p(V, C.c_double), C.c_int(len(V)), _p(F, C.c_int), C.c_int(len(F)), _p(P, C.c_double),
                           C.c_int(len(P)), _p(out, C.c_double))
    return out


def geom_project(ctype, k, params, pts):
    """Constraint projection of transformed points pts (cols x 3)."""
    L = lib()
    prm = np.zeros(3)
    if params is not None:
        prm[:len(np.atleast_1d(params))] = np.atleast_1d(params)
    inp = np.ascontiguousarray(pts, np.float64)
    out = np.zeros_like(inp)
    L.oracle_geom_project(C.c_int(ctype), C.c_int(k), _p(prm, C.c_double), _p(inp, C.c_double), _p(out, C.c_double))
    return out
