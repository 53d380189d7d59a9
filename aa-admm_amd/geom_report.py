"""Before/after quality reports of the reference's geometry applications.

A PlanarityOpt / WireMeshOpt caller diffs these files after a run; they are computed on the host
from the input mesh and the solver's solution (`Geom.solution()`), exactly as the applications
do after `solve_ADMM`:

* `planarity_report` -- Geometry/PlanarityOpt.cpp:263-275: `check_planarity_error` (:67-108)
  and `check_ref_surface_distance` (:110-131) before and after, then `save_error` (:39-65):
  result/planarityErrBefore.txt and result/planatityErrAfter.txt (sic, the reference's name);
* `wiremesh_report` -- Geometry/WireMeshOpt.cpp:306-325: `check_wiremesh_error` (:102-157) and
  `check_ref_surface_distance` (:159-182) before and after, then `save_error` (:64-100):
  result/{edge,angle,ref}_wiremeshErr{Before,After}.txt.

Files: one value per line, 16 significant digits (the reference's `setprecision(16)`); the
summary lines go to `out` as the applications print them. Distances to the reference surface are
exact point-triangle distances (igl::AABB::squared_distance in the reference): on the host by
default (k-d tree over triangle centroids, every triangle that can be closer tested exactly), or
through a `closest(P) -> C` callable, e.g. the GPU BVH of a bound solver
(`lambda P: geom.closest_points(0, P)`).
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

from .geom_scenes import average_edge_length, edges_of


# ---- point-triangle distance (host) ---------------------------------------------------------

def closest_on_triangles(P, A, B, C):
    """Closest points of P[i] on triangles (A[i], B[i], C[i]) (Ericson's region test, vectorised)."""
    ab, ac, ap = B - A, C - A, P - A
    d1 = np.einsum("ij,ij->i", ab, ap)
    d2 = np.einsum("ij,ij->i", ac, ap)
    bp = P - B
    d3 = np.einsum("ij,ij->i", ab, bp)
    d4 = np.einsum("ij,ij->i", ac, bp)
    cp = P - C
    d5 = np.einsum("ij,ij->i", ab, cp)
    d6 = np.einsum("ij,ij->i", ac, cp)
    va = d3 * d6 - d5 * d4
    vb = d5 * d2 - d1 * d6
    vc = d1 * d4 - d3 * d2
    out = np.empty_like(P)
    done = np.zeros(len(P), bool)

    def put(mask, val):
        m = mask & ~done
        out[m] = val[m] if val.ndim == 2 else val
        done[m] = True

    put((d1 <= 0) & (d2 <= 0), A)
    put((d3 >= 0) & (d4 <= d3), B)
    with np.errstate(divide="ignore", invalid="ignore"):
        v = d1 / (d1 - d3)
        put((vc <= 0) & (d1 >= 0) & (d3 <= 0), A + v[:, None] * ab)
        put((d6 >= 0) & (d5 <= d6), C)
        w = d2 / (d2 - d6)
        put((vb <= 0) & (d2 >= 0) & (d6 <= 0), A + w[:, None] * ac)
        w = (d4 - d3) / ((d4 - d3) + (d5 - d6))
        put((va <= 0) & ((d4 - d3) >= 0) & ((d5 - d6) >= 0), B + w[:, None] * (C - B))
        den = 1.0 / (va + vb + vc)
        v, w = vb * den, vc * den
        put(np.ones(len(P), bool), A + v[:, None] * ab + w[:, None] * ac)
    return out


def closest_points_host(P, refV, refF, chunk=200_000):
    """Exact closest points of P on the triangle mesh (refV, refF)."""
    from scipy.spatial import cKDTree

    P = np.asarray(P, np.float64)
    refV = np.asarray(refV, np.float64)
    refF = np.asarray(refF, np.int64)
    A, B, C = refV[refF[:, 0]], refV[refF[:, 1]], refV[refF[:, 2]]
    cen = (A + B + C) / 3.0
    rad = np.max(np.stack([np.linalg.norm(A - cen, axis=1), np.linalg.norm(B - cen, axis=1),
                           np.linalg.norm(C - cen, axis=1)]), axis=0)
    R = float(rad.max())
    tree = cKDTree(cen)
    _, t0 = tree.query(P, k=1)
    Q = closest_on_triangles(P, A[t0], B[t0], C[t0])
    best = np.sum((P - Q) ** 2, axis=1)
    # any triangle closer than the first candidate has its centroid within sqrt(best) + R
    cands = tree.query_ball_point(P, np.sqrt(best) + R * (1 + 1e-12) + 1e-300)
    cnt = np.array([len(c) for c in cands])
    pi = np.repeat(np.arange(len(P)), cnt)
    ti = np.concatenate([np.asarray(c, np.int64) for c in cands]) if len(P) else np.zeros(0, np.int64)
    for s in range(0, len(pi), chunk):
        p, t = pi[s:s + chunk], ti[s:s + chunk]
        q = closest_on_triangles(P[p], A[t], B[t], C[t])
        d = np.sum((P[p] - q) ** 2, axis=1)
        order = np.lexsort((d, p))       # per point, the smallest distance first
        p, d, q = p[order], d[order], q[order]
        first = np.ones(len(p), bool)
        first[1:] = p[1:] != p[:-1]
        p, d, q = p[first], d[first], q[first]
        better = d < best[p]
        best[p[better]] = d[better]
        Q[p[better]] = q[better]
    return Q


def ref_surface_distance(V, faces, refV, refF, closest=None, out=None):
    """check_ref_surface_distance (PlanarityOpt.cpp:110-131, WireMeshOpt.cpp:159-182): distance of
    every vertex to the reference surface / the mesh's average edge length."""
    V = np.asarray(V, np.float64)
    C = closest(V) if closest is not None else closest_points_host(V, refV, refF)
    d = np.sqrt(np.sum((V - np.asarray(C, np.float64)) ** 2, axis=1)) / average_edge_length(V, faces)
    if out is not None:
        out.write(f"Reference surface distance (normalized by edge length): Max {_g(d.max())}, Average {_g(d.mean())}\n")
    return d


# ---- per-element errors ---------------------------------------------------------------------

def planarity_errors(V, faces, out=None):
    """check_planarity_error (PlanarityOpt.cpp:67-108): per face, the largest distance of its
    mean-centred vertices from their least-squares plane (normal = the left singular vector of
    the smallest singular value), and for quads the diagonals' distance |n(d1 x d2) . (c1 - c2)|;
    both / the mesh's average edge length. Returns (planarity, diagonal)."""
    V = np.asarray(V, np.float64)
    nf = len(faces)
    plan, diag = np.zeros(nf), np.zeros(nf)
    by_k = {}
    for i, f in enumerate(faces):
        by_k.setdefault(len(f), []).append(i)
    for k, ids in by_k.items():
        ids = np.asarray(ids)
        F = np.asarray([faces[i] for i in ids])
        pts = V[F]                                      # (n, k, 3)
        if k == 4:
            d1, d2 = pts[:, 2] - pts[:, 0], pts[:, 3] - pts[:, 1]
            c1, c2 = (pts[:, 2] + pts[:, 0]) * 0.5, (pts[:, 3] + pts[:, 1]) * 0.5
            n = np.cross(d1, d2)
            nn = np.linalg.norm(n, axis=1)
            n = np.where(nn[:, None] > 0, n / np.where(nn > 0, nn, 1.0)[:, None], n)
            diag[ids] = np.abs(np.einsum("ij,ij->i", n, c1 - c2))
        cen = pts - pts.mean(axis=1, keepdims=True)
        U = np.linalg.svd(np.transpose(cen, (0, 2, 1)), full_matrices=True)[0]   # (n, 3, 3)
        N = U[:, :, 2]
        plan[ids] = np.abs(np.einsum("nj,nkj->nk", N, cen)).max(axis=1)
    el = average_edge_length(V, faces)
    diag /= el
    plan /= el
    if out is not None:
        out.write(f"Diagonal error (normalized by edge length): max {_g(diag.max())}, average {_g(diag.mean())}\n")
        out.write(f"Planarity error (normalized by edge length): max {_g(plan.max())}, average {_g(plan.mean())}\n")
    return plan, diag


def wiremesh_errors(V, faces, target_edge_length, min_angle=math.pi * 0.25, max_angle=math.pi * 0.75, out=None):
    """check_wiremesh_error (WireMeshOpt.cpp:102-157) on a quad mesh. Returns
    (angle_error, edge_error): per face corner |angle - 90| in degrees (4 per face, corner i at
    vertex i between its edges to i+1 and i+3), and per face half-edge the relative length error
    |len - target| / target of its edge, half-edges in OpenMesh's face circulation order (the face's
    half-edge is its last, v3 -> v0, then v0 -> v1, v1 -> v2, v2 -> v3). The printed angle error is
    the violation of [min_angle, max_angle]."""
    V = np.asarray(V, np.float64)
    F = np.asarray(faces, np.int64)
    if F.ndim != 2 or F.shape[1] != 4:
        raise ValueError("wiremesh_errors: quad mesh expected")
    edges, _ = edges_of([list(f) for f in F])
    e = np.asarray(edges, np.int64)
    edge_err = np.abs(np.linalg.norm(V[e[:, 1]] - V[e[:, 0]], axis=1) - target_edge_length) / target_edge_length
    eid = {(min(u, v), max(u, v)): k for k, (u, v) in enumerate(edges)}
    he = np.array([[eid[(min(f[(j + 3) % 4], f[j]), max(f[(j + 3) % 4], f[j]))] for j in range(4)] for f in F.tolist()],
                  np.int64).reshape(-1, 4)
    edge_error = edge_err[he].ravel()

    def unit(x):
        n = np.linalg.norm(x, axis=-1, keepdims=True)
        return np.where(n > 0, x / np.where(n > 0, n, 1.0), x)

    P = V[F]                                             # (nf, 4, 3)
    e1 = unit(np.roll(P, -1, axis=1) - P)                # to corner i + 1
    e2 = unit(np.roll(P, 1, axis=1) - P)                 # to corner i + 3
    with np.errstate(invalid="ignore"):
        ang = np.arccos(np.einsum("fij,fij->fi", e1, e2))
    angle_error = (np.abs(ang - 0.5 * math.pi) * (180.0 / math.pi)).ravel()
    viol = np.where(ang < min_angle, min_angle - ang, np.where(ang >= max_angle, ang - max_angle, 0.0))
    viol = viol.ravel() * (180.0 / math.pi)
    if out is not None:
        out.write(f"Normalized edge length error: max {_g(edge_err.max())},  average {_g(edge_err.mean())}\n")
        out.write(f"Angle error: max {_g(viol.max())},  average {_g(viol.mean())}\n")
    return angle_error, edge_error


# ---- the applications' reports ----------------------------------------------------------------

def save_error(path_before, path_after, before, after):
    """save_error: one value per line, setprecision(16)."""
    for path, v in ((path_before, before), (path_after, after)):
        with open(path, "w") as f:
            f.write("".join(f"{x:.16g}\n" for x in np.asarray(v, np.float64)))


def planarity_report(V_before, V_after, faces, refV, refF, result_dir="./result", closest=None, out=sys.stdout):
    """PlanarityOpt.cpp:263-275 after a solve: prints the reports, writes
    result/planarityErrBefore.txt and result/planatityErrAfter.txt. Returns the arrays."""
    os.makedirs(result_dir, exist_ok=True)
    out.write("Before optimization:\n")
    p0, d0 = planarity_errors(V_before, faces, out)
    r0 = ref_surface_distance(V_before, faces, refV, refF, closest, out)
    out.write("After optimization:\n")
    p1, d1 = planarity_errors(V_after, faces, out)
    r1 = ref_surface_distance(V_after, faces, refV, refF, closest, out)
    save_error(os.path.join(result_dir, "planarityErrBefore.txt"), os.path.join(result_dir, "planatityErrAfter.txt"),
               p0, p1)
    return {"planarity": (p0, p1), "diagonal": (d0, d1), "ref_distance": (r0, r1)}


def wiremesh_report(V_before, V_after, faces, refV, refF, target_edge_length, min_angle=math.pi * 0.25,
                    max_angle=math.pi * 0.75, result_dir="./result", closest=None, out=sys.stdout):
    """WireMeshOpt.cpp:306-325 after a solve (faces: the subdivided quad mesh the solver ran on):
    prints the reports, writes result/{edge,angle,ref}_wiremeshErr{Before,After}.txt."""
    os.makedirs(result_dir, exist_ok=True)
    out.write("Before optimization:\n")
    a0, e0 = wiremesh_errors(V_before, faces, target_edge_length, min_angle, max_angle, out)
    r0 = ref_surface_distance(V_before, faces, refV, refF, closest, out)
    out.write("After optimization:\n")
    a1, e1 = wiremesh_errors(V_after, faces, target_edge_length, min_angle, max_angle, out)
    r1 = ref_surface_distance(V_after, faces, refV, refF, closest, out)
    for tag, b, a in (("edge", e0, e1), ("angle", a0, a1), ("ref", r0, r1)):
        save_error(os.path.join(result_dir, f"{tag}_wiremeshErrBefore.txt"),
                   os.path.join(result_dir, f"{tag}_wiremeshErrAfter.txt"), b, a)
    return {"angle": (a0, a1), "edge": (e0, e1), "ref_distance": (r0, r1)}


def _g(x):
    """std::cout's default formatting of a double (precision 6, %g)."""
    return f"{x:g}"
