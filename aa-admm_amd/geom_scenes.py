"""Headless scene builders for the Geometry (ALM) hot path (host side, numpy).

A `GeomScene` holds exactly what the reference's `ALMGeometrySolver<3>` is fed with
(Geometry/ALMGeometrySolver.h:81-320): hard and soft `Constraint<3>` objects
(Geometry/Constraint.h), linear regularisation rows (Geometry/LinearRegularization.h:47-87),
reference surfaces, the penalty and the Anderson window. Constraints of one kind are kept as
homogeneous groups (same type / index count / weight / hard-soft), which is also how the C ABI
(`include/aa_admm.h`, `aa_geom_add_constraints`) and the device kernels batch them.

Builders (the callers SURVEY.md §8f item 2 asks to reproduce headlessly):

* `planarity_from_mesh` -- the constraint recipe of `optimize_mesh` in
  Geometry/PlanarityOpt.cpp:134-246 (soft PointToRefSurface per vertex, relative uniform
  Laplacians with the interior-valence-4 split and the boundary rule, hard PlaneConstraint
  per face with more than 3 vertices), applied to any polygon mesh;
* `pq_heightfield` -- configs[2]: a quad grid on z = 0.15 sin(2 pi x) cos(2 pi y) whose
  reference surface is the same field triangulated at twice the resolution;
* `wire_from_mesh` / `wire_grid` -- the recipe of Geometry/WireMeshOpt.cpp:233-289 (one soft
  ReferenceSurfceConstraint over all points, 4 AngleConstraints per quad, one
  EdgeLengthConstraint per edge) -- configs[4] uses a sheared height-field quad grid;
* `read_obj` -- minimal OBJ reader (v / f records) for the reference's own data files.
"""
from __future__ import annotations

import dataclasses
import math
from typing import List, Optional

import numpy as np

# constraint types (Geometry/Constraint.h)
PLANE, ANGLE, EDGE, CLOSENESS, POINT_TO_REF, REF_SURFACE = 0, 1, 2, 3, 4, 5
TYPE_NAMES = {PLANE: "plane", ANGLE: "angle", EDGE: "edge", CLOSENESS: "closeness",
              POINT_TO_REF: "point_to_ref", REF_SURFACE: "ref_surface"}
N_PARAMS = {PLANE: 0, ANGLE: 2, EDGE: 1, CLOSENESS: 3, POINT_TO_REF: 1, REF_SURFACE: 1}
# regularisation row kinds (LinearRegularization.h)
REG_LAPLACIAN, REG_RELATIVE, REG_CLOSENESS = 0, 1, 2


@dataclasses.dataclass
class ConstraintGroup:
    type: int
    idx: np.ndarray            # (count, k) int32 point indices (idI_)
    weight: float              # constructor weight (weight_ = sqrt(weight))
    hard: bool
    params: Optional[np.ndarray] = None   # (count, N_PARAMS[type]) fp64
    # params: EDGE target length; ANGLE (min_radian, max_radian); CLOSENESS target xyz;
    #         POINT_TO_REF / REF_SURFACE reference-surface id (stored as a double)

    @property
    def count(self) -> int:
        return int(self.idx.shape[0])

    @property
    def k(self) -> int:
        return int(self.idx.shape[1])


@dataclasses.dataclass
class GeomScene:
    x0: np.ndarray                                  # (n, 3) initial points (solve_ADMM init_x)
    groups: List[ConstraintGroup]
    reg_kind: np.ndarray                            # (r,) int32
    reg_ptr: np.ndarray                             # (r+1,) int32 into reg_idx / reg_coef
    reg_idx: np.ndarray                             # int32
    reg_coef: np.ndarray                            # fp64 raw coefficients (before sqrt(weight))
    reg_weight: np.ndarray                          # (r,) fp64
    reg_target: np.ndarray                          # (r, 3) closeness targets (unused otherwise)
    ref_points: np.ndarray                          # (n, 3) points the relative Laplacians refer to
    surfaces: List[tuple]                           # [(V (nv,3) fp64, F (nf,3) int32)]
    penalty: float = 1e5
    iters: int = 100
    aa_m: int = 10
    name: str = "geom"
    solver: str = "alm"                             # "alm": ALMGeometrySolver<3>; "plain": GeometrySolver<3>

    @property
    def n_points(self) -> int:
        return int(self.x0.shape[0])

    def hard_cols(self) -> int:
        return int(sum(g.count * cols_per(g.type, g.k) for g in self.groups if g.hard))

    def avg_edge_length(self) -> float:
        return float(self.__dict__.get("_avg_edge", 0.0))


def cols_per(ctype: int, k: int) -> int:
    """num_transformed_points (Constraint.h:168-174): SUBTRACT_FIRST drops one column."""
    return k - 1 if ctype in (ANGLE, EDGE) else k


class RegBuilder:
    """Collects LinearRegularization rows (add_uniform_laplacian / add_laplacian /
    add_relative_* / add_closeness, Geometry/LinearRegularization.h:47-87)."""

    def __init__(self):
        self.kind, self.idx, self.coef, self.weight, self.target = [], [], [], [], []

    def _add(self, kind, idx, coefs, weight, target=(0.0, 0.0, 0.0)):
        assert len(idx) == len(coefs)
        self.kind.append(kind); self.idx.append(list(idx)); self.coef.append(list(coefs))
        self.weight.append(float(weight)); self.target.append(list(target))

    def uniform_laplacian(self, idx, weight, relative=False):
        n = len(idx)
        coefs = [1.0] + [-1.0 / float(n - 1)] * (n - 1)
        self._add(REG_RELATIVE if relative else REG_LAPLACIAN, idx, coefs, weight)

    def laplacian(self, idx, coefs, weight, relative=False):
        self._add(REG_RELATIVE if relative else REG_LAPLACIAN, idx, coefs, weight)

    def closeness(self, i, weight, target):
        self._add(REG_CLOSENESS, [i], [1.0], weight, target)

    def arrays(self):
        r = len(self.kind)
        ptr = np.zeros(r + 1, np.int32)
        for i, l in enumerate(self.idx):
            ptr[i + 1] = ptr[i] + len(l)
        flat = lambda ll, dt: np.array([v for l in ll for v in l], dtype=dt)
        return dict(reg_kind=np.array(self.kind, np.int32), reg_ptr=ptr, reg_idx=flat(self.idx, np.int32),
                    reg_coef=flat(self.coef, np.float64), reg_weight=np.array(self.weight, np.float64),
                    reg_target=np.array(self.target, np.float64).reshape(r, 3))


# ----------------------------------------------------------------------------------------
# mesh helpers
# ----------------------------------------------------------------------------------------

def read_obj(path, float32=True):
    """Vertices (n,3) fp64 and faces (list of int lists, 0-based) of an OBJ file.

    float32=True rounds coordinates through fp32 like OpenMesh's OBJ reader, which parses
    `v` records into `float` (Geometry/external/OpenMesh/Core/IO/reader/OBJReader.cc:294,334):
    the reference applications see exactly these positions."""
    V, F = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                V.append([float(t) for t in line.split()[1:4]])
            elif line.startswith("f "):
                F.append([int(t.split("/")[0]) - 1 for t in line.split()[1:]])
    V = np.array(V, np.float64)
    if float32:
        V = V.astype(np.float32).astype(np.float64)
    return V, F


def edges_of(faces):
    """Unique undirected edges in first-seen half-edge order, plus per-edge face lists."""
    eid, edges, efaces = {}, [], []
    for fi, f in enumerate(faces):
        for a in range(len(f)):
            u, v = f[a], f[(a + 1) % len(f)]
            key = (min(u, v), max(u, v))
            if key not in eid:
                eid[key] = len(edges); edges.append((u, v)); efaces.append([])
            efaces[eid[key]].append(fi)
    return edges, efaces


def average_edge_length(V, faces):
    """average_edge_length (Geometry/MeshTypes.h:143-156): mean over the unique edges."""
    edges, _ = edges_of(faces)
    e = np.array(edges)
    return float(np.linalg.norm(V[e[:, 0]] - V[e[:, 1]], axis=1).mean())


def one_rings(n, faces):
    """Cyclic one-ring of every interior manifold vertex (neighbours in circulation order)
    and the boundary neighbours of boundary vertices with the faces of those boundary edges."""
    nxt = [dict() for _ in range(n)]   # v -> {prev_nb: next_nb} per incident face
    for f in faces:
        k = len(f)
        for a in range(k):
            v = f[a]
            nxt[v][f[(a - 1) % k]] = f[(a + 1) % k]
    edges, efaces = edges_of(faces)
    bnd_nbs = [[] for _ in range(n)]
    for (u, v), fl in zip(edges, efaces):
        if len(fl) == 1:
            bnd_nbs[u].append((v, fl[0]))
            bnd_nbs[v].append((u, fl[0]))
    rings = [None] * n
    for v in range(n):
        if bnd_nbs[v] or not nxt[v]:
            continue
        start = next(iter(nxt[v]))
        ring, cur = [start], nxt[v][start]
        while cur != start and len(ring) <= len(nxt[v]):
            ring.append(cur)
            cur = nxt[v].get(cur, start)
        rings[v] = ring
    return rings, bnd_nbs


def _surface_field(x, y, amp=0.15):
    return amp * np.sin(2 * np.pi * x) * np.cos(2 * np.pi * y)


def quad_grid(nx, ny, shear=0.0, amp=0.15):
    """(nx+1)(ny+1) points on the height field over [0,1]^2 (optionally sheared in-plane) and
    nx*ny counter-clockwise quads."""
    u, v = np.meshgrid(np.linspace(0, 1, nx + 1), np.linspace(0, 1, ny + 1), indexing="ij")
    u, v = u.ravel(), v.ravel()
    x = u + shear * np.sin(np.pi * v) * v
    y = v
    P = np.stack([x, y, _surface_field(x, y, amp)], 1)
    node = lambda i, j: i * (ny + 1) + j
    I, J = np.meshgrid(np.arange(nx), np.arange(ny), indexing="ij")
    I, J = I.ravel(), J.ravel()
    Q = np.stack([node(I, J), node(I + 1, J), node(I + 1, J + 1), node(I, J + 1)], 1).astype(np.int32)
    return P, Q


def field_trimesh(nx, ny, shear=0.0, amp=0.15, x_range=None):
    """Triangulated height field (2 triangles per cell) -- the reference surface."""
    P, Q = quad_grid(nx, ny, shear, amp)
    T = np.concatenate([Q[:, [0, 1, 2]], Q[:, [0, 2, 3]]], 0).astype(np.int32)
    return P, T


# ----------------------------------------------------------------------------------------
# recipes
# ----------------------------------------------------------------------------------------

def planarity_from_mesh(V, faces, refV, refF, *, iters=100, aa_m=10, penalty=1e5, closeness_weight=1.0,
                        laplacian_weight=0.0, relative_laplacian_weight=0.1, name="pq") -> GeomScene:
    """optimize_mesh of Geometry/PlanarityOpt.cpp:134-246 (defaults: main() :322-325)."""
    n = len(V)
    groups: List[ConstraintGroup] = []
    if closeness_weight > 0:
        groups.append(ConstraintGroup(POINT_TO_REF, np.arange(n, dtype=np.int32)[:, None], closeness_weight, False,
                                      np.zeros((n, 1))))
    reg = RegBuilder()
    rings, bnd = one_rings(n, faces)
    if laplacian_weight > 0 or relative_laplacian_weight > 0:
        for v in range(n):
            if not bnd[v]:
                ring = rings[v]
                if ring is None:
                    continue
                vhs = [v] + ring
                rows = [[vhs[0], vhs[1], vhs[3]], [vhs[0], vhs[2], vhs[4]]] if len(vhs) == 5 else [vhs]
                for r in rows:
                    if relative_laplacian_weight > 0:
                        reg.uniform_laplacian(r, relative_laplacian_weight, relative=True)
                    if laplacian_weight > 0:
                        reg.uniform_laplacian(r, laplacian_weight)
            else:
                nbs = bnd[v]
                if len(nbs) == 2 and nbs[0][1] != nbs[1][1]:
                    r = [v, nbs[0][0], nbs[1][0]]
                    if relative_laplacian_weight > 0:
                        reg.uniform_laplacian(r, relative_laplacian_weight, relative=True)
                    if laplacian_weight > 0:
                        reg.uniform_laplacian(r, laplacian_weight)
    by_k = {}
    for f in faces:
        if len(f) > 3:
            by_k.setdefault(len(f), []).append(f)
    for k in sorted(by_k):
        groups.append(ConstraintGroup(PLANE, np.array(by_k[k], np.int32), 1.0, True))
    sc = GeomScene(x0=np.asarray(V, np.float64).copy(), groups=groups, ref_points=np.asarray(V, np.float64).copy(),
                   surfaces=[(np.asarray(refV, np.float64), np.asarray(refF, np.int32))], penalty=penalty,
                   iters=iters, aa_m=aa_m, name=name, **reg.arrays())
    sc._avg_edge = average_edge_length(V, faces)
    return sc


def pq_heightfield(nx=317, ny=317, *, iters=100, aa_m=10, ref_factor=2, noise=0.0, **kw) -> GeomScene:
    """configs[2]: planar-quad optimisation of a (nx x ny)-quad height-field grid (100 489
    faces at 317 x 317), reference surface = the same field triangulated at `ref_factor`x.
    noise > 0 displaces the initial points off the surface by noise * edge length (seeded,
    deterministic) -- a scanned-surface start, so that closeness and planarity both act."""
    V, Q = quad_grid(nx, ny)
    if noise > 0:
        rng = np.random.default_rng(20191015)
        V = V + (noise / max(nx, ny)) * rng.standard_normal(V.shape)
    RV, RF = field_trimesh(ref_factor * nx, ref_factor * ny)
    return planarity_from_mesh(V, [list(q) for q in Q], RV, RF, iters=iters, aa_m=aa_m,
                               name=f"pq{nx}x{ny}", **kw)


def wire_from_mesh(V, faces, refV, refF, edge_length, *, iters=100, aa_m=20, penalty=1000.0,
                   min_angle=math.pi * 0.25, max_angle=math.pi * 0.75, closeness_weight=1.0,
                   name="wire") -> GeomScene:
    """optimize_mesh of Geometry/WireMeshOpt.cpp:233-289 (laplacian_weight = -1 as in main)."""
    n = len(V)
    groups: List[ConstraintGroup] = []
    if closeness_weight > 0:
        groups.append(ConstraintGroup(REF_SURFACE, np.arange(n, dtype=np.int32)[:, None], closeness_weight, False,
                                      np.zeros((n, 1))))
    ang = []
    for f in faces:
        assert len(f) == 4, "WireMeshOpt expects a quad mesh"
        for i in range(4):
            ang.append([f[i], f[(i + 1) % 4], f[(i + 3) % 4]])
    groups.append(ConstraintGroup(ANGLE, np.array(ang, np.int32), 1.0, True,
                                  np.tile([min_angle, max_angle], (len(ang), 1)).astype(np.float64)))
    edges, _ = edges_of(faces)
    groups.append(ConstraintGroup(EDGE, np.array(edges, np.int32), 1.0, True,
                                  np.full((len(edges), 1), float(edge_length))))
    reg = RegBuilder()
    sc = GeomScene(x0=np.asarray(V, np.float64).copy(), groups=groups, ref_points=np.asarray(V, np.float64).copy(),
                   surfaces=[(np.asarray(refV, np.float64), np.asarray(refF, np.int32))], penalty=penalty,
                   iters=iters, aa_m=aa_m, name=name, **reg.arrays())
    sc._avg_edge = average_edge_length(V, faces)
    return sc


def subdivide_and_smooth(V, faces):
    """subdivide_and_smooth_mesh (Geometry/MeshTypes.h:214-342), the pre-processing of
    WireMeshOpt's main (WireMeshOpt.cpp:364): one subdivision step and a Laplacian smoothing.

    Topology (OpenMesh's add_face order): the output vertices are the input vertices, then one
    midpoint (p_from + p_to) * 0.5 per edge in edge-creation order, then one centroid per face
    (sum of its vertices in face order / n). Face i of the input (v_0..v_{n-1}) yields n quads
    [e(v_{j-1}, v_j), v_j, e(v_j, v_{j+1}), centroid] -- OpenMesh's face half-edge is the last
    one, (v_{n-1}, v_0), so its circulation starts at v_0.
    Smoothing: a uniform Laplacian row for every interior vertex (all neighbours) and for every
    boundary vertex whose two boundary edges belong to different faces (its two boundary
    neighbours); the input vertices are fixed and the others minimise |L x|^2 (the reference
    solves (A^T A) x_free = -(A^T L) x_fixed with A = L restricted to the free columns, by
    SimplicialLDLT -- a sparse direct solve here). Returns (V_out, faces_out)."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla

    V = np.asarray(V, np.float64)
    nv = len(V)
    edges, _ = edges_of(faces)
    eid = {(min(u, v), max(u, v)): k for k, (u, v) in enumerate(edges)}
    ne = len(edges)
    out = [V]
    e = np.array(edges, np.int64).reshape(-1, 2)
    out.append((V[e[:, 0]] + V[e[:, 1]]) * 0.5)
    cents, newf = [], []
    for fi, f in enumerate(faces):
        c = np.zeros(3)
        for v in f:
            c = c + V[v]
        cents.append(c / float(len(f)))
        fv = nv + ne + fi
        n = len(f)
        for j in range(n):
            a, b, cc = f[j - 1], f[j], f[(j + 1) % n]
            newf.append([nv + eid[(min(a, b), max(a, b))], b, nv + eid[(min(b, cc), max(b, cc))], fv])
    X = np.vstack(out + [np.array(cents).reshape(-1, 3)])
    n_out = len(X)
    # Laplacian rows (MeshTypes.h:264-296)
    edges2, efaces2 = edges_of(newf)
    nbrs = [set() for _ in range(n_out)]
    bnd = [[] for _ in range(n_out)]   # (neighbour, face) per boundary edge
    for (u, v), fl in zip(edges2, efaces2):
        nbrs[u].add(v); nbrs[v].add(u)
        if len(fl) == 1:
            bnd[u].append((v, fl[0])); bnd[v].append((u, fl[0]))
    rows, cols, vals = [], [], []
    r = 0
    for v in range(n_out):
        if bnd[v]:
            if len(bnd[v]) == 2 and bnd[v][0][1] != bnd[v][1][1]:
                lap = [v] + [w for w, _ in bnd[v]]
            else:
                continue
        else:
            lap = [v] + sorted(nbrs[v])
        k = len(lap)
        rows += [r] * k; cols += lap; vals += [1.0] + [-1.0 / float(k - 1)] * (k - 1)
        r += 1
    L = sp.csr_matrix((vals, (rows, cols)), shape=(r, n_out))
    fixed = np.zeros((n_out, 3))
    fixed[:nv] = V
    free = np.arange(nv, n_out)
    A = L[:, free]
    M = (A.T @ A).tocsc()
    rhs = -(A.T @ L) @ fixed
    sol = np.column_stack([spla.spsolve(M, rhs[:, d]) for d in range(3)]) if len(free) else np.zeros((0, 3))
    X = fixed.copy()
    X[free] = sol
    return X, newf


def wire_from_polymesh(V, faces, refV, refF, **kw) -> GeomScene:
    """WireMeshOpt's main (Geometry/WireMeshOpt.cpp:341-391) from a polygon mesh: target edge
    length = half the input's average edge length, the mesh subdivided and smoothed
    (subdivide_and_smooth), then the optimize_mesh recipe (wire_from_mesh)."""
    L = 0.5 * average_edge_length(np.asarray(V, np.float64), faces)
    SV, SF = subdivide_and_smooth(V, faces)
    return wire_from_mesh(SV, SF, refV, refF, L, **kw)


def wire_grid(nx=707, ny=707, *, iters=100, aa_m=20, shear=1.2, ref_factor=2, **kw) -> GeomScene:
    """configs[4]: wire-mesh optimisation of a sheared height-field quad grid (501 264 points
    at 707 x 707). The in-plane shear drives corner angles below 45 degrees over part of the
    grid so the angle constraints are active; the edge target is the mean edge length."""
    V, Q = quad_grid(nx, ny, shear=shear)
    RV, RF = field_trimesh(ref_factor * nx, ref_factor * ny, shear=shear)
    faces = [list(q) for q in Q]
    L = average_edge_length(V, faces)
    return wire_from_mesh(V, faces, RV, RF, L, iters=iters, aa_m=aa_m, name=f"wire{nx}x{ny}", **kw)


# ----------------------------------------------------------------------------------------
# reference-driver I/O (test infrastructure; oracle/ref_drivers/ref_geom_driver.cpp)
# ----------------------------------------------------------------------------------------
