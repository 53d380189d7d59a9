"""Headless scene builders for the admm-elastic hot path (host side, numpy).

These replace the reference's GUI sample glue that *feeds* `admm::Solver`
(SURVEY.md §8f item 2):

* `tri_blocks(nx, ny)`  -- the mesh of mclscene `factory::make_tri_blocks`
  (admm_anderson_hard_zxu/deps/mclscene/include/MCL/ShapeFactory.hpp:499-548): unit
  squares with a centre vertex, 4 triangles per square [(d,a,e),(a,b,e),(b,c,e),(c,d,e)].
  Vertices are indexed directly on the structured grid (corners first, then centres)
  instead of through mclscene's O(T*n) `refine()` merge -- the connectivity is the same,
  only the vertex numbering differs.
* `tet_blocks(cx, cy, cz)` -- `factory::make_tet_blocks` (ShapeFactory.hpp:436-496), five
  tets per unit cube with the reference's corner labelling (a..h) and tet table.
* lumped masses as `TriangleMesh::weighted_masses` (TriangleMesh.hpp:281-296) and
  `TetMesh::weighted_masses` (TetMesh.hpp:297-315), bound per node x3 like
  `binding::add_trimesh/add_tetmesh` (samples/utils/AddMeshes.hpp:97-235).
* pin rules of the samples: windyflag `get_pins` (two corners of the min-x edge,
  samples/Asia2019/windyflag.cpp:29-61) and the cantilever "x = min face" rule.

A `Scene` is a plain container of fp64/int32 arrays -- exactly what the C ABI
(`include/aa_admm.h`) takes -- plus the solver settings of the reference's
`Solver::Settings` (Solver.hpp:45-67). `oracle/refio.write_scene` serialises it for the reference
driver under oracle/ (test infrastructure only).
"""
from __future__ import annotations

import dataclasses
import os
from typing import List, Optional

import numpy as np

TET, TRI = 0, 1
# passive obstacles (PassiveObject.hpp:32-136; include/aa_admm.h AA_OBS_*)
OBS_FLOOR, OBS_SLIDE_FLOOR, OBS_SPHERE, OBS_PLANE_HALF_SPHERE, OBS_CYLINDER = 0, 1, 2, 3, 4
LINEAR, NEOHOOKEAN, STVK = 0, 1, 2
VARIANT_X, VARIANT_H = 0, 1  # admm_anderson_xzu (z-AA) / admm_anderson_hard_zxu ((u,x)-AA)


def lame(E: float, nu: float):
    """mu, lambda, bulk modulus k = lambda + 2/3 mu (EnergyTerm.hpp:35-61)."""
    mu = E / (2.0 * (1.0 + nu))
    lam = E * nu / ((1.0 + nu) * (1.0 - 2.0 * nu))
    return mu, lam, lam + (2.0 / 3.0) * mu


@dataclasses.dataclass
class ElementGroup:
    kind: int             # TET or TRI
    material: int         # LINEAR / NEOHOOKEAN / STVK (tets); LINEAR for tris
    E: float
    nu: float
    idx: np.ndarray       # int32 (count, 4) or (count, 3)
    limit_min: float = -100.0   # Lame defaults (EnergyTerm.hpp:54-55)
    limit_max: float = 100.0


@dataclasses.dataclass
class Scene:
    x: np.ndarray                 # (n, 3) fp64 rest/initial positions
    masses: np.ndarray            # (n,) fp64 lumped node masses
    groups: List[ElementGroup]
    pin_idx: np.ndarray           # (p,) int32
    pin_pts: np.ndarray           # (p, 3) fp64 pin targets for the first step
    pin_vel: np.ndarray           # (p, 3) fp64 pin displacement per time step
    variant: int = VARIANT_H
    dt: float = 1.0 / 30.0
    gravity: float = -9.8
    penalty: float = 1.0
    iters: int = 100
    accel: int = 1
    aa_m: int = 6
    n_steps: int = 1
    name: str = "scene"
    rest: Optional[np.ndarray] = None   # (n, 3) rest positions of the elements; None = x
    # (u,x) variant extras (admm_anderson_hard_zxu): passive obstacles [(type, params)] and the
    # collision-checked nodes (Solver::add_obstacle / set_collisions), and WindForces
    # [(tris (t, 3) int32, direction (3,))] (Solver::ext_forces)
    obstacles: list = dataclasses.field(default_factory=list)
    collision_idx: Optional[np.ndarray] = None
    winds: list = dataclasses.field(default_factory=list)

    @property
    def rest_x(self) -> np.ndarray:
        return self.x if self.rest is None else self.rest

    @property
    def n_nodes(self) -> int:
        return int(self.x.shape[0])

    def n_elements(self) -> int:
        return int(sum(len(g.idx) for g in self.groups))


# ----------------------------------------------------------------------------------------
# mesh generators
# ----------------------------------------------------------------------------------------

def tri_blocks(nx: int, ny: int):
    """Vertices (n,3) and triangles (4*nx*ny, 3) of make_tri_blocks(nx, ny)."""
    nx, ny = max(1, nx), max(1, ny)
    gx, gy = np.meshgrid(np.arange(nx + 1, dtype=np.float64), np.arange(ny + 1, dtype=np.float64), indexing="ij")
    corners = np.stack([gx.ravel(), gy.ravel(), np.zeros(gx.size)], axis=1)
    cx, cy = np.meshgrid(np.arange(nx, dtype=np.float64) + 0.5, np.arange(ny, dtype=np.float64) + 0.5, indexing="ij")
    centres = np.stack([cx.ravel(), cy.ravel(), np.zeros(cx.size)], axis=1)
    verts = np.concatenate([corners, centres], axis=0)
    ix, iy = np.meshgrid(np.arange(nx), np.arange(ny), indexing="ij")
    ix, iy = ix.ravel(), iy.ravel()          # cell order x-major, y-minor as in the reference loops
    corner = lambda i, j: i * (ny + 1) + j
    a = corner(ix, iy)
    b = corner(ix + 1, iy)
    c = corner(ix + 1, iy + 1)
    d = corner(ix, iy + 1)
    e = (nx + 1) * (ny + 1) + ix * ny + iy
    tris = np.stack([np.stack([d, a, e], 1), np.stack([a, b, e], 1),
                     np.stack([b, c, e], 1), np.stack([c, d, e], 1)], axis=1).reshape(-1, 3)
    return verts, tris.astype(np.int32)


def tet_blocks(cx: int, cy: int, cz: int):
    """Vertices (n,3) and tets (5*cx*cy*cz, 4) of make_tet_blocks(cx, cy, cz)."""
    cx, cy, cz = max(1, cx), max(1, cy), max(1, cz)
    g = np.stack(np.meshgrid(np.arange(cx + 1), np.arange(cy + 1), np.arange(cz + 1), indexing="ij"), -1)
    verts = g.reshape(-1, 3).astype(np.float64)
    node = lambda i, j, k: (i * (cy + 1) + j) * (cz + 1) + k
    X, Y, Z = np.meshgrid(np.arange(cx), np.arange(cy), np.arange(cz), indexing="ij")
    X, Y, Z = X.ravel(), Y.ravel(), Z.ravel()
    a = node(X + 1, Y + 1, Z + 1)
    b = node(X, Y + 1, Z + 1)
    c = node(X, Y + 1, Z)
    d = node(X + 1, Y + 1, Z)
    e = node(X + 1, Y, Z + 1)
    f = node(X, Y, Z + 1)
    gg = node(X, Y, Z)
    h = node(X + 1, Y, Z)
    lab = [a, b, c, d, e, f, gg, h]
    table = [(0, 5, 7, 4), (5, 7, 2, 0), (5, 0, 2, 1), (7, 2, 0, 3), (5, 2, 7, 6)]
    tets = np.stack([np.stack([lab[t[0]], lab[t[1]], lab[t[2]], lab[t[3]]], 1) for t in table], 1).reshape(-1, 4)
    return verts, tets.astype(np.int32)


def tet_voxels(occ):
    """make_tet_blocks' 5 tets (same table, same corner labels) for every occupied cell of a
    boolean grid occ[x, y, z]; vertices = the lattice nodes the cells use (lattice units),
    numbered in lattice order. Cells in x-major, then y, then z order as in tet_blocks."""
    cx, cy, cz = occ.shape
    X, Y, Z = (a.astype(np.int64) for a in np.nonzero(occ))   # x-major order
    node = lambda i, j, k: (i * (cy + 1) + j) * (cz + 1) + k
    lab = [node(X + 1, Y + 1, Z + 1), node(X, Y + 1, Z + 1), node(X, Y + 1, Z), node(X + 1, Y + 1, Z),
           node(X + 1, Y, Z + 1), node(X, Y, Z + 1), node(X, Y, Z), node(X + 1, Y, Z)]
    table = [(0, 5, 7, 4), (5, 7, 2, 0), (5, 0, 2, 1), (7, 2, 0, 3), (5, 2, 7, 6)]
    tets = np.stack([np.stack([lab[t[0]], lab[t[1]], lab[t[2]], lab[t[3]]], 1) for t in table], 1).reshape(-1, 4)
    used = np.unique(tets)
    remap = np.full((cx + 1) * (cy + 1) * (cz + 1), -1, np.int64)
    remap[used] = np.arange(len(used))
    i, r = np.divmod(used, (cy + 1) * (cz + 1))
    j, k = np.divmod(r, cz + 1)
    verts = np.stack([i, j, k], 1).astype(np.float64)
    return verts, remap[tets].astype(np.int32)


def load_voxels(name):
    """Occupancy grid committed under aa-admm_amd/data (tools/make_bunny_voxels.py)."""
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", name + ".npz"))
    dims = tuple(int(a) for a in d["dims"])
    return np.unpackbits(d["bits"])[:int(np.prod(dims))].reshape(dims).astype(bool)


def tri_masses(verts, tris, density=1.0):
    e1 = verts[tris[:, 1]] - verts[tris[:, 0]]
    e2 = verts[tris[:, 2]] - verts[tris[:, 0]]
    area = 0.5 * np.linalg.norm(np.cross(e1, e2), axis=1)
    m = np.zeros(len(verts))
    for k in range(3):
        np.add.at(m, tris[:, k], density * area / 3.0)
    return m


def tet_masses(verts, tets, density=1522.0):
    B = np.stack([verts[tets[:, k]] - verts[tets[:, 0]] for k in (1, 2, 3)], axis=2)
    vol = np.abs(np.linalg.det(B)) / 6.0
    m = np.zeros(len(verts))
    for k in range(4):
        np.add.at(m, tets[:, k], density * vol / 4.0)
    return m


# ----------------------------------------------------------------------------------------
# the BASELINE.json scenes
# ----------------------------------------------------------------------------------------

def cloth(nx: int = 112, ny: int = 112, size: float = 2.0, *, variant=VARIANT_H, aa_m=6, iters=100,
          n_steps=1, accel=1) -> Scene:
    """C2: cloth drop (`make_tri_blocks(112,112)` scaled to `size` m, 50 176 tris).

    Material Lame(50, 0.1) with strain limits [0.95, 1.05] and area density 1 as the
    windyflag sample (windyflag.cpp:84-87, AddMeshes.hpp:203); two corners of the min-x
    edge pinned in place (windyflag.cpp:29-61,101); wind omitted (out of scope).
    """
    v, t = tri_blocks(nx, ny)
    v = v * (size / max(nx, ny))
    m = tri_masses(v, t, 1.0)
    xmin = v[:, 0].min() + 1e-3 * size / max(nx, ny)
    cand = np.nonzero(v[:, 0] <= xmin)[0]
    up = cand[np.argmin(v[cand, 1])]
    down = cand[np.argmax(v[cand, 1])]
    pins = np.array([up, down], dtype=np.int32)
    return Scene(x=v, masses=m, groups=[ElementGroup(TRI, LINEAR, 50.0, 0.1, t, 0.95, 1.05)],
                 pin_idx=pins, pin_pts=v[pins].copy(), pin_vel=np.zeros((2, 3)), variant=variant,
                 iters=iters, aa_m=aa_m, n_steps=n_steps, accel=accel, name=f"cloth{nx}x{ny}")


def cantilever(cx=20, cy=4, cz=5, material=NEOHOOKEAN, *, variant=VARIANT_X, aa_m=6, iters=50,
               n_steps=1, accel=1, E=1e7, nu=0.399) -> Scene:
    """C1: single cantilever `make_tet_blocks(20,4,5)` scaled 1/cy, x = 0 face pinned."""
    v, t = tet_blocks(cx, cy, cz)
    v = v / float(cy)
    m = tet_masses(v, t, 1522.0)
    pins = np.nonzero(v[:, 0] < v[:, 0].min() + 1e-3)[0].astype(np.int32)
    return Scene(x=v, masses=m, groups=[ElementGroup(TET, material, E, nu, t)],
                 pin_idx=pins, pin_pts=v[pins].copy(), pin_vel=np.zeros((len(pins), 3)), variant=variant,
                 iters=iters, aa_m=aa_m, n_steps=n_steps, accel=accel, name=f"cantilever{cx}x{cy}x{cz}")


def tet_drop(cx=100, cy=40, cz=50, material=NEOHOOKEAN, *, squash=0.9, variant=VARIANT_X, aa_m=6, iters=100,
             n_steps=1, accel=1, E=1e7, nu=0.399) -> Scene:
    """C4: elastic block free fall, `make_tet_blocks(cx, cy, cz)` (5 tets per cube; 100x40x50 =
    1 000 000 tets, 211 191 nodes) scaled by 1/cy, density 1522, NeoHookean Lame(1e7, 0.399).
    No pins, no collisions; the initial pose is the rest shape squashed to `squash` in y so that
    the elastic prox has work (a rigid free fall converges trivially) -- SURVEY.md §8d C4.
    The z-AA (X) order, as BASELINE.json asks (the (u,x) order goes NaN on large-deformation
    NeoHookean scenes)."""
    v, t = tet_blocks(cx, cy, cz)
    v = v / float(cy)
    m = tet_masses(v, t, 1522.0)
    x = v.copy()
    c = 0.5 * (v[:, 1].min() + v[:, 1].max())
    x[:, 1] = c + squash * (v[:, 1] - c)
    return Scene(x=x, masses=m, groups=[ElementGroup(TET, material, E, nu, t)], pin_idx=np.zeros(0, np.int32),
                 pin_pts=np.zeros((0, 3)), pin_vel=np.zeros((0, 3)), variant=variant, iters=iters, aa_m=aa_m,
                 n_steps=n_steps, accel=accel, name=f"drop{cx}x{cy}x{cz}", rest=v)


def bunny_drop(res=100, material=NEOHOOKEAN, *, cell=1.0 / 40.0, squash=0.9, variant=VARIANT_X, aa_m=6, iters=100,
               n_steps=1, accel=1, E=1e7, nu=0.399) -> Scene:
    """C4 on the mesh BASELINE configs[3] names: the reference's closed bunny
    (deps/mclscene/src/data/bunny_closed.obj) voxelised into `res` cells along its longest side
    (aa-admm_amd/data/bunny_vox<res>.npz; res 100 = 200 556 cells = 1 002 780 tets), 5
    make_tet_blocks tets per cell of size `cell` (the C4 block's 1/40 m), then the tet_drop
    recipe: NeoHookean Lame(1e7, 0.399), density 1522, free fall from the rest shape squashed to
    `squash` in y, z-AA (X order). An irregular, boundary-heavy mesh beside the regular block."""
    v, t = tet_voxels(load_voxels(f"bunny_vox{res}"))
    v = v * cell
    m = tet_masses(v, t, 1522.0)
    x = v.copy()
    c = 0.5 * (v[:, 1].min() + v[:, 1].max())
    x[:, 1] = c + squash * (v[:, 1] - c)
    return Scene(x=x, masses=m, groups=[ElementGroup(TET, material, E, nu, t)], pin_idx=np.zeros(0, np.int32),
                 pin_pts=np.zeros((0, 3)), pin_vel=np.zeros((0, 3)), variant=variant, iters=iters, aa_m=aa_m,
                 n_steps=n_steps, accel=accel, name=f"bunny{res}", rest=v)


def beams(dim=3, *, variant=VARIANT_X, aa_m=6, iters=100, n_steps=1, accel=1, materials=(LINEAR, NEOHOOKEAN, STVK)) -> Scene:
    """C1 beams: three make_tet_blocks(4*dim, dim, dim) beams, 1 m tall, at y = +1.75 / 0 / -1.75,
    Lame(1e7, 0.399), x-extreme faces pinned and pulled apart by dt per step
    (samples/Asia2019/beams.cpp:94-167 and its stretch_beams callback)."""
    xs, groups, pins, pts, vel = [], [], [], [], []
    off = 0
    dt = 1.0 / 30.0
    for i, mat in enumerate(materials):
        v, t = tet_blocks(4 * dim, dim, dim)
        lo, hi = v.min(0), v.max(0)
        v = (v - 0.5 * (lo + hi)) / (hi[1] - lo[1])
        v[:, 1] += (1.75, 0.0, -1.75)[i % 3]
        bl, bh = v[:, 0].min() + 1e-2, v[:, 0].max() - 1e-2
        for j in range(len(v)):
            if v[j, 0] < bl:
                pins.append(off + j); pts.append(v[j] - [dt, 0, 0]); vel.append([-dt, 0, 0])
            if v[j, 0] > bh:
                pins.append(off + j); pts.append(v[j] + [dt, 0, 0]); vel.append([dt, 0, 0])
        groups.append(ElementGroup(TET, mat, 1e7, 0.399, t + off))
        xs.append(v)
        off += len(v)
    x = np.concatenate(xs)
    m = np.concatenate([tet_masses(xs[i], groups[i].idx - sum(len(xx) for xx in xs[:i])) for i in range(len(xs))])
    return Scene(x=x, masses=m, groups=groups, pin_idx=np.array(pins, np.int32), pin_pts=np.array(pts),
                 pin_vel=np.array(vel), variant=variant, iters=iters, aa_m=aa_m, n_steps=n_steps, accel=accel,
                 name=f"beams{dim}")


# ----------------------------------------------------------------------------------------
# tet-mesh files and the sample binding (f2)
# ----------------------------------------------------------------------------------------

def load_elenode(path: str):
    """mcl::meshio::load_elenode (deps/mclscene/include/MCL/MeshIO.hpp:180-290): `path`.ele and
    `path`.node (TetGen format); 1-based files are detected from the first record's index, as the
    reference does. Vertices come back as float32 (mcl::TetMesh stores Vec3f), tets as int32."""
    def records(fname):
        with open(fname) as f:
            lines = [ln.split("#", 1)[0].split() for ln in f]
        lines = [ln for ln in lines if ln]
        return int(lines[0][0]), lines[1:]
    n_tets, rows = records(path + ".ele")
    tets = np.zeros((n_tets, 4), np.int32)
    seen = np.zeros(n_tets, bool)
    one = False
    for i, r in enumerate(rows[:n_tets]):
        idx, ids = int(r[0]), [int(v) for v in r[1:5]]
        if i == 0 and idx == 1:
            one = True
        if one:
            idx -= 1
            ids = [v - 1 for v in ids]
        if idx >= n_tets:
            raise ValueError("**TetMesh Error: Your indices are bad for file " + path + ".ele")
        tets[idx] = ids
        seen[idx] = True
    if not seen.all():
        raise ValueError("**TetMesh Error: Your indices are bad for file " + path + ".ele")
    n_nodes, rows = records(path + ".node")
    verts = np.zeros((n_nodes, 3), np.float32)
    seen = np.zeros(n_nodes, bool)
    one = False
    for i, r in enumerate(rows[:n_nodes]):
        idx = int(r[0])
        if i == 0 and idx == 1:
            one = True
        if one:
            idx -= 1
        if idx >= n_nodes:
            raise ValueError("**TetMesh Error: Your indices are bad for file " + path + ".node")
        verts[idx] = np.array([float(r[1]), float(r[2]), float(r[3])], np.float64).astype(np.float32)
        seen[idx] = True
    if not seen.all():
        raise ValueError("**TetMesh Error: Your indices are bad for file " + path + ".node")
    return verts, tets


def xform_scale_trans(verts32: np.ndarray, scale, trans) -> np.ndarray:
    """mesh->apply_xform(make_trans(t) * make_scale(s)) in float32 (mcl::XForm<float>): v' = s v + t."""
    s = np.asarray(scale, np.float32).reshape(1, 3)
    t = np.asarray(trans, np.float32).reshape(1, 3)
    return (verts32.astype(np.float32) * s + t).astype(np.float32)


def tetmesh_masses32(verts32: np.ndarray, tets: np.ndarray, density: float = 1522.0) -> np.ndarray:
    """TetMesh::weighted_masses (TetMesh.hpp:297-315) in float32, tets in order: |det(E)/6| * density / 4
    added to each corner, det of the edge matrix by Eigen's 3x3 cofactor expansion."""
    v = verts32.astype(np.float32)
    m = np.zeros(len(v), np.float32)
    dens = np.float32(density)
    six, four = np.float32(6.0), np.float32(4.0)
    e1 = v[tets[:, 1]] - v[tets[:, 0]]
    e2 = v[tets[:, 2]] - v[tets[:, 0]]
    e3 = v[tets[:, 3]] - v[tets[:, 0]]
    # columns are the edges: m(r, c) = e_c[r]
    m00, m10, m20 = e1[:, 0], e1[:, 1], e1[:, 2]
    m01, m11, m21 = e2[:, 0], e2[:, 1], e2[:, 2]
    m02, m12, m22 = e3[:, 0], e3[:, 1], e3[:, 2]
    # Eigen determinant_impl<3>: first-row expansion (Eigen/src/LU/Determinant.h)
    det = (m00 * (m11 * m22 - m12 * m21) - m01 * (m10 * m22 - m12 * m20)) + m02 * (m10 * m21 - m11 * m20)
    tm = (dens * np.abs(det / six)).astype(np.float32) / four
    for t in range(len(tets)):          # float accumulation in tet order
        for a in range(4):
            m[tets[t, a]] = np.float32(m[tets[t, a]] + tm[t])
    return m


def tetmesh_scene(verts32, tets, material=LINEAR, E=1e7, nu=0.499, **kw) -> Scene:
    """binding::add_tetmesh (samples/utils/AddMeshes.hpp:97-178) for one mesh: positions and the
    element rest shape are the float32 vertices (create_tets_from_mesh<float, ...>), masses
    TetMesh::weighted_masses(1522) per node x3 (zero mass throws, as the binding does)."""
    m = tetmesh_masses32(verts32, tets)
    if np.any(m <= 0):
        raise ValueError("TetMesh Error: Zero mass")
    x = verts32.astype(np.float64)
    return Scene(x=x, masses=m.astype(np.float64), groups=[ElementGroup(TET, material, E, nu, np.asarray(tets, np.int32))],
                 pin_idx=np.zeros(0, np.int32), pin_pts=np.zeros((0, 3)), pin_vel=np.zeros((0, 3)), **kw)


# ----------------------------------------------------------------------------------------
# collision / wind scenes of the (u,x) variant (samples/Asia2019/plinko*.cpp, windyflag.cpp)
# ----------------------------------------------------------------------------------------

def plinko_hit(verts32, tets, *, y0=-1.0, iters=13, accel=0, aa_m=2, n_steps=20, dt=1.0 / 30.0, squash=0.95) -> Scene:
    """plinkohit.cpp:39-103: a linear-rubber tet mesh (Lame::rubber, `binding::LINEAR`) scaled by 13
    and moved to (0.25, y0, 0), dropped on PlaneAndHalfSphere(center (0,-3,0), radius 1) with every
    node collision-checked; admm_iters 13 and the other Solver::Settings defaults (dt 1/30, no
    acceleration, m = 2). y0 = 2.5 in the sample; lower here so contact starts within a few steps.
    The initial pose is the rest shape squashed to `squash` in y (rest kept for the elements), so
    the residuals carry signal before the first contact (an unstressed free fall is all rounding
    noise, which Anderson mixing then amplifies differently from run to run of any two codes)."""
    v = xform_scale_trans(verts32, (13.0, 13.0, 13.0), (0.25, y0, 0.0))
    sc = tetmesh_scene(v, tets, LINEAR, 10000000.0, 0.499, variant=VARIANT_H, iters=iters, accel=accel, aa_m=aa_m,
                       n_steps=n_steps, dt=dt, name="plinkohit")
    _squash(sc, squash)
    sc.obstacles = [(OBS_PLANE_HALF_SPHERE, (0.0, float(np.float32(-3.0)), 0.0, float(np.float32(1.0))))]
    sc.collision_idx = np.arange(sc.n_nodes, dtype=np.int32)
    return sc


def obstacle_course(verts32, tets, *, iters=15, accel=1, aa_m=5, n_steps=18, dt=1.0 / 30.0, squash=0.95) -> Scene:
    """Every PassiveObject.hpp shape at once under a falling rubber mesh (plinkopony.cpp:54-117
    uses Cylinder and SlideFloor, plinkohit PlaneAndHalfSphere): a sphere and two z-axis cylinders
    the mesh hits first, then a tilted SlideFloor, a Floor and a PlaneAndHalfSphere below."""
    v = xform_scale_trans(verts32, (13.0, 13.0, 13.0), (0.0, 0.2, 0.0))
    sc = tetmesh_scene(v, tets, LINEAR, 10000000.0, 0.499, variant=VARIANT_H, iters=iters, accel=accel, aa_m=aa_m,
                       n_steps=n_steps, dt=dt, name="obstacles")
    _squash(sc, squash)
    sc.obstacles = [
        (OBS_SPHERE, (0.3, -1.2, 0.1, 0.45)),
        (OBS_CYLINDER, (-0.6, -1.0, 0.0, 0.3)),
        (OBS_CYLINDER, (0.9, -1.4, 0.0, 0.25)),
        (OBS_SLIDE_FLOOR, (0.0, -2.0, 0.0, 0.5, 3.0 ** 0.5 / 2.0, 0.0)),
        (OBS_FLOOR, (-2.3,)),
        (OBS_PLANE_HALF_SPHERE, (0.2, -2.6, 0.0, 0.8)),
    ]
    sc.collision_idx = np.arange(sc.n_nodes, dtype=np.int32)
    return sc


def _squash(sc: Scene, f: float) -> None:
    """initial pose = rest squashed by f in y about its centre (tet_drop's recipe); rest unchanged"""
    if f == 1.0:
        return
    sc.rest = sc.x.copy()
    c = 0.5 * (sc.x[:, 1].min() + sc.x[:, 1].max())
    sc.x = sc.x.copy()
    sc.x[:, 1] = c + f * (sc.x[:, 1] - c)


def windy_cloth(nx=12, ny=12, *, iters=30, aa_m=6, accel=1, n_steps=3, direction=(25.0, 0.0, 5.0)) -> Scene:
    """windyflag.cpp:63-127 headless: the C2 cloth (two pinned corners) with a WindForce on all of
    its faces, direction = orig_wind (10, 0, 2) * 2.5."""
    sc = cloth(nx, ny, iters=iters, n_steps=n_steps, aa_m=aa_m, accel=accel)
    sc.winds = [(np.asarray(sc.groups[0].idx, np.int32), np.asarray(direction, np.float64))]
    sc.name = f"windycloth{nx}x{ny}"
    return sc
