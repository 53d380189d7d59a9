#!/usr/bin/env python3
"""Voxelise the reference's closed bunny (deps/mclscene/src/data/bunny_closed.obj, the mesh
BASELINE configs[3] names; container only -- the reference is not on the GPU box) into an
occupancy grid committed as data: aa-admm_amd/data/bunny_vox<N>.npz (cells whose centre is inside
the surface, by ray parity along z). scenes.bunny_drop builds 5 make_tet_blocks tets per
occupied cell from it (SURVEY.md §8d allows a voxelised bunny for C4).

    python tools/make_bunny_voxels.py 96 40     # longest bounding-box side in cells (one file each)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = "/root/reference/admm_anderson_xzu/deps/mclscene/src/data/bunny_closed.obj"


def load_obj(path):
    V, F = [], []
    for line in open(path):
        t = line.split()
        if not t:
            continue
        if t[0] == "v":
            V.append([float(a) for a in t[1:4]])
        elif t[0] == "f":
            F.append([int(a.split("/")[0]) - 1 for a in t[1:4]])
    return np.array(V), np.array(F, np.int64)


def voxelise(V, F, n):
    lo, hi = V.min(0), V.max(0)
    h = (hi - lo).max() / n
    dims = np.ceil((hi - lo) / h).astype(int) + 2            # one empty layer of cells around
    org = lo - h * (dims * h - (hi - lo)) / (2 * h)          # centred
    xs = org[0] + h * (np.arange(dims[0]) + 0.5)
    ys = org[1] + h * (np.arange(dims[1]) + 0.5)
    zs = org[2] + h * (np.arange(dims[2]) + 0.5)
    occ = np.zeros(dims, bool)
    A, B, C = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    # crossings of the vertical line (x, y) with every triangle: barycentric test in xy
    for i, x in enumerate(xs):
        # triangles whose x-range contains x
        sel = (np.minimum(np.minimum(A[:, 0], B[:, 0]), C[:, 0]) <= x) & (np.maximum(np.maximum(A[:, 0], B[:, 0]), C[:, 0]) >= x)
        a, b, c = A[sel], B[sel], C[sel]
        for j, y in enumerate(ys):
            d = (b[:, 1] - c[:, 1]) * (a[:, 0] - c[:, 0]) + (c[:, 0] - b[:, 0]) * (a[:, 1] - c[:, 1])
            ok = np.abs(d) > 1e-300
            l1 = ((b[:, 1] - c[:, 1]) * (x - c[:, 0]) + (c[:, 0] - b[:, 0]) * (y - c[:, 1])) / np.where(ok, d, 1)
            l2 = ((c[:, 1] - a[:, 1]) * (x - c[:, 0]) + (a[:, 0] - c[:, 0]) * (y - c[:, 1])) / np.where(ok, d, 1)
            l3 = 1 - l1 - l2
            hit = ok & (l1 >= 0) & (l2 >= 0) & (l3 >= 0)
            if not hit.any():
                continue
            zc = np.sort(l1[hit] * a[hit, 2] + l2[hit] * b[hit, 2] + l3[hit] * c[hit, 2])
            zc = zc[np.concatenate([[True], np.diff(zc) > 1e-12])]   # a crossing on a shared edge counts once
            inside = (np.searchsorted(zc, zs) % 2) == 1
            occ[i, j, :] = inside
    return occ, h, org


def main():
    V, F = load_obj(OBJ)
    for a in sys.argv[1:] or ["96", "40"]:
        n = int(a)
        occ, h, org = voxelise(V, F, n)
        out = os.path.join(REPO, "aa-admm_amd", "data", f"bunny_vox{n}.npz")
        np.savez_compressed(out, bits=np.packbits(occ.ravel()), dims=np.array(occ.shape), h=np.array(h), origin=org,
                            source=np.array("bunny_closed.obj (deps/mclscene/src/data), ray-parity voxelisation "
                                            "by tools/make_bunny_voxels.py"))
        print(f"{out}: grid {occ.shape}, {int(occ.sum())} occupied cells -> {5 * int(occ.sum())} tets, "
              f"{os.path.getsize(out)} bytes")


if __name__ == "__main__":
    main()
