"""Scene-binding parity: the TetGen ele/node loader and binding::add_tetmesh's
float32 transform and lumped masses against the reference's own mcl code run on the plinko
samples' mesh (oracle/_ref/ref_tetmesh -> tests/golden/mesh_horse759.npz, made by
tests/golden/make_golden.py). CPU only."""
import os

import numpy as np

from golden_io import GOLDEN, scenes


def _write_elenode(base, nodes64, tets, one_based=False):
    off = 1 if one_based else 0
    with open(base + ".node", "w") as f:
        f.write(f"{len(nodes64)}  3  0  0\n")
        for i, p in enumerate(nodes64):
            f.write(f"{i + off} {float(p[0])!r} {float(p[1])!r} {float(p[2])!r}\n")
        f.write("# generated\n")
    with open(base + ".ele", "w") as f:
        f.write(f"{len(tets)}  4  0\n")
        for i, t in enumerate(tets):
            f.write(f"{i + off} {t[0] + off} {t[1] + off} {t[2] + off} {t[3] + off}\n")


def test_elenode_binding_matches_reference(tmp_path):
    d = np.load(os.path.join(GOLDEN, "mesh_horse759.npz"))
    for one_based in (False, True):
        base = str(tmp_path / ("m1" if one_based else "m0"))
        _write_elenode(base, d["nodes64"], d["tets"], one_based)
        v, t = scenes.load_elenode(base)
        assert v.dtype == np.float32 and np.array_equal(t, d["ref_tets"])
        xf = d["xform"]
        vx = scenes.xform_scale_trans(v, xf[:3], xf[3:])
        assert np.array_equal(vx, d["ref_verts_xf"])                               # apply_xform, float32
        assert np.array_equal(scenes.tetmesh_masses32(vx, t), d["ref_masses_xf"])  # weighted_masses(1522)


def test_elenode_rejects_bad_indices(tmp_path):
    base = str(tmp_path / "bad")
    _write_elenode(base, np.zeros((4, 3)), np.array([[0, 1, 2, 3]]))
    with open(base + ".ele", "w") as f:
        f.write("2 4 0\n0 0 1 2 3\n0 0 1 2 3\n")   # record 1 never set
    try:
        scenes.load_elenode(base)
    except ValueError as e:
        assert "indices are bad" in str(e)
    else:
        raise AssertionError("bad .ele accepted")


def test_plinko_scene_uses_the_binding():
    d = np.load(os.path.join(GOLDEN, "mesh_horse759.npz"))
    sc = scenes.plinko_hit(d["verts"], d["tets"], squash=1.0)
    assert np.array_equal(sc.x, d["ref_verts_xf"].astype(np.float64))
    assert np.array_equal(sc.masses, d["ref_masses_xf"].astype(np.float64))
    assert sc.variant == scenes.VARIANT_H and len(sc.collision_idx) == sc.n_nodes
