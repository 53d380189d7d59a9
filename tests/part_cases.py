"""Scenes of the partitioned-solver GPU tests: (builder, tolerance relative to comb_0 / |x|).
Closed-form element paths 1e-9, L-BFGS (NeoHookean) paths 1e-6 -- the same bars as the
single-GPU parity tests; the partitioned run only reorders floating-point sums."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
scenes = importlib.import_module("aa-admm_amd.scenes")
geom_scenes = importlib.import_module("aa-admm_amd.geom_scenes")

CASES = {
    # (u,x)-AA cloth with two pinned corners (C2 recipe, 3 200 tris)
    "cloth_ux": (lambda: scenes.cloth(40, 40, iters=60, n_steps=3), 1e-9),
    # (u,x)-AA linear cantilever, x=0 face pinned
    "cant_ux": (lambda: scenes.cantilever(12, 3, 3, scenes.LINEAR, iters=40, n_steps=2,
                                          variant=scenes.VARIANT_H), 1e-9),
    # z-AA NeoHookean block drop (C4 recipe, 1 440 tets), no pins
    "drop_z": (lambda: scenes.tet_drop(12, 4, 6, iters=40, n_steps=2), 1e-6),
    # z-AA beams with moving pins (C1 recipe)
    "beams_z": (lambda: scenes.beams(3, iters=50, n_steps=2, variant=scenes.VARIANT_X), 1e-6),
    # no Anderson, z order, linear tets
    "cant_z_noaa": (lambda: scenes.cantilever(10, 3, 3, scenes.LINEAR, iters=30, n_steps=2,
                                              variant=scenes.VARIANT_X, accel=0), 1e-9),
    # at scale: the C4 recipe at the reference golden's size (64 000 tets, checked
    # against tests/golden/full_drop40_z_nh_aa6.npz) and at full size (1 000 000 tets, against
    # the single-GPU run) -- per-part fused subtrees, split-K tiles inside a part, the dense top
    # split by rows, GPU-backend top fronts (AA_DENSE_MIN_FRONT default)
    "drop40_ref": (lambda: scenes.tet_drop(40, 16, 20, iters=10, n_steps=3), 1e-6),
    "block1m": (lambda: scenes.tet_drop(100, 40, 50, iters=40, n_steps=3), 1e-6),
}

# Geometry (ALM) cases: the same bars as tests/test_gpu_geom.py (comb relative to comb_0: 1e-8 over
# the first 40 accepted iterations, 1e-6 over the curve; solution 1e-8 / 1e-6 relative)
GEOM_CASES = {
    "pq": lambda: geom_scenes.pq_heightfield(24, 20, iters=40, aa_m=10, noise=0.3),
    "wire": lambda: geom_scenes.wire_grid(24, 24, iters=40, aa_m=20),
    "pq_noaa": lambda: geom_scenes.pq_heightfield(16, 16, iters=30, aa_m=0, noise=0.3),
}
