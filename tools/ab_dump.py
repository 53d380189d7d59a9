"""Run one scene through the library AA_ADMM_LIB points at and dump its trajectory (A/B builds:
two runs, then `python tools/ab_dump.py --compare a.npz b.npz` checks they are bit-identical).

    AA_ADMM_LIB=ab/lib_x.so python tools/ab_dump.py out.npz [drop40|c4small|cloth|pq|wire]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
        print("bit-identical" if not bad else f"DIFFER: {bad}")
        sys.exit(1 if bad else 0)
    import importlib
    pkg = importlib.import_module("aa-admm_amd")
    scenes = importlib.import_module("aa-admm_amd.scenes")
    which = sys.argv[2] if len(sys.argv) > 2 else "drop40"
    ctx = pkg.capi.Context(0)
    out = {}
    if which in ("pq", "wire"):
        gs = importlib.import_module("aa-admm_amd.geom_scenes")
        sc = gs.pq_heightfield(64, 64, iters=60, aa_m=10, noise=0.3) if which == "pq" else \
            gs.wire_grid(40, 40, iters=60, aa_m=20)
        h, g = pkg.capi.run_geom(ctx, sc)
        out = {"comb": h["comb"], "x": h["x"]}
        g.close()
    else:
        sc = {"drop40": lambda: scenes.tet_drop(40, 16, 20, iters=12, n_steps=2),
              "c4small": lambda: scenes.tet_drop(60, 24, 28, iters=8, n_steps=1),
              "cloth": lambda: scenes.cloth(64, 64, iters=40, n_steps=2)}[which]()
        got, _ = pkg.capi.run_scene(ctx, sc)
        for i, h in enumerate(got):
            for k in ("prim", "comb", "reject", "x", "v"):
                out[f"{k}{i}"] = np.asarray(h[k])
    np.savez(sys.argv[1], **out)
    ctx.close()


if __name__ == "__main__":
    main()
