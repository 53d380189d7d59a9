"""Run a golden case's scene on the GPU and save its per-step histories (prim, comb, reject) to
an npz, for a side-by-side look against the fixture (tests/golden/<case>.npz).

    python tools/golden_dump.py drop20_z_nh_aa6_rej gpurun_out/golden_dump.npz
"""
import importlib, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
pkg = importlib.import_module("aa-admm_amd")
from golden_io import load_case

name, out = sys.argv[1], sys.argv[2]
sc, ref = load_case(name)
ctx = pkg.capi.Context(0)
got, _ = pkg.capi.run_scene(ctx, sc)
arrs = {}
for k, h in enumerate(got):
    for key in ("prim", "comb", "reject"):
        arrs[f"{key}{k}"] = np.asarray(h[key])
np.savez(out, **arrs)
print(name, [int(np.sum(h["reject"])) for h in got], [int(np.sum(r["reject"])) for r in ref])
