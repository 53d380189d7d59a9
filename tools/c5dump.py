import importlib, sys, os, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
pkg = importlib.import_module("aa-admm_amd")
sc = pkg.geom_scenes.wire_grid(707, 707, iters=10)
ctx = pkg.capi.Context(0)
h, g = pkg.capi.run_geom(ctx, sc)
np.save("gpurun_out/c5_x10.npy", h["x"])
print("comb", h["comb"][:3], h["comb"][-1])
