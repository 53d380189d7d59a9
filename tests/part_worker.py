"""One rank of a partitioned elastic run (launched by torch.distributed.run from
tests/test_gpu_partition.py). Every rank binds the same scene, attaches a communicator and
runs the time steps; rank r writes its per-step history and final state to OUT/rank{r}.npz.

    AA_CASE=<name> AA_TRANSPORT=host|rccl AA_OUT=<dir> python -m torch.distributed.run ... part_worker.py
"""
import importlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from part_cases import CASES, GEOM_CASES  # noqa: E402


def main():
    # no torch in a rank process: the library is loaded and its ROCm runtime checked first
    # (aa-admm_amd/dist.py rank_setup), the rendezvous is aa-admm_amd/rdzv.py
    pkg = importlib.import_module("aa-admm_amd")
    group, report = pkg.dist.rank_setup()
    rank, size = group.rank, group.size
    with open(os.path.join(os.environ["AA_OUT"], f"rank{rank}.runtime.json"), "w") as f:
        json.dump(report, f)
    case = os.environ["AA_CASE"]
    device = int(os.environ.get("AA_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    ctx = pkg.capi.Context(device)
    if os.environ.get("AA_TRANSPORT", "host") == "rccl":
        comm = pkg.dist.rccl_comm(ctx, group)
    else:
        comm = pkg.dist.host_comm(group)
    if case.startswith("geom:"):
        sc = GEOM_CASES[case[5:]]()
        h, g = pkg.capi.run_geom(ctx, sc, comm=comm)
        np.savez(os.path.join(os.environ["AA_OUT"], f"rank{rank}.npz"), comb=h["comb"], x=h["x"],
                 n_constraints=np.array([g.runtime().n_constraints]))
        g.close()
        comm.close()
        ctx.close()
        group.close()
        return
    sc = CASES[case][0]()
    steps, s = pkg.capi.run_scene(ctx, sc, comm=comm)
    out = {}
    for k, st in enumerate(steps):
        for key in ("prim", "comb", "reject", "x", "v"):
            out[f"{key}{k}"] = st[key]
    rt = s.runtime()
    out["n_elements"] = np.array([rt.n_elements])
    out["iterations"] = np.array([rt.iterations])
    np.savez(os.path.join(os.environ["AA_OUT"], f"rank{rank}.npz"), **out)
    s.close()
    comm.close()
    ctx.close()
    group.close()


if __name__ == "__main__":
    try:
        main()
    except BaseException:   # the rank's own traceback, where the test can read it (torchrun's
        import traceback    # summary crowds it out of the captured stderr)
        with open(os.path.join(os.environ.get("AA_OUT", "."), f"rank{os.environ.get('RANK', '0')}.err"), "w") as f:
            traceback.print_exc(file=f)
        raise
