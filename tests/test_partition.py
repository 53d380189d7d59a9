"""CPU tests of the multi-GPU partition.

* the partitioned global solve: nested dissection with forced top bisections, each rank
  forward/backward-sweeping its own part + the shared separators on a partial right-hand side,
  an all-reduce of the separator rows in between (tests/cpp/part_solve.cpp, threads as ranks);
* the host transport of the C ABI (aa_comm_create_host / aa_comm_allreduce_host) under
  torch.distributed with gloo, world size 2 -- the transport the GPU partition tests use to put
  several ranks on one GPU.
"""
import os
import shutil
import socket
import subprocess
import sys

import pytest

from conftest import REPO


def test_partitioned_solve_matches_unpartitioned(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path / "part_solve")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fopenmp", os.path.join(REPO, "tests", "cpp", "part_solve.cpp"),
                    os.path.join(REPO, "aa-admm_amd", "csrc", "spd_direct.cpp"), "-o", exe], check=True)
    for dims in ([], ["24", "10", "17"]):
        r = subprocess.run([exe] + dims, capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, OMP_NUM_THREADS="2"))
        print(r.stdout)
        assert r.returncode == 0, r.stdout + r.stderr
        assert r.stdout.count(" OK") == 10 and r.stdout.count("SINGULAR_OK") == 2


def test_fused_subtree_cut_checks_aggregate_lds(tmp_path):
    """The fused-subtree cut height (csrc/solve_plan.hpp) is checked against the launch's own
    LDS aggregate -- the widest level vector of any subtree plus the records of the largest one --
    on a tree whose two subtrees each fit alone but not together (tests/cpp/cut_height.cpp)."""
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path / "cut_height")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "aa-admm_amd", "csrc"),
                    os.path.join(REPO, "tests", "cpp", "cut_height.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_fused_subtree_update_slots_never_overlap_live(tmp_path):
    """The LDS slots of the fused subtrees' update vectors (solve_plan.hpp plan_update_slots):
    on 300 random trees, no slot written in a level overlaps one still to be read
    (tests/cpp/update_slots.cpp replays the forward kernel's two-phase schedule)."""
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path / "update_slots")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "aa-admm_amd", "csrc"),
                    os.path.join(REPO, "tests", "cpp", "update_slots.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


WORKER = r"""
import importlib, os, sys
import numpy as np
import torch.distributed as dist
sys.path.insert(0, os.environ["AA_REPO"])
pkg = importlib.import_module("aa-admm_amd")
dist.init_process_group("gloo")
rank, size = dist.get_rank(), dist.get_world_size()
comm = pkg.dist.host_comm(rank, size)
assert comm.info() == (rank, size)
a = np.arange(7, dtype=np.float64) * (rank + 1) + 0.1 * rank
out = comm.allreduce_host(a.copy())
want = sum(np.arange(7, dtype=np.float64) * (r + 1) + 0.1 * r for r in range(size))
assert np.allclose(out, want, rtol=1e-15, atol=0), (out, want)
# every rank holds the same bits (the transport broadcasts rank 0's sum)
g = [None] * size
dist.all_gather_object(g, out.tobytes())
assert all(x == g[0] for x in g)
comm.close()
dist.destroy_process_group()
print("RANK_OK", rank)
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_host_transport_gloo_world2(tmp_path, pkg):
    w = tmp_path / "worker.py"
    w.write_text(WORKER)
    env = dict(os.environ, AA_REPO=REPO, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(w)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert r.stdout.count("RANK_OK") == 2


def test_solo_rehearsal_comm_host_semantics(pkg):
    """aa_comm_create_solo (bench.py --rehearse): one rank of a P-way partition alone -- a host
    all-reduce multiplies by P (the setup's scene-identity checks pass), no GPU needed to create it."""
    import numpy as np
    c = pkg.capi.Comm.solo(1, 4)
    assert c.info() == (1, 4)
    assert np.array_equal(c.allreduce_host(np.array([1.0, -2.5, 0.0])), np.array([4.0, -10.0, 0.0]))
    c.close()
    with pytest.raises(pkg.capi.AAError):
        pkg.capi.Comm.solo(4, 4)
