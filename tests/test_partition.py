"""CPU tests of the multi-GPU partition.

* the partitioned global solve: nested dissection with forced top bisections, each rank
  forward/backward-sweeping its own part + the shared separators on a partial right-hand side,
  an all-reduce of the separator rows in between (tests/cpp/part_solve.cpp, threads as ranks);
* the multi-rank launch: torch.distributed.run ranks that never import torch, bound to the ROCm
  runtime the library was built against (capi.check_runtime), rendezvous over aa-admm_amd/rdzv.py,
  and the host transport of the C ABI (aa_comm_create_host / aa_comm_allreduce_host) over it --
  the transport the GPU partition tests use to put several ranks on one GPU.
"""
import json
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
import importlib, json, os, sys
import numpy as np
sys.path.insert(0, os.environ["AA_REPO"])
pkg = importlib.import_module("aa-admm_amd")
group, report = pkg.dist.rank_setup(timeout=120)     # library + runtime check first, no torch
assert "torch" not in sys.modules, "a rank process imported torch"
rank, size = group.rank, group.size
# the RCCL id path: librccl is loaded from the runtime's directory (ncclGetUniqueId itself needs a
# GPU, so on the CPU only the load is exercised); the check is repeated after it
try:
    pkg.capi.Comm.unique_id()
except pkg.capi.AAError:
    pass
report = pkg.capi.check_runtime()
comm = pkg.dist.host_comm(group)
assert comm.info() == (rank, size)
a = np.arange(7, dtype=np.float64) * (rank + 1) + 0.1 * rank
out = comm.allreduce_host(a.copy())
want = np.zeros(7)
for r in range(size):   # the transport sums in rank order: exactly this
    want += np.arange(7, dtype=np.float64) * (r + 1) + 0.1 * r
assert np.array_equal(out, want), (out, want)
# every rank holds the same bits
g = group.all_gather_json(out.tobytes().hex())
assert all(x == g[0] for x in g)
assert group.allreduce_scalar(rank + 0.5, "max") == size - 0.5
assert group.broadcast_bytes(b"id-from-0" if rank == 0 else None) == b"id-from-0"
group.barrier()
comm.close()
with open(os.path.join(os.environ["AA_OUT"], f"rank{rank}.json"), "w") as f:   # ranks share stdout
    json.dump(report["bound"], f)
group.close()
"""

TORCH_FIRST = r"""
import importlib, os, sys
import torch   # a framework with its own bundled ROCm runtime, loaded BEFORE the library
sys.path.insert(0, os.environ["AA_REPO"])
pkg = importlib.import_module("aa-admm_amd")
try:
    pkg.dist.rank_setup(timeout=5)
except RuntimeError as e:
    print("REFUSED", str(e)[:200])
else:
    print("ACCEPTED")
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(script, nproc, env, timeout=300):
    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
                           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script)],
                          capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("nproc", [2, 3])
def test_host_transport_world_n_runs_on_the_built_runtime(nproc, tmp_path, pkg):
    """torch.distributed.run ranks (the launch bench.py --gpus N makes): every rank loads
    libaa_admm.so before anything else and binds the ROCm runtime `ldd libaa_admm.so` names --
    libamdhip64, libhsa-runtime64, rocBLAS, rocSOLVER and (dlopened) RCCL, by dladdr AND by every
    mapped copy in /proc/self/maps -- never torch's bundled build; the torch-free group then runs
    the host transport (rank-order sums, identical bits on every rank) and its collectives."""
    w = tmp_path / "worker.py"
    w.write_text(WORKER)
    env = dict(os.environ, AA_REPO=REPO, AA_OUT=str(tmp_path), OMP_NUM_THREADS="1")
    r = _torchrun(w, nproc, env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    want = pkg.capi.expected_runtime_dir()
    for k in range(nproc):
        bound = json.load(open(tmp_path / f"rank{k}.json"))
        assert set(bound) == set(pkg.capi.RUNTIME_LIBS)
        for k, path in bound.items():
            assert os.path.dirname(path) == want and "torch" not in path, (k, path)


def test_runtime_check_refuses_a_process_bound_to_another_rocm(tmp_path):
    """The check is not vacuous: a process that imported torch first (torch 2.10+rocm7.0 bundles
    libamdhip64 / rocBLAS / rocSOLVER / RCCL under the SONAMEs of /opt/rocm) is refused."""
    w = tmp_path / "torch_first.py"
    w.write_text(TORCH_FIRST)
    r = subprocess.run([sys.executable, str(w)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, AA_REPO=REPO))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "REFUSED" in r.stdout and "torch" in r.stdout, r.stdout


GROUP_WORKER = r"""
import importlib, os, sys
import numpy as np
sys.path.insert(0, os.environ["AA_REPO"])
rdzv = importlib.import_module("aa-admm_amd.rdzv")
g = rdzv.Group.from_env(timeout=60)
rng = np.random.default_rng(g.rank)
a = rng.standard_normal(100_003)
parts = g.all_gather_json(a.tolist())
want = np.array(parts[0])
for p in parts[1:]:
    want = want + np.array(p)
got = g.allreduce_array(a.copy())
assert np.array_equal(got, want)
if os.environ.get("AA_MISMATCH") == "1":
    try:
        g.barrier() if g.rank == 0 else g.allreduce_scalar(1.0)
    except rdzv.GroupError as e:
        with open(os.path.join(os.environ["AA_OUT"], f"mismatch{g.rank}"), "w") as f:
            f.write(str(e))
        sys.exit(0)
    sys.exit(3)
g.close()
open(os.path.join(os.environ["AA_OUT"], f"ok{g.rank}"), "w").close()
"""


@pytest.mark.parametrize("mismatch", ["0", "1"])
def test_rdzv_group_sums_in_rank_order_and_names_mismatches(mismatch, tmp_path):
    w = tmp_path / "gw.py"
    w.write_text(GROUP_WORKER)
    r = _torchrun(w, 4, dict(os.environ, AA_REPO=REPO, AA_OUT=str(tmp_path), AA_MISMATCH=mismatch), timeout=200)
    if mismatch == "0":
        assert r.returncode == 0 and all((tmp_path / f"ok{k}").exists() for k in range(4)), r.stderr[-3000:]
    else:   # rank 0 sees the first frame of another collective and says so
        f = tmp_path / "mismatch0"
        assert f.exists() and "collective mismatch" in f.read_text(), r.stderr[-3000:]


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
