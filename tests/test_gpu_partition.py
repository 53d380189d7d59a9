"""GPU: the mesh-partitioned solver reproduces the single-GPU solver.

Several ranks share the one test GPU through the host transport (torch.distributed/gloo;
RCCL refuses two ranks on one device), so this exercises exactly the partitioned code path
of an N-GPU run -- ownership of elements, the separator all-reduce inside the global solve,
all-reduced residual/Anderson partials, the step-end state gather -- except the transport.
The RCCL transport itself is exercised with a one-rank communicator (identity all-reduce),
which must give bit-identical results to the plain solver.

Tolerances as the single-GPU parity tests (residual curves relative to comb_0: 1e-9 closed-
form, 1e-6 L-BFGS; final x the same relative bars); the partition only reorders sums. All
ranks must agree bit for bit (their decisions come from identical all-reduced values)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO
from golden_io import GOLDEN, check_full_golden, compare, compare_geom
from part_cases import CASES, GEOM_CASES

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(case, nranks, out, transport="host", extra_env=None, timeout=240):
    out.mkdir(parents=True, exist_ok=True)
    env = dict(os.environ, AA_CASE=case, AA_OUT=str(out), AA_TRANSPORT=transport, AA_DEVICE="0", AA_COMM_VERIFY="1",
               OMP_NUM_THREADS="4", **(extra_env or {}))
    env.pop("AA_FRONT_RETRY", None)   # a wrong first factorization fails the run (dense_gpu.hip front check)
    dump = os.environ.get("AA_TEST_FRONT_DUMP", "/tmp/aa_front_dump")   # f x f doubles per matrix: not under gpurun_out
    os.makedirs(dump, exist_ok=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    env["AA_FRONT_DUMP"] = dump
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
                        "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
                        os.path.join(REPO, "tests", "part_worker.py")],
                       capture_output=True, text=True, timeout=timeout, env=env)
    # any GPU front that failed a check is a failed run (the backend throws; its line and the dump
    # of the kept copy and first attempt stay in gpurun_out/ for tools/front_replay.py)
    notes = [ln for ln in (r.stderr or "").splitlines() if "[front-check]" in ln]
    if notes:
        with open(os.path.join(REPO, "gpurun_out", "front_check.log"), "a") as fh:
            fh.write(f"{case} P={nranks}: " + " | ".join(notes) + "\n")
    assert not notes, notes
    # every rank bound the ROCm runtime the library was built for (part_worker.py: rank_setup)
    for k in range(nranks):
        rep = json.load(open(out / f"rank{k}.runtime.json"))
        assert all(os.path.dirname(v) == rep["expected"] for v in rep["bound"].values()), rep
    if r.returncode != 0:
        errs = "".join(f"--- {f.name}:\n{f.read_text()[-3000:]}\n" for f in sorted(out.glob("rank*.err")))
        assert False, errs + r.stdout[-1000:] + r.stderr[-2000:]
    return [dict(np.load(out / f"rank{k}.npz")) for k in range(nranks)]


def as_steps(d, n_steps):
    return [{k: d[f"{k}{i}"] for k in ("prim", "comb", "reject", "x", "v")} for i in range(n_steps)]


# 3 ranks: an uneven part count (proportional bisections); top=0: the round-1 layout with one
# supernode per shared separator, solved whole on every rank (AA_TOP_DENSE=0) -- the default is
# one dense top root split over the ranks by rows
# minfront: AA_DENSE_MIN_FRONT -- 64 sends the top fronts (and the larger part fronts) to the GPU
# backend, so the partitioned factorization's device all-reduce of a partial top front runs
# (each rank factors only its own part and the top: aa::PartFactor)
@pytest.mark.parametrize("case,nranks,top,minfront", [("cloth_ux", 2, 1, 0), ("cloth_ux", 4, 1, 0), ("cloth_ux", 3, 1, 0),
                                                      ("cant_ux", 2, 1, 0), ("drop_z", 2, 1, 0), ("drop_z", 4, 1, 0),
                                                      ("drop_z", 3, 1, 0), ("drop_z", 4, 0, 0), ("drop_z", 3, 1, 64),
                                                      ("drop_z", 4, 0, 64), ("beams_z", 2, 1, 0), ("cant_z_noaa", 2, 1, 0)])
def test_partitioned_matches_single_gpu(case, nranks, top, minfront, tmp_path, pkg, ctx):
    builder, tol = CASES[case]
    sc = builder()
    want, _ = pkg.capi.run_scene(ctx, sc)
    env = {"AA_TOP_DENSE": str(top)}
    if minfront:
        env["AA_DENSE_MIN_FRONT"] = str(minfront)
    ranks = run_ranks(case, nranks, tmp_path, extra_env=env)
    # every element is owned by exactly one rank
    assert sum(int(r["n_elements"][0]) for r in ranks) == sc.n_elements()
    # all ranks hold the same bits
    for r in ranks[1:]:
        for k in ranks[0]:
            if k not in ("n_elements",):
                assert np.array_equal(r[k], ranks[0][k]), k
    got = as_steps(ranks[0], len(want))
    assert [len(s["prim"]) for s in got] == [len(s["prim"]) for s in want]
    for s in want:
        s["x"] = s["x"].reshape(-1, 3)
    fails = compare(want, got, tol, tol)
    assert not fails, fails


def _same_bits(ranks):
    for r in ranks[1:]:
        for k in ranks[0]:
            if k not in ("n_elements",):
                assert np.array_equal(r[k], ranks[0][k]), k


@pytest.mark.parametrize("nranks", [2, 4])
def test_partitioned_drop40_matches_reference(nranks, tmp_path, pkg):
    """The partitioned solver at a size where its design matters: the C4 recipe at
    64 000 NeoHookean tets (make_tet_blocks(40,16,20), 3 steps x 10 iterations) on 2 and 4 ranks
    against the REFERENCE's own run (tests/golden/full_drop40_z_nh_aa6.npz) at the single-GPU
    test's bars (test_gpu_full_drop40_matches_reference): each part has its own fused subtrees and
    split-K tile levels, the shared separators are one dense top split over the ranks by rows."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from make_golden import scene_digest
    from part_cases import CASES as C
    ref = np.load(os.path.join(GOLDEN, "full_drop40_z_nh_aa6.npz"))
    sc = C["drop40_ref"][0]()
    assert np.array_equal(scene_digest(sc), ref["digest"]), "regenerated scene differs from the fixture's"
    ranks = run_ranks("drop40_ref", nranks, tmp_path)
    assert sum(int(r["n_elements"][0]) for r in ranks) == sc.n_elements()
    _same_bits(ranks)
    fails = check_full_golden(as_steps(ranks[0], len(ref["nrec"])), ref)
    assert not fails, fails


def test_partitioned_block1m_matches_single_gpu(tmp_path, pkg, ctx):
    """BASELINE configs[3] at full size (1 000 000 NeoHookean tets) on 2 ranks against the
    single-GPU solver, 3 steps x 40 iterations: residual curves within 1e-6 comb_0, final
    positions 1e-6 relative, and the momentum invariant of the partitioned result itself (no pins:
    mass-weighted mean velocity = g dt after the first step, 1e-9). The top fronts of the two-way
    partition are large enough for the GPU backend (AA_DENSE_MIN_FRONT default), so the device
    all-reduce of the partial top fronts runs."""
    sc = CASES["block1m"][0]()
    want, s = pkg.capi.run_scene(ctx, sc)
    s.close()
    ranks = run_ranks("block1m", 2, tmp_path, timeout=420)
    assert sum(int(r["n_elements"][0]) for r in ranks) == sc.n_elements()
    _same_bits(ranks)
    got = as_steps(ranks[0], len(want))
    assert [len(g["prim"]) for g in got] == [len(w["prim"]) for w in want]
    for w in want:
        w["x"] = w["x"].reshape(-1, 3)
    fails = compare(want, got, 1e-6, 1e-6)
    assert not fails, fails
    m = sc.masses
    v1 = got[0]["v"].reshape(-1, 3)
    vbar = (m[:, None] * v1).sum(0) / m.sum()
    g_dt = sc.gravity * sc.dt
    assert abs(vbar[1] - g_dt) <= 1e-9 * abs(g_dt), vbar
    assert abs(vbar[0]) <= 1e-9 * abs(g_dt) and abs(vbar[2]) <= 1e-9 * abs(g_dt), vbar


@pytest.mark.parametrize("graph", ["0", "1"])
def test_rccl_transport_one_rank_is_identity(graph, pkg, ctx, monkeypatch, capfd):
    """ncclCommInitRank / ncclAllReduce on the solver's stream with a one-rank communicator:
    every reduction of the iteration runs through RCCL and the result is bit-identical -- launched
    eagerly (the default) and with the all-reduces recorded into the step's hipGraph
    (AA_RCCL_GRAPH=1)."""
    monkeypatch.setenv("AA_RCCL_GRAPH", graph)
    capi = pkg.capi
    sc = CASES["drop_z"][0]()
    want, _ = capi.run_scene(ctx, sc)
    comm = capi.Comm.rccl(ctx, 0, 1, capi.Comm.unique_id())
    assert comm.info() == (0, 1)
    capfd.readouterr()
    got, s = capi.run_scene(ctx, sc, comm=comm)
    assert "capture failed" not in capfd.readouterr().err   # graph = 1: RCCL recorded and replayed
    for a, b in zip(want, got):
        assert np.array_equal(a["comb"], b["comb"]) and np.array_equal(a["x"], b["x"])
    s.close()
    assert np.array_equal(comm.allreduce_host(np.arange(5.0)), np.arange(5.0))
    comm.close()


def test_front_check_failure_is_an_error_with_a_replayable_dump(pkg, ctx, monkeypatch, capfd, tmp_path):
    """The GPU front check (dense_gpu.hip) is an assertion: a front whose first
    factorization yields a wrong output (here injected: AA_FRONT_CHECK_POISON=1 puts a NaN into the
    first GPU front's first attempt) fails initialize with AA_ERR_NUMERIC -- no silent retry -- and
    AA_FRONT_DUMP writes the kept copy and the first attempt's outputs, which tools/front_replay.py
    replays on the host: it names the outputs that differ from a CPU factor of the kept copy."""
    monkeypatch.setenv("AA_DENSE_MIN_FRONT", "64")
    monkeypatch.delenv("AA_FRONT_RETRY", raising=False)
    monkeypatch.setenv("AA_FRONT_CHECK_POISON", "1")
    monkeypatch.setenv("AA_FRONT_DUMP", str(tmp_path))
    sc = CASES["drop_z"][0]()
    with pytest.raises(pkg.capi.AAError) as ei:
        pkg.capi.run_scene(ctx, sc)
    assert ei.value.code == -4 and "factored wrongly on the first attempt" in str(ei.value), str(ei.value)
    notes = [ln for ln in capfd.readouterr().err.splitlines() if "[front-check]" in ln]
    assert len(notes) == 1, notes
    kept = sorted(tmp_path.glob("front*_kept.bin"))
    assert len(kept) == 1
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import front_replay
    rep = front_replay.replay(str(kept[0]))
    assert rep["kept_factors"] and "first_F" in rep["differ"], rep


def test_front_check_retry_is_bit_identical(pkg, ctx, monkeypatch, capfd):
    """The opt-in kept-copy retry (AA_FRONT_RETRY=1): the poisoned front is factored again from the
    kept copy, reported on stderr, and the run's results are the unpoisoned run's bits (rocBLAS
    atomics off: deterministic)."""
    monkeypatch.setenv("AA_DENSE_MIN_FRONT", "64")
    sc = CASES["drop_z"][0]()
    want, s = pkg.capi.run_scene(ctx, sc)
    s.close()
    assert "[front-check]" not in capfd.readouterr().err   # the product check: no false alarm
    monkeypatch.setenv("AA_FRONT_RETRY", "1")
    monkeypatch.setenv("AA_FRONT_CHECK_POISON", "1")
    got, s = pkg.capi.run_scene(ctx, sc)
    s.close()
    err = capfd.readouterr().err
    notes = [ln for ln in err.splitlines() if "[front-check]" in ln]
    assert len(notes) == 1 and "again on the copy: potrf info 0, 0 non-finite outputs" in notes[0], notes
    for a, b in zip(want, got):
        assert np.array_equal(a["comb"], b["comb"]) and np.array_equal(a["x"], b["x"])


@pytest.mark.parametrize("case,nranks,minfront", [("pq", 2, 0), ("pq", 4, 0), ("pq", 3, 0), ("pq", 3, 64), ("wire", 2, 0),
                                                  ("pq_noaa", 2, 0)])
def test_partitioned_geometry_matches_single_gpu(case, nranks, minfront, tmp_path, pkg, ctx):
    sc = GEOM_CASES[case]()
    want, g = pkg.capi.run_geom(ctx, sc)
    n_cons = g.runtime().n_constraints
    g.close()
    ranks = run_ranks("geom:" + case, nranks, tmp_path,
                      extra_env={"AA_DENSE_MIN_FRONT": str(minfront)} if minfront else None)
    assert sum(int(r["n_constraints"][0]) for r in ranks) == n_cons   # each constraint on one rank
    for r in ranks[1:]:
        assert np.array_equal(r["comb"], ranks[0]["comb"]) and np.array_equal(r["x"], ranks[0]["x"])
    got = {"comb": ranks[0]["comb"], "x": ranks[0]["x"]}
    fails = compare_geom(want, got, 1e-8, 1e-8, n_check=40) + compare_geom(want, got, 1e-6, 1e-6)
    assert not fails, fails


def test_partitioned_solve_branches_bit_identical(tmp_path, pkg):
    """A rank's share of the partitioned solve swept as parallel branches (AA_SOLVE_BRANCHES=2: its
    part's subtrees on two streams, the part's top and the shared top after the join, the top's
    all-reduces in between unchanged) gives every rank the same bits as the single-stream sweep:
    the C4 recipe at 64 000 tets on 2 ranks, 3 steps x 10 iterations."""
    a = run_ranks("drop40_ref", 2, tmp_path / "b1", extra_env={"AA_SOLVE_BRANCHES": "1"})
    b = run_ranks("drop40_ref", 2, tmp_path / "b2", extra_env={"AA_SOLVE_BRANCHES": "2", "AA_SOLVE_STATS": "1"})
    for ra, rb in zip(a, b):
        for k in ra:
            assert np.array_equal(ra[k], rb[k]), k
