"""The C++ drop-in facades compile against the C ABI on CPU; on the GPU they run reference-style
callers: include/aa_admm.hpp (admm::Solver, tests/cpp/facade_cloth.cpp) checked against the
oracle, include/aa_geometry.hpp (ALMGeometrySolver<3> + Constraint<3>,
tests/cpp/facade_geom.cpp) checked bit for bit against the same scene bound through the Python
binding (both drive the identical device path, so any mapping error shows)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO
from golden_io import scenes
import refio  # noqa: E402  (oracle/ on sys.path via conftest)

SRC = os.path.join(REPO, "tests", "cpp", "facade_cloth.cpp")


GEOM_SRC = os.path.join(REPO, "tests", "cpp", "facade_geom.cpp")


def build(out, src=SRC):
    lib = os.path.join(REPO, "aa-admm_amd")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I" + os.path.join(REPO, "include"), src, "-o", out,
                    "-L" + lib, "-laa_admm", "-Wl,-rpath," + lib], check=True)


def test_facade_builds(tmp_path):
    build(str(tmp_path / "facade_cloth"))


def test_geometry_facade_builds(tmp_path):
    build(str(tmp_path / "facade_geom"), GEOM_SRC)


def _plain(sc, penalty):
    sc.solver, sc.penalty = "plain", penalty
    return sc


@pytest.mark.gpu
@pytest.mark.parametrize("builder", [
    lambda gs: gs.pq_heightfield(12, 10, iters=40, aa_m=10, noise=0.3),
    lambda gs: gs.wire_grid(12, 12, iters=40, aa_m=20),
    lambda gs: _plain(gs.pq_heightfield(12, 10, iters=40, aa_m=10, noise=0.3), 1e3),   # GeometrySolver<3>
])
def test_geometry_facade_matches_binding(builder, tmp_path, pkg, ctx):
    sc = builder(pkg.geom_scenes)
    exe, scene, out = str(tmp_path / "facade_geom"), str(tmp_path / "s.bin"), str(tmp_path / "o.bin")
    build(exe, GEOM_SRC)
    refio.write_geom_scene(sc, scene)
    eps = 1e-8 * max(sc.avg_edge_length(), 1e-300)
    r = subprocess.run([exe, scene, out, repr(eps), sc.solver], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(out, "rb").read()
    nf = int(np.frombuffer(raw[:4], np.int32)[0])
    comb = np.frombuffer(raw[4:4 + 8 * nf], np.float64)
    x = np.frombuffer(raw[4 + 8 * nf:], np.float64).reshape(-1, 3)
    want, g = pkg.capi.run_geom(ctx, sc)
    g.close()
    assert nf == len(want["comb"]) == sc.iters
    assert np.array_equal(comb, want["comb"])
    assert np.array_equal(x, want["x"])


@pytest.mark.gpu
def test_facade_runs_and_matches_oracle(tmp_path, oracle):
    exe = str(tmp_path / "facade_cloth")
    build(exe)
    os.makedirs(tmp_path / "result")   # Solver::step() then writes result/residual-6.txt, as the reference
    out = subprocess.run([exe], capture_output=True, text=True, check=True, cwd=str(tmp_path)).stdout.split()
    n, comb0, combl = int(out[0]), float(out[1]), float(out[2])
    rows = [l.split("\t") for l in open(tmp_path / "result" / "residual-6.txt").read().splitlines()]
    assert len(rows) == n and all(len(r) == 4 for r in rows)   # (u,x) variant: time, prim, comb, reject
    # %.16g in the file (setprecision(16)), %.17g on stdout
    assert abs(float(rows[0][2]) - comb0) <= 1e-15 * comb0 and abs(float(rows[-1][2]) - combl) <= 1e-15 * comb0
    x1 = np.array([float(v) for v in out[3:6]])
    v, t = scenes.tri_blocks(8, 8)
    v = v * 0.25
    pins = np.array([0, 8], np.int32)
    sc = scenes.Scene(x=v, masses=np.full(len(v), 1e-3), groups=[scenes.ElementGroup(1, 0, 50.0, 0.1, t, 0.95, 1.05)],
                      pin_idx=pins, pin_pts=v[pins].copy(), pin_vel=np.zeros((2, 3)), iters=30, aa_m=6)
    want = oracle.run_elastic(sc)
    assert n == len(want[0]["comb"])
    assert abs(comb0 - want[0]["comb"][0]) <= 1e-9 * want[0]["comb"][0]
    assert abs(combl - want[0]["comb"][-1]) <= 1e-9 * want[0]["comb"][0]
    np.testing.assert_allclose(x1, want[0]["x"].reshape(-1, 3)[1], rtol=0, atol=1e-9)
