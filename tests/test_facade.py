"""The C++ drop-in facade (include/aa_admm.hpp): compiles against the C ABI on CPU; on the GPU
it runs a reference-style caller (tests/cpp/facade_cloth.cpp) checked against the oracle."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO
from golden_io import scenes

SRC = os.path.join(REPO, "tests", "cpp", "facade_cloth.cpp")


def build(out):
    lib = os.path.join(REPO, "aa-admm_amd")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I" + os.path.join(REPO, "include"), SRC, "-o", out,
                    "-L" + lib, "-laa_admm", "-Wl,-rpath," + lib], check=True)


def test_facade_builds(tmp_path):
    build(str(tmp_path / "facade_cloth"))


@pytest.mark.gpu
def test_facade_runs_and_matches_oracle(tmp_path, oracle):
    exe = str(tmp_path / "facade_cloth")
    build(exe)
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    n, comb0, combl = int(out[0]), float(out[1]), float(out[2])
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
