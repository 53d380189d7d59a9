"""The result/residual-*.txt writers (Solver::save, Solver.hpp:130-155 in both
admm-elastic copies; ALMGeometrySolver::save, ALMGeometrySolver.h:343-365). Pinned to the
reference's own files (tests/golden/ref_residual_{h,x}.txt, written by the reference's save()
during `make_golden.py --residual-files`): the CPU test re-writes the reference's numbers with
our writer and must reproduce its text byte for byte (format: columns, %.16g = ostream
setprecision(16)); the GPU test runs the same scenes and compares the written columns with
the reference's (residuals at 1e-9 of the first comb, reject flags equal; the time column is
wall/device clock and only checked to be increasing)."""
import os

import numpy as np
import pytest

from golden_io import GOLDEN, load_case

CASES = {"ref_residual_h.txt": ("cant8_ux_lin_aa6", 4), "ref_residual_x.txt": ("cloth12_z_noaa", 3)}


def _read(path):
    with open(path) as f:
        lines = [l for l in f.read().splitlines() if l and not l.startswith("#")]
    return lines, [l.split("\t") for l in lines]


@pytest.mark.parametrize("fixture", sorted(CASES))
def test_writer_reproduces_reference_text(fixture, pkg, tmp_path):
    lines, rows = _read(os.path.join(GOLDEN, fixture))
    ncol = CASES[fixture][1]
    assert all(len(r) == ncol for r in rows)
    cols = [np.array([float(r[0]) for r in rows]), np.array([float(r[1]) for r in rows]),
            np.array([float(r[2]) for r in rows])]
    if ncol == 4:
        cols.append(np.array([int(r[3]) for r in rows], np.int32))
    m = 6 if "aa6" in CASES[fixture][0] else 0
    path = pkg.capi.write_residual_file(str(tmp_path), m, *cols)
    assert os.path.basename(path) == ("residual-6.txt" if m else "residual-no.txt")
    with open(path) as f:
        assert f.read().splitlines() == lines


@pytest.mark.gpu
@pytest.mark.parametrize("fixture", sorted(CASES))
def test_gpu_save_matches_reference_file(fixture, pkg, ctx, tmp_path):
    name, ncol = CASES[fixture]
    _, rows = _read(os.path.join(GOLDEN, fixture))
    sc, ref = load_case(name)
    got, solver = pkg.capi.run_scene(ctx, sc)
    path = solver.save(str(tmp_path))
    solver.close()
    _, mine = _read(path)
    assert len(mine) == len(rows) and all(len(r) == ncol for r in mine)
    a = np.array([[float(x) for x in r[1:3]] for r in mine])
    b = np.array([[float(x) for x in r[1:3]] for r in rows])
    assert np.abs(a - b).max() <= 1e-9 * b[0, 1]
    t = np.array([float(r[0]) for r in mine])
    assert np.all(np.diff(t) >= 0) and t[0] >= 0
    if ncol == 4:
        assert [r[3] for r in mine][:20] == [r[3] for r in rows][:20]
