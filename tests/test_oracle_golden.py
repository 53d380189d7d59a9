"""CPU: the oracle (our C++ restatement) against golden vectors produced by the REFERENCE
compiled from its own sources (tests/golden/make_golden.py). Pins the oracle before it is
trusted as the checker of the HIP path."""
import numpy as np
import pytest

from golden_io import case_names, compare, load_case

# closed-form element paths are pinned to rounding; L-BFGS prox paths (NH/StVK) only to the
# 1e-6 relative-gradient tolerance of the per-element solve
def tolerances(name):
    hyper = ("nh" in name) or ("stvk" in name) or ("beams" in name)
    return (1e-6, 1e-6) if hyper else (1e-9, 1e-9)


@pytest.mark.parametrize("name", case_names(extras=False))
def test_oracle_matches_reference_trajectory(name, oracle):
    sc, ref = load_case(name)
    got = oracle.run_elastic(sc)
    tc, tx = tolerances(name)
    assert [len(s["prim"]) for s in got] == [len(s["prim"]) for s in ref]
    fails = compare(ref, got, tc, tx)
    assert not fails, fails


def test_oracle_elements(oracle):
    import os
    from golden_io import GOLDEN
    d = np.load(os.path.join(GOLDEN, "elements.npz"))
    for X, Y in zip(d["tet_linear_in"], d["tet_linear_out"]):
        np.testing.assert_allclose(oracle.tet_prox_linear(X), Y, rtol=0, atol=1e-12)
    for name in ("tri_h_limits", "tri_h_free"):
        prm = d[name + "_prm"]
        for X, Y in zip(d[name + "_in"], d[name + "_out"]):
            np.testing.assert_allclose(oracle.tri_prox(X, prm[2], prm[3]), Y, rtol=0, atol=1e-12)
    for mat, name in ((1, "tet_nh"), (2, "tet_stvk")):
        E, nu, h = d[name + "_prm"][:3]
        mu, lam = E / (2 * (1 + nu)), E * nu / ((1 + nu) * (1 - 2 * nu))
        for X, Y in zip(d[name + "_in"], d[name + "_out"]):
            out, _ = oracle.tet_prox_hyper(mat, mu, lam, lam + 2 * mu / 3, h ** 3 / 6, X)
            np.testing.assert_allclose(out, Y, rtol=0, atol=1e-6 * max(1, np.linalg.norm(Y)))
    i = 0
    while f"cod{i}_M" in d:
        th = oracle.cod_solve(d[f"cod{i}_M"], d[f"cod{i}_b"])
        ref = d[f"cod{i}_theta"]
        np.testing.assert_allclose(th, ref, rtol=0, atol=1e-6 * max(1.0, np.linalg.norm(ref)))
        i += 1


def test_z_reference_reject_flags_are_the_references():
    """The z-AA reference logs no reject column (admm_anderson_xzu/src/Solver.hpp:142-144), so
    make_golden.py rebuilds its flags: a recorded prim rise is a reject (Solver.cpp:159-176), and
    the per-step count it prints ("reset number", Solver.cpp:253) is kept as ref_resets. Every
    accelerated z-AA fixture's flags must account for exactly that count (reject_exact), so the
    flags the GPU tests compare are the reference's own, not a column of zeros."""
    import os
    from golden_io import GOLDEN
    seen = 0
    for name in case_names():
        d = np.load(os.path.join(GOLDEN, name + ".npz"))
        if "ref_resets" not in d.files:
            continue
        seen += 1
        o = 0
        for k, n in enumerate(d["nrec"]):
            flags = d["reject"][o:o + n]
            o += n
            assert d["reject_exact"][k] == 1, (name, k)
            assert int(flags.sum()) == int(d["ref_resets"][k]), (name, k)
            p = d["prim"][o - n:o]
            assert np.array_equal(flags[1:] == 1, p[1:] > p[:-1]), (name, k)
    assert seen >= 5
