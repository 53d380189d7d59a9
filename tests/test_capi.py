"""CPU: the HIP C-ABI library builds for gfx950, loads, and exports every entry point that
include/aa_admm.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

from conftest import REPO


def declared_symbols():
    src = open(os.path.join(REPO, "include", "aa_admm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(aa_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("aa_elastic_create", "aa_elastic_initialize", "aa_elastic_step", "aa_elastic_get_history"):
        assert s in syms


def test_library_exports_every_declared_symbol(pkg):
    lib = ctypes.CDLL(pkg.capi.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(pkg.capi.EXPORTS) == declared_symbols()


def test_library_is_gfx950_code_object(pkg):
    data = open(pkg.capi.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_error_without_device(pkg):
    lib = pkg.capi.lib()
    assert b"gfx950" in lib.aa_version()
    # argument validation works without touching a GPU
    assert lib.aa_elastic_step(None) == -1
    assert b"null" in lib.aa_last_error()
