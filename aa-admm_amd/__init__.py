"""aa-admm_amd: MI355X-native Anderson-accelerated ADMM hot path.

The product is libaa_admm.so (HIP kernels + host C++ + C ABI in include/aa_admm.h);
`capi` is its Python binding and `scenes` the headless scene builders. Import as
`importlib.import_module("aa-admm_amd")` (the directory name is not an identifier).
"""
from . import capi, dist, geom_report, geom_scenes, rdzv, scenes  # noqa: F401
