"""ctypes binding of libaa_admm.so (include/aa_admm.h) -- the Python host mirror of the
reference's admm::Solver API (admm_anderson_hard_zxu/src/Solver.hpp:39-262).

This is exactly the stub a maintainer would add on the Python side of the boundary
(INTEGRATION.md). There is no CPU fallback: if the HIP library is missing or no GPU is
visible, constructing a context raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AA_ADMM_LIB") or os.path.join(HERE, "libaa_admm.so")   # override: A/B builds

AA_LINEAR, AA_NEOHOOKEAN, AA_STVK = 0, 1, 2
AA_VARIANT_Z, AA_VARIANT_UX = 0, 1
NOACC, ANDERSON = 0, 1

EXPORTS = [
    "aa_last_error", "aa_version", "aa_ctx_create", "aa_ctx_destroy", "aa_ctx_synchronize", "aa_ctx_bench_read",
    "aa_ctx_warm_dense", "aa_lame_from_young",
    "aa_settings_default", "aa_elastic_create", "aa_elastic_destroy", "aa_elastic_add_nodes", "aa_elastic_add_tets",
    "aa_elastic_add_tris", "aa_elastic_set_pins", "aa_elastic_initialize", "aa_elastic_step",
    "aa_elastic_add_obstacle", "aa_elastic_set_collisions", "aa_elastic_add_wind", "aa_elastic_set_wind",
    "aa_elastic_num_nodes", "aa_elastic_get_x", "aa_elastic_get_v", "aa_elastic_set_v", "aa_elastic_get_history",
    "aa_elastic_get_times", "aa_elastic_set_iterations", "aa_elastic_set_x",
    "aa_elastic_runtime", "aa_elastic_bench_iterations", "aa_elastic_kernel_stats", "aa_elastic_local_stats",
    "aa_elastic_setup_phases",
    "aa_runtime_libraries", "aa_comm_unique_id", "aa_comm_create_rccl", "aa_comm_create_host", "aa_comm_create_solo", "aa_comm_destroy", "aa_comm_info",
    "aa_comm_allreduce_host", "aa_elastic_set_comm", "aa_geom_set_comm",
    "aa_geom_create", "aa_geom_create_kind", "aa_geom_destroy", "aa_geom_add_ref_surface", "aa_geom_add_constraints", "aa_geom_add_laplacian",
    "aa_geom_add_closeness", "aa_geom_add_laplacians", "aa_geom_add_closenesses", "aa_geom_setup", "aa_geom_solve", "aa_geom_set_stop", "aa_geom_get_solution", "aa_geom_get_history",
    "aa_geom_runtime_info", "aa_geom_closest_points", "aa_geom_bench_iterations", "aa_geom_kernel_stats",
    "aa_test_prox", "aa_test_cod_solve", "aa_test_geom_project",
]

# Geometry constraint types (Geometry/Constraint.h) and SPD solver types (SolverCommon.h)
AA_CON_PLANE, AA_CON_ANGLE, AA_CON_EDGE, AA_CON_CLOSENESS, AA_CON_POINT_TO_REF, AA_CON_REF_SURFACE = range(6)
AA_SPD_LDLT, AA_SPD_LLT = 0, 1
AA_GEOM_ALM, AA_GEOM_PLAIN = 0, 1   # ALMGeometrySolver<3> / GeometrySolver<3>


class Lame(C.Structure):
    """admm::Lame (EnergyTerm.hpp:35-61)."""
    _fields_ = [("mu", C.c_double), ("lambda_", C.c_double), ("limit_min", C.c_double), ("limit_max", C.c_double)]

    @classmethod
    def from_young(cls, E, nu, limit_min=-100.0, limit_max=100.0):
        mu = E / (2.0 * (1.0 + nu))
        lam = E * nu / ((1.0 + nu) * (1.0 - 2.0 * nu))
        return cls(mu, lam, limit_min, limit_max)


class Settings(C.Structure):
    """admm::Solver::Settings (Solver.hpp:45-67) + the variant."""
    _fields_ = [("timestep_s", C.c_double), ("verbose", C.c_int), ("admm_iters", C.c_int), ("gravity", C.c_double),
                ("constraint_w", C.c_double), ("anderson_m", C.c_int), ("penalty", C.c_double),
                ("acceleration_type", C.c_int), ("variant", C.c_int), ("eps_rel", C.c_double)]

    def __init__(self, **kw):
        super().__init__(1.0 / 30.0, 1, 500, -9.8, -1.0, 2, 1.0, NOACC, AA_VARIANT_UX, 0.0)
        for k, v in kw.items():
            setattr(self, k, v)


class Runtime(C.Structure):
    _fields_ = [("global_ms", C.c_double), ("local_ms", C.c_double), ("acceleration_ms", C.c_double),
                ("initialization_ms", C.c_double), ("step_ms", C.c_double), ("setup_ms", C.c_double),
                ("iterations", C.c_int), ("rejects", C.c_int), ("nnz_factor", C.c_longlong), ("n_free", C.c_int),
                ("n_pinned", C.c_int), ("n_elements", C.c_int), ("z_dim", C.c_int)]


_LIB = None


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"aa_admm HIP library not built: {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        L.aa_last_error.restype = C.c_char_p
        L.aa_version.restype = C.c_char_p
        _LIB = L
    return _LIB


RUNTIME_LIBS = ("amdhip64", "hsa-runtime64", "rocblas", "rocsolver", "rccl")


def runtime_libraries() -> dict:
    """{name: path} of the HIP / HSA / rocBLAS / rocSOLVER / RCCL objects this process has bound
    (aa_runtime_libraries, dladdr; loads librccl, needs no GPU)."""
    n = C.c_longlong()
    buf = C.create_string_buffer(4096)
    _chk(lib().aa_runtime_libraries(buf, C.c_longlong(len(buf)), C.byref(n)))
    out = {}
    for ln in buf.value.decode().splitlines():
        k, _, v = ln.partition("=")
        out[k] = v
    return out


def expected_runtime_dir() -> str:
    """The ROCm lib directory `ldd libaa_admm.so` resolves libamdhip64 to (the build's RUNPATH)."""
    import subprocess
    r = subprocess.run(["ldd", LIB_PATH], capture_output=True, text=True, check=True)
    for ln in r.stdout.splitlines():
        if "libamdhip64" in ln and "=>" in ln:
            return os.path.dirname(os.path.realpath(ln.split("=>")[1].split("(")[0].strip()))
    raise RuntimeError(f"ldd {LIB_PATH}: libamdhip64 not found")


def mapped_runtime_objects() -> dict:
    """{name: sorted real paths} of every mapped copy of the RUNTIME_LIBS (/proc/self/maps)."""
    out = {k: set() for k in RUNTIME_LIBS}
    with open("/proc/self/maps") as f:
        for ln in f:
            parts = ln.split()
            if len(parts) < 6 or not parts[5].startswith("/"):
                continue
            base = os.path.basename(parts[5])
            for k in RUNTIME_LIBS:
                if base.startswith("lib" + k + ".so"):
                    out[k].add(os.path.realpath(parts[5]))
    return {k: sorted(v) for k, v in out.items()}


def check_runtime() -> dict:
    """Fail unless every runtime object bound by this process (and every mapped copy of one) lives in
    the ROCm directory the library was linked against -- e.g. not a framework's bundled ROCm loaded
    before libaa_admm.so. Returns {"expected": dir, "bound": {...}, "mapped": {...}}."""
    want = expected_runtime_dir()
    bound = {k: os.path.realpath(v) if v else "" for k, v in runtime_libraries().items()}
    mapped = mapped_runtime_objects()
    bad = [f"{k} bound to {v or '(not loaded)'}" for k, v in bound.items() if os.path.dirname(v) != want]
    bad += [f"{k} mapped from {p}" for k, ps in mapped.items() for p in ps if os.path.dirname(p) != want]
    if bad:
        raise RuntimeError(f"libaa_admm.so was built against {want}, but this process uses: " + "; ".join(bad)
                           + " (load the library before any framework that bundles its own ROCm runtime)")
    return {"expected": want, "bound": bound, "mapped": mapped}


class AAError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _chk(rc):
    if rc != 0:
        raise AAError(rc, lib().aa_last_error().decode())


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


class Context:
    def __init__(self, device=0):
        self.h = C.c_void_p()
        _chk(lib().aa_ctx_create(C.c_int(device), C.byref(self.h)))

    def bench_read(self, nbytes=1 << 30):
        """GB/s of a 16-B/lane streaming read of nbytes (aa_ctx_bench_read): the measured HBM ceiling."""
        g = C.c_double()
        _chk(lib().aa_ctx_bench_read(self.h, C.c_longlong(nbytes), C.byref(g)))
        return g.value

    def warm_dense(self):
        """Wall ms of the one-time rocBLAS / rocSOLVER code-object load (aa_ctx_warm_dense); 0 when warm."""
        ms = C.c_double()
        _chk(lib().aa_ctx_warm_dense(self.h, C.byref(ms)))
        return ms.value

    def synchronize(self):
        _chk(lib().aa_ctx_synchronize(self.h))

    def close(self):
        if self.h:
            lib().aa_ctx_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_longlong, C.c_void_p)


class Comm:
    """Communicator of the partitioned multi-GPU solver (aa_comm_*).

    Comm.rccl(ctx, rank, size, unique_id): RCCL over xGMI, one process per GPU.
    Comm.host(fn, rank, size): host-staged transport; fn(np.ndarray) sums the array in place
    over the ranks (e.g. torch.distributed over gloo) -- lets several ranks share one GPU.
    """

    def __init__(self, h, keep=None):
        self.h = h
        self._keep = keep

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_ubyte * 128)()
        _chk(lib().aa_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def rccl(cls, ctx: Context, rank: int, size: int, unique_id: bytes):
        h = C.c_void_p()
        uid = (C.c_ubyte * 128).from_buffer_copy(unique_id)
        _chk(lib().aa_comm_create_rccl(ctx.h, uid, C.c_int(rank), C.c_int(size), C.byref(h)))
        return cls(h)

    @classmethod
    def host(cls, fn, rank: int, size: int):
        def cb(buf, n, _user):
            try:
                fn(np.ctypeslib.as_array(buf, shape=(int(n),)))
                return 0
            except Exception:   # noqa: BLE001 -- reported to C as a failed reduction
                return 1
        cfn = HOST_ALLREDUCE_FN(cb)
        h = C.c_void_p()
        _chk(lib().aa_comm_create_host(cfn, None, C.c_int(rank), C.c_int(size), C.byref(h)))
        return cls(h, keep=cfn)

    @classmethod
    def solo(cls, rank: int, size: int):
        """Timing rehearsal: one rank of a size-way partition alone (aa_comm_create_solo)."""
        h = C.c_void_p()
        _chk(lib().aa_comm_create_solo(C.c_int(rank), C.c_int(size), C.byref(h)))
        return cls(h)

    def info(self):
        r, n = C.c_int(), C.c_int()
        _chk(lib().aa_comm_info(self.h, C.byref(r), C.byref(n)))
        return r.value, n.value

    def allreduce_host(self, a):
        a = np.ascontiguousarray(a, np.float64)
        _chk(lib().aa_comm_allreduce_host(self.h, _dp(a), C.c_longlong(a.size)))
        return a

    def close(self):
        if self.h:
            lib().aa_comm_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Solver:
    """Mirror of admm::Solver: add_nodes / create_*_from_mesh / set_pins / initialize / step."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self.h = C.c_void_p()
        _chk(lib().aa_elastic_create(ctx.h, C.byref(self.h)))

    def close(self):
        if self.h:
            lib().aa_elastic_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_nodes(self, x, m3):
        x = np.ascontiguousarray(x, np.float64).reshape(-1)
        m3 = np.ascontiguousarray(m3, np.float64).reshape(-1)
        tot = C.c_int()
        _chk(lib().aa_elastic_add_nodes(self.h, _dp(x), _dp(m3), C.c_int(len(x) // 3), C.byref(tot)))
        return tot.value

    def add_tets(self, verts, tets, material, lame: Lame, vertex_offset=0):
        v = np.ascontiguousarray(verts, np.float64).reshape(-1)
        t = np.ascontiguousarray(tets, np.int32).reshape(-1)
        _chk(lib().aa_elastic_add_tets(self.h, _dp(v), _ip(t), C.c_int(len(t) // 4), C.c_int(material),
                                       C.byref(lame), C.c_int(vertex_offset)))

    def add_tris(self, verts, tris, lame: Lame, vertex_offset=0):
        v = np.ascontiguousarray(verts, np.float64).reshape(-1)
        t = np.ascontiguousarray(tris, np.int32).reshape(-1)
        _chk(lib().aa_elastic_add_tris(self.h, _dp(v), _ip(t), C.c_int(len(t) // 3), C.byref(lame),
                                       C.c_int(vertex_offset)))

    def set_pins(self, inds, points=None):
        i = np.ascontiguousarray(inds, np.int32).reshape(-1)
        if points is None:
            _chk(lib().aa_elastic_set_pins(self.h, _ip(i), None, C.c_int(len(i))))
        else:
            p = np.ascontiguousarray(points, np.float64).reshape(-1)
            _chk(lib().aa_elastic_set_pins(self.h, _ip(i), _dp(p), C.c_int(len(i))))

    def add_obstacle(self, kind, params):
        """Solver::add_obstacle with a PassiveObject.hpp shape (AA_OBS_*)."""
        p = np.zeros(8)
        q = np.asarray(params, np.float64).reshape(-1)
        p[:len(q)] = q
        _chk(lib().aa_elastic_add_obstacle(self.h, C.c_int(kind), _dp(p)))

    def set_collisions(self, inds):
        i = np.ascontiguousarray(inds, np.int32).reshape(-1)
        _chk(lib().aa_elastic_set_collisions(self.h, _ip(i), C.c_int(len(i))))

    def add_wind(self, tris, direction):
        t = np.ascontiguousarray(tris, np.int32).reshape(-1)
        d = np.ascontiguousarray(direction, np.float64).reshape(3)
        k = C.c_int()
        _chk(lib().aa_elastic_add_wind(self.h, _ip(t), C.c_int(len(t) // 3), _dp(d), C.byref(k)))
        return k.value

    def set_wind(self, wid, direction):
        d = np.ascontiguousarray(direction, np.float64).reshape(3)
        _chk(lib().aa_elastic_set_wind(self.h, C.c_int(wid), _dp(d)))

    def set_comm(self, comm):
        """Partition over comm's ranks at initialize() (every rank binds the same scene)."""
        self.comm = comm   # the communicator must outlive the solver
        _chk(lib().aa_elastic_set_comm(self.h, comm.h if comm is not None else None))

    def initialize(self, settings: Settings):
        _chk(lib().aa_elastic_initialize(self.h, C.byref(settings)))
        self.settings = settings

    def save(self, result_dir="./result"):
        """Solver::save() (Solver.hpp:130-155): result_dir/residual-<m>.txt (residual-no.txt
        without acceleration), one row per iteration of the last step -- time (ms since the step
        started, device clock), prim, comb and, for the (u,x) variant (admm_anderson_hard_zxu),
        the reject flag; numbers as `ofs << setprecision(16)` writes them (%.16g)."""
        st = self.settings
        h = self.history()
        t = self.times()
        rej = h["reject"] if st.variant == AA_VARIANT_UX else None
        return write_residual_file(result_dir, st.anderson_m if st.acceleration_type else 0, t, h["prim"], h["comb"], rej)

    def step(self):
        _chk(lib().aa_elastic_step(self.h))

    def num_nodes(self):
        n = C.c_int()
        _chk(lib().aa_elastic_num_nodes(self.h, C.byref(n)))
        return n.value

    @property
    def x(self):
        out = np.zeros(3 * self.num_nodes())
        _chk(lib().aa_elastic_get_x(self.h, _dp(out)))
        return out.reshape(-1, 3)

    @property
    def v(self):
        out = np.zeros(3 * self.num_nodes())
        _chk(lib().aa_elastic_get_v(self.h, _dp(out)))
        return out.reshape(-1, 3)

    def set_state(self, x, v):
        """Solver::m_x / m_v assignment between steps (positions and velocities, n x 3)."""
        x = np.ascontiguousarray(x, np.float64).reshape(-1)
        v = np.ascontiguousarray(v, np.float64).reshape(-1)
        _chk(lib().aa_elastic_set_x(self.h, _dp(x)))
        _chk(lib().aa_elastic_set_v(self.h, _dp(v)))

    def history(self, cap=100000):
        p, c, r = np.zeros(cap), np.zeros(cap), np.zeros(cap, np.int32)
        n = C.c_int()
        _chk(lib().aa_elastic_get_history(self.h, _dp(p), _dp(c), _ip(r), C.c_int(cap), C.byref(n)))
        k = min(n.value, cap)
        return dict(prim=p[:k].copy(), comb=c[:k].copy(), reject=r[:k].copy())

    def times(self, cap=100000):
        """Device-clock ms from the start of the last step to the end of each recorded iteration."""
        t = np.zeros(cap)
        n = C.c_int()
        _chk(lib().aa_elastic_get_times(self.h, _dp(t), C.c_int(cap), C.byref(n)))
        return t[:min(n.value, cap)].copy()

    def set_iterations(self, admm_iters, eps_rel=0.0):
        """Settings::admm_iters and the run-to-epsilon stop of later steps (no re-factor)."""
        _chk(lib().aa_elastic_set_iterations(self.h, C.c_int(admm_iters), C.c_double(eps_rel)))

    def runtime(self) -> Runtime:
        rt = Runtime()
        _chk(lib().aa_elastic_runtime(self.h, C.byref(rt)))
        return rt

    def bench_iterations(self, iters):
        ms = C.c_double()
        _chk(lib().aa_elastic_bench_iterations(self.h, C.c_int(iters), C.byref(ms)))
        return ms.value

    def setup_phases(self):
        """{phase: ms} of the last initialize() (aa_elastic_setup_phases), in order."""
        names = C.create_string_buffer(4096)
        ms = (C.c_double * 64)()
        n = C.c_int()
        _chk(lib().aa_elastic_setup_phases(self.h, names, 4096, ms, 64, C.byref(n)))
        keys = names.value.decode().split("\n") if n.value else []
        return {k: round(ms[i], 1) for i, k in enumerate(keys[:64])}

    def kernel_stats(self, name):
        a, b, n = C.c_double(), C.c_double(), C.c_int()
        _chk(lib().aa_elastic_kernel_stats(self.h, name.encode(), C.byref(a), C.byref(b), C.byref(n)))
        return dict(avg_ms=a.value, bytes=b.value, launches=n.value)

    def local_stats(self, reset=True):
        """Work-queue diagnostics of the hyperelastic local step (AA_LQ_STATS=1 at initialize):
        the per-element L-BFGS iteration histogram and the trip / refill / wave counts."""
        out = np.zeros(104, np.int64)
        n = C.c_int()
        _chk(lib().aa_elastic_local_stats(self.h, out.ctypes.data_as(C.POINTER(C.c_longlong)), C.c_int(104),
                                          C.c_int(1 if reset else 0), C.byref(n)))
        return dict(hist=out[:101].copy(), trips=int(out[101]), refills=int(out[102]), waves=int(out[103]))


def solver_from_scene(ctx: Context, scene, comm=None) -> Solver:
    """Binds a scenes.Scene the way binding::add_trimesh/add_tetmesh + the samples do."""
    s = Solver(ctx)
    if comm is not None:
        s.set_comm(comm)
    s.add_nodes(scene.x, np.repeat(np.asarray(scene.masses, np.float64), 3))
    for g in scene.groups:
        lame = Lame.from_young(g.E, g.nu, g.limit_min, g.limit_max)
        if g.kind == 0:
            s.add_tets(scene.rest_x, g.idx, g.material, lame)
        else:
            s.add_tris(scene.rest_x, g.idx, lame)
    s.set_pins(scene.pin_idx, scene.pin_pts)
    for kind, prm in getattr(scene, "obstacles", []):
        s.add_obstacle(kind, prm)
    if getattr(scene, "collision_idx", None) is not None:
        s.set_collisions(scene.collision_idx)
    for tris, direction in getattr(scene, "winds", []):
        s.add_wind(tris, direction)
    return s


def settings_from_scene(scene) -> Settings:
    return Settings(timestep_s=scene.dt, admm_iters=scene.iters, gravity=scene.gravity, anderson_m=scene.aa_m,
                    penalty=scene.penalty, acceleration_type=ANDERSON if scene.accel else NOACC,
                    variant=scene.variant, verbose=0)


def run_scene(ctx: Context, scene, n_steps=None, comm=None):
    """Runs the scene like the reference driver; returns per-step dicts (prim, comb, reject, x, v)."""
    s = solver_from_scene(ctx, scene, comm)
    s.initialize(settings_from_scene(scene))
    out = []
    n_steps = scene.n_steps if n_steps is None else n_steps
    for k in range(1, n_steps + 1):
        if np.any(scene.pin_vel != 0):
            s.set_pins(scene.pin_idx, scene.pin_pts + k * scene.pin_vel)
        s.step()
        h = s.history()
        h["x"], h["v"] = s.x, s.v
        rt = s.runtime()
        h["step_ms"] = rt.step_ms
        h["iterations"], h["rejects"] = rt.iterations, rt.rejects
        out.append(h)
    return out, s


# ------------------------------------------------------------------------------------------
# Geometry: ALMGeometrySolver<3> (Geometry/ALMGeometrySolver.h)
# ------------------------------------------------------------------------------------------

def write_residual_file(result_dir, anderson_m, *cols):
    """The residual-<m>.txt / residual-no.txt writer shared by Solver.save and GeomSolver.save:
    tab-separated columns, floats as %.16g (C++ setprecision(16), default float format), ints
    as %d; a None column is left out."""
    cols = [c for c in cols if c is not None]
    n = min(len(c) for c in cols)
    path = os.path.join(result_dir, f"residual-{anderson_m}.txt" if anderson_m > 0 else "residual-no.txt")
    with open(path, "w") as f:
        for i in range(n):
            f.write("\t".join(("%d" % c[i]) if np.issubdtype(np.asarray(c).dtype, np.integer) else ("%.16g" % c[i])
                              for c in cols) + "\n")
    return path


class GeomRuntime(C.Structure):
    _fields_ = [("setup_ms", C.c_double), ("factor_ms", C.c_double), ("solve_ms", C.c_double),
                ("iterations", C.c_int), ("accepted", C.c_int), ("rejects", C.c_int), ("n_points", C.c_int),
                ("nnz_factor", C.c_longlong), ("hard_cols", C.c_longlong), ("soft_cols", C.c_longlong),
                ("n_constraints", C.c_longlong)]


class GeomSolver:
    """Mirror of ALMGeometrySolver<3> (kind AA_GEOM_ALM) or GeometrySolver<3> (AA_GEOM_PLAIN):
    add_hard/soft constraints, add_*laplacian, add_closeness, setup_ADMM, solve_ADMM,
    get_solution, function_values_ / elapsed_time_."""

    def __init__(self, ctx: Context, kind=AA_GEOM_ALM):
        self.ctx = ctx
        self.h = C.c_void_p()
        self.n = 0
        _chk(lib().aa_geom_create_kind(ctx.h, C.c_int(kind), C.byref(self.h)))

    def close(self):
        if self.h:
            lib().aa_geom_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_ref_surface(self, V, F):
        V = np.ascontiguousarray(V, np.float64).reshape(-1)
        F = np.ascontiguousarray(F, np.int32).reshape(-1)
        i = C.c_int()
        _chk(lib().aa_geom_add_ref_surface(self.h, _dp(V), C.c_int(len(V) // 3), _ip(F), C.c_int(len(F) // 3),
                                           C.byref(i)))
        return i.value

    def add_constraints(self, hard, ctype, idx, weight=1.0, params=None):
        idx = np.ascontiguousarray(idx, np.int32)
        if idx.ndim == 1:
            idx = idx[:, None]
        count, k = idx.shape
        prm = None if params is None else np.ascontiguousarray(params, np.float64).reshape(count, -1)
        _chk(lib().aa_geom_add_constraints(self.h, C.c_int(int(hard)), C.c_int(ctype), _ip(idx), C.c_int(k),
                                           C.c_int(count), C.c_double(weight), None if prm is None else _dp(prm)))

    def add_laplacian(self, idx, coefs, weight, ref_points=None):
        i = np.ascontiguousarray(idx, np.int32)
        c = np.ascontiguousarray(coefs, np.float64)
        r = None if ref_points is None else np.ascontiguousarray(ref_points, np.float64).reshape(-1)
        _chk(lib().aa_geom_add_laplacian(self.h, _ip(i), _dp(c), C.c_int(len(i)), C.c_double(weight),
                                         None if r is None else _dp(r)))

    def add_closeness(self, idx, weight, target):
        t = np.ascontiguousarray(target, np.float64)
        _chk(lib().aa_geom_add_closeness(self.h, C.c_int(idx), C.c_double(weight), _dp(t)))

    def add_laplacians(self, row_ptr, idx, coefs, weights, relative=None, ref_points=None):
        """n_rows add_laplacian calls in one (CSR rows; relative[r] != 0: add_relative_laplacian)."""
        rp = np.ascontiguousarray(row_ptr, np.int32)
        i = np.ascontiguousarray(idx, np.int32)
        c = np.ascontiguousarray(coefs, np.float64)
        w = np.ascontiguousarray(weights, np.float64)
        rl = None if relative is None else np.ascontiguousarray(relative, np.int32)
        r = None if ref_points is None else np.ascontiguousarray(ref_points, np.float64).reshape(-1)
        _chk(lib().aa_geom_add_laplacians(self.h, C.c_int(len(rp) - 1), _ip(rp), _ip(i), _dp(c), _dp(w),
                                          None if rl is None else _ip(rl), None if r is None else _dp(r)))

    def add_closenesses(self, idx, weights, targets):
        i = np.ascontiguousarray(idx, np.int32)
        w = np.ascontiguousarray(weights, np.float64)
        t = np.ascontiguousarray(targets, np.float64).reshape(-1)
        _chk(lib().aa_geom_add_closenesses(self.h, C.c_int(len(i)), _ip(i), _dp(w), _dp(t)))

    def set_comm(self, comm):
        """Partition over comm's ranks at the first solve (every rank adds the same problem)."""
        self.comm = comm
        _chk(lib().aa_geom_set_comm(self.h, comm.h if comm is not None else None))

    def setup(self, n_points, penalty, spd=AA_SPD_LDLT):
        self.n = n_points
        _chk(lib().aa_geom_setup(self.h, C.c_int(n_points), C.c_double(penalty), C.c_int(spd)))

    def solve(self, init_x, rel_eps, max_iter, m):
        x = np.ascontiguousarray(init_x, np.float64).reshape(-1)
        _chk(lib().aa_geom_solve(self.h, _dp(x), C.c_double(rel_eps), C.c_int(max_iter), C.c_int(m)))

    def set_stop(self, at_eps=False, eps_rel=0.0):
        """Run-to-epsilon for later solves (aa_geom_set_stop): stop at the reference's
        commented-out criterion comb < rel_eps^2 hard_cols^2 2 and/or comb <= eps_rel comb_0."""
        _chk(lib().aa_geom_set_stop(self.h, C.c_int(1 if at_eps else 0), C.c_double(eps_rel)))

    def solution(self):
        out = np.zeros(3 * self.n)
        _chk(lib().aa_geom_get_solution(self.h, _dp(out)))
        return out.reshape(-1, 3)

    def history(self, cap=1 << 20):
        n = C.c_int()
        _chk(lib().aa_geom_get_history(self.h, None, None, C.c_int(0), C.byref(n)))
        k = n.value
        c, t = np.zeros(max(k, 1)), np.zeros(max(k, 1))
        _chk(lib().aa_geom_get_history(self.h, _dp(c), _dp(t), C.c_int(k), C.byref(n)))
        return dict(comb=c[:k].copy(), time_s=t[:k].copy())

    def save(self, anderson_m, result_dir="./result"):
        """ALMGeometrySolver::save(Anderson_m) (ALMGeometrySolver.h:343-365; GeometrySolver.h
        likewise): "elapsed_time_ <tab> function_values_" per recorded iteration."""
        h = self.history()
        return write_residual_file(result_dir, anderson_m, h["time_s"], h["comb"])

    def runtime(self) -> GeomRuntime:
        rt = GeomRuntime()
        _chk(lib().aa_geom_runtime_info(self.h, C.byref(rt)))
        return rt

    def closest_points(self, surface, P):
        P = np.ascontiguousarray(P, np.float64).reshape(-1)
        out = np.zeros_like(P)
        _chk(lib().aa_geom_closest_points(self.h, C.c_int(surface), _dp(P), C.c_int(len(P) // 3), _dp(out)))
        return out.reshape(-1, 3)

    def bench_iterations(self, iters):
        ms = C.c_double()
        _chk(lib().aa_geom_bench_iterations(self.h, C.c_int(iters), C.byref(ms)))
        return ms.value

    def kernel_stats(self, name):
        a, b, n = C.c_double(), C.c_double(), C.c_int()
        _chk(lib().aa_geom_kernel_stats(self.h, name.encode(), C.byref(a), C.byref(b), C.byref(n)))
        return dict(avg_ms=a.value, bytes=b.value, launches=n.value)


def geom_from_scene(ctx: Context, sc, comm=None, timings=None) -> GeomSolver:
    """Binds a geom_scenes.GeomScene the way optimize_mesh (PlanarityOpt.cpp / WireMeshOpt.cpp) does.
    timings (dict, optional) receives the wall ms of each binding phase."""
    import time
    t = [time.perf_counter()]

    def lap(name):
        t.append(time.perf_counter())
        if timings is not None:
            timings[name] = round((t[-1] - t[-2]) * 1e3, 1)
    g = GeomSolver(ctx, AA_GEOM_PLAIN if getattr(sc, "solver", "alm") == "plain" else AA_GEOM_ALM)
    lap("create_ms")
    if comm is not None:
        g.set_comm(comm)
    sids = [g.add_ref_surface(V, F) for V, F in sc.surfaces]
    for grp in sc.groups:
        prm = grp.params
        if grp.type in (AA_CON_POINT_TO_REF, AA_CON_REF_SURFACE):   # scene surface ids -> solver ids
            prm = np.asarray(sids, np.float64)[np.asarray(prm).reshape(grp.count, -1)[:, 0].astype(np.int64)][:, None]
        g.add_constraints(grp.hard, grp.type, grp.idx, grp.weight, prm)
    lap("surfaces_constraints_ms")
    # regularisation rows in insertion order, one batched call per run of laplacian (kinds 0, 1)
    # or closeness (kind 2) rows -- the same rows as one add_* call each
    kind = np.asarray(sc.reg_kind, np.int32)
    ptr = np.asarray(sc.reg_ptr, np.int64)
    i = 0
    while i < len(kind):
        clo = kind[i] == 2
        j = i + 1
        while j < len(kind) and (kind[j] == 2) == clo:
            j += 1
        if clo:
            g.add_closenesses(np.asarray(sc.reg_idx)[ptr[i:j]], np.asarray(sc.reg_weight)[i:j],
                              np.asarray(sc.reg_target)[i:j])
        else:
            a, b = int(ptr[i]), int(ptr[j])
            rel = kind[i:j] == 1
            g.add_laplacians(ptr[i:j + 1] - a, np.asarray(sc.reg_idx)[a:b], np.asarray(sc.reg_coef)[a:b],
                             np.asarray(sc.reg_weight)[i:j], rel.astype(np.int32) if rel.any() else None,
                             sc.ref_points if rel.any() else None)
        i = j
    lap("regularization_ms")
    g.setup(sc.n_points, sc.penalty)
    lap("setup_admm_ms")
    return g


def run_geom(ctx: Context, sc, comm=None):
    """setup_ADMM + solve_ADMM of a GeomScene; returns dict(comb, time_s, x) and the solver."""
    g = geom_from_scene(ctx, sc, comm)
    g.solve(sc.x0, 1e-8 * max(sc.avg_edge_length(), 1e-300), sc.iters, sc.aa_m)
    h = g.history()
    h["x"] = g.solution()
    return h, g


# ------------------------------------------------------------------------------------------
# element-level test hooks (aa_test_*): the device prox / COD / projection functions
# ------------------------------------------------------------------------------------------

def hook_prox(ctx: Context, op, prm4, X):
    """op 0 linear tet, 1 NeoHookean, 2 StVK (prm4 = E, nu, h), 3 / 4 tri H / X prox (prm4[2:] =
    limits); X (n, 9|6). Returns (out, L-BFGS iterations)."""
    X = np.ascontiguousarray(X, np.float64)
    n = X.shape[0]
    out, it = np.zeros_like(X), np.zeros(n, np.int32)
    p = np.ascontiguousarray(prm4, np.float64)
    _chk(lib().aa_test_prox(ctx.h, C.c_int(op), _dp(p), _dp(X), C.c_int(n), _dp(out), _ip(it)))
    return out, it


def hook_cod_solve(ctx: Context, M, b):
    Mc = np.asfortranarray(M, np.float64).ravel(order="F").copy()
    bb = np.ascontiguousarray(b, np.float64)
    th = np.zeros(len(bb))
    _chk(lib().aa_test_cod_solve(ctx.h, C.c_int(len(bb)), _dp(Mc), _dp(bb), _dp(th)))
    return th


def hook_geom_project(ctx: Context, ctype, k, params, P):
    """P (n, cols, 3) transformed points; params (2,) (angle min/max or edge length)."""
    P = np.ascontiguousarray(P, np.float64)
    out = np.zeros_like(P)
    prm = np.zeros(2)
    if params is not None:
        a = np.atleast_1d(np.asarray(params, np.float64))
        prm[:len(a)] = a
    _chk(lib().aa_test_geom_project(ctx.h, C.c_int(ctype), C.c_int(k), _dp(prm), _dp(P), C.c_int(P.shape[0]), _dp(out)))
    return out

