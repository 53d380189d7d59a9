#!/usr/bin/env python3
"""Benchmark of the admm-elastic hot path on MI355X (BASELINE.json metric: ADMM iterations/s
and time-to-epsilon).

Default workload (BASELINE.json configs[3], the 1M-tet elastic drop that north_star's target
names for 1/2/4/8 GPUs): make_tet_blocks(100,40,50) = 1 000 000 NeoHookean tets, 211 191 nodes,
initial pose squashed 0.9 in y, free fall, z-Anderson m=6 (admm_anderson_xzu order), dt = 1/30,
100 ADMM iterations per time step. --config c2: cloth drop make_tri_blocks(112,112) = 50 176
triangles, (u,x)-Anderson m=6 (configs[1]); c3 / c5: the Geometry ALM configs.
A bench "step" is one Solver::step() time step; `value` = ADMM iterations executed / max-over-
ranks wall time. Synthetic input (generated mesh, no datasets).

Multi-GPU: one process per GPU (torch.distributed.run as the launcher only: the ranks never import
torch, see aa-admm_amd/rdzv.py). Elastic configs partition ONE mesh over the ranks
(--partition rccl, the default for N>1: nested-dissection parts, separator rows of the global
solve and all residual/Anderson partials all-reduced on RCCL over xGMI; strong scaling);
--partition none runs independent replicas (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--iters 100] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import statistics
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.3 TB/s is the measured copy ceiling
EPS_ELASTIC = 1e-8      # time-to-epsilon: comb <= 1e-8 * comb_0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--iters", type=int, default=100)
    p.add_argument("--nx", type=int, default=112)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-iters", type=int, default=40)
    p.add_argument("--config", default="c4", choices=["c2", "c3", "c4", "c5"],
                   help="c4 (default): 1M-tet NeoHookean block drop (configs[3]) -- the workload north_star's "
                        "target names for 1/2/4/8 GPUs; c2: cloth 50k tris (configs[1]); c3: planar-quad 317x317 "
                        "(configs[2]); c5: wire mesh 707x707 (configs[4])")
    p.add_argument("--tets", type=str, default="100,40,50", help="c4 block size in cubes (5 tets per cube)")
    p.add_argument("--mesh", default="block", choices=["block", "bunny"],
                   help="c4 mesh: make_tet_blocks (default) or the voxelised bunny configs[3] names "
                        "(scenes.bunny_drop, --bunny-res cells along its longest side: 100 = 1 002 780 tets)")
    p.add_argument("--bunny-res", type=int, default=100)
    p.add_argument("--partition", default="auto", choices=["auto", "none", "rccl", "host"],
                   help="N>1: partition ONE mesh over the ranks (rccl: RCCL over xGMI, one "
                        "GPU per rank; host: host-staged gloo transport, for rehearsals with several ranks on one "
                        "GPU) or run independent replicas (none). auto = rccl when N>1")
    p.add_argument("--same-device", action="store_true", help="all ranks on GPU 0 (rehearsal with --partition host)")
    p.add_argument("--eps-steps", type=int, default=-1,
                   help="run-to-epsilon leg: time steps run with the reference's default cap of 500 ADMM iterations "
                        "(Solver.hpp:62-65) and the stop comb <= 1e-8 comb_0; -1 (default) = the same time steps as "
                        "the timed region (--steps); 0 = skip")
    p.add_argument("--eps-cap", type=int, default=500)
    p.add_argument("--geom-eps-cap", type=int, default=2000,
                   help="geometry run-to-epsilon leg: accepted-iteration cap of the solves that stop at the reference's "
                        "residual_eps (ALMGeometrySolver.h:172)")
    p.add_argument("--geom-eps-solves", type=int, default=2, help="geometry run-to-epsilon solves (0 = skip)")
    p.add_argument("--no-secondary", action="store_true",
                   help="c4 only: skip the secondary C3 (planar-quad, configs[2]) object in the same JSON line")
    p.add_argument("--rehearse", type=int, default=0, metavar="P",
                   help="c4/c2, one GPU: time ONE rank's share of a P-way mesh partition (aa_comm_create_solo: "
                        "collectives replaced by local stand-ins, so the numbers are not a solution) -- the "
                        "per-rank kernel time of a P-GPU run, for the DESIGN.md scaling projection")
    p.add_argument("--rehearse-rank", type=int, default=0)
    p.add_argument("--launch-check", action="store_true",
                   help="print the rank layout this invocation runs with (after the --gpus N launch) and exit "
                        "without touching a GPU -- CPU test of the multi-rank launcher")
    p.add_argument("--lq-stats", action="store_true",
                   help="c4: count the local step's L-BFGS iterations per element and its work-queue trips over "
                        "the timed steps (AA_LQ_STATS=1; atomics in the kernel, so not for the timed number)")
    return p.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n):
    """`--gpus N` without an outside launcher: start N ranks (one process per GPU) through
    torch.distributed.run as a CHILD process -- this process has made no HIP call yet and never
    makes one -- relay its output (rank 0 prints the JSON line) and exit with its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"[bench] --gpus {n}: launching {n} ranks (torch.distributed.run)", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def dist_setup(n_gpus):
    """(world, rank, local rank, group, runtime report). A rank process never imports torch
    (torch.distributed.run is only the launcher): libaa_admm.so is loaded and checked against the
    ROCm runtime it was built for BEFORE the rendezvous (aa-admm_amd/dist.py rank_setup), which is
    a torch-free socket group (aa-admm_amd/rdzv.py) -- RCCL id broadcast, barriers, timing max."""
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != n_gpus:
        raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']} "
                         "(the launcher and the flag must agree)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pkg = importlib.import_module("aa-admm_amd")
    group, report = pkg.dist.rank_setup()
    return world, rank, local, group, report


def allreduce(group, val, op):
    return group.allreduce_scalar(val, op)


def barrier(group, ctx):
    ctx.synchronize()
    group.barrier()
    ctx.synchronize()


def run_logged(cmd, cwd, env, timeout):
    """subprocess.run with a heartbeat on stderr every 30 s (long CPU-baseline legs must not look
    hung to a supervisor that watches the output)."""
    p = subprocess.Popen(cmd, cwd=cwd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    t0 = time.time()
    while True:
        try:
            out, err = p.communicate(timeout=30)
            return subprocess.CompletedProcess(cmd, p.returncode, out, err)
        except subprocess.TimeoutExpired:
            el = time.time() - t0
            print(f"[bench] {os.path.basename(cmd[0])} running for {el:.0f} s", file=sys.stderr, flush=True)
            if el > timeout:
                p.kill()
                p.communicate()
                raise


def host_info():
    """CPU the baseline runs on: nproc, model, threads used and their binding."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "model": model}


def cpu_threads():
    """All the CPUs this job may use: OMP_NUM_THREADS when the launcher sets it (the GPU box
    allots 16 CPUs per job and exports it), else every CPU of the host."""
    return int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1)))


def cpu_env(threads):
    return dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES="cores")


def cpu_sample(sc):
    """The REFERENCE (oracle/_ref/ref_elastic_{h,x}, compiled from the reference's own sources) on
    the host cores, bounded sample `sc`; the first time step (OpenMP spin-up, Anderson
    allocation) is excluded. Returns (median iters/s of the other steps, wall s incl. setup, kind)."""
    scenes = importlib.import_module("aa-admm_amd.scenes")
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import refio  # test infrastructure: the reference driver's file format
    drv = os.path.join(REPO, "oracle", "_ref", "ref_elastic_h" if sc.variant == scenes.VARIANT_H else "ref_elastic_x")
    threads = cpu_threads()
    with tempfile.TemporaryDirectory() as tmp:
        refio.write_scene(sc, os.path.join(tmp, "s.bin"))
        if os.path.exists(drv):
            t0 = time.time()
            r = run_logged([drv, "s.bin", "o.bin"], tmp, cpu_env(threads), 900)
            wall = time.time() - t0
            if r.returncode != 0:
                raise RuntimeError(r.stderr[-500:])
            steps = refio.read_ref_result(os.path.join(tmp, "o.bin"), sc.n_nodes)
            kind = "reference"
        else:  # reference binary absent: time our own C++ restatement instead
            import pyoracle
            t0 = time.time()
            steps = pyoracle.run_elastic(sc)
            wall = time.time() - t0
            kind, threads = "port", 1
    per = [len(s["prim"]) / (s["step_ms"] / 1000.0) for s in steps[1:]]
    return statistics.median(per), wall, kind, threads


def cpu_baseline(sc):
    raw, wall, kind, threads = cpu_sample(sc)
    return {"value": round(raw, 3), "unit": "ADMM iters/s", "cores": threads, "kind": kind,
            "host": {**host_info(), "OMP_NUM_THREADS": threads, "OMP_PROC_BIND": "close", "OMP_PLACES": "cores"},
            "sample": f"{sc.name} ({sc.n_elements()} elements), {sc.n_steps} steps x {sc.iters} ADMM iters, "
                      f"m={sc.aa_m}; median iters/s of steps 2-{sc.n_steps} (step 1 = warm-up); wall incl. setup "
                      f"{wall:.1f} s"}


def make_comm(pkg, ctx, args, world, rank, group):
    """Communicator of a mesh-partitioned run (None for replicas)."""
    part = args.partition if args.partition != "auto" else ("rccl" if world > 1 else "none")
    comm = None
    if getattr(args, "rehearse", 0) > 1 and world == 1:
        return (pkg.capi.Comm.solo(args.rehearse_rank, args.rehearse),
                f"solo rehearsal: rank {args.rehearse_rank} of {args.rehearse}, collectives replaced")
    if part == "rccl":
        try:
            comm = pkg.dist.rccl_comm(ctx, group)
        except Exception as e:   # transport only: the compute stays on the GPUs either way
            print(f"[bench] RCCL communicator failed ({e}); using the host-staged transport", file=sys.stderr)
            part = "host (rccl init failed)"
            comm = pkg.dist.host_comm(group)
    elif part == "host":
        comm = pkg.dist.host_comm(group)
    return comm, part


def geom_scene(args):
    gs = importlib.import_module("aa-admm_amd.geom_scenes")
    if args.config == "c3":
        n = args.nx if args.nx != 112 else 317
        return (gs.pq_heightfield(n, n, iters=args.iters, aa_m=10, noise=0.3),
                f"planar-quad height field {n}x{n} quads, initial points scattered 0.3 h off the surface")
    n = args.nx if args.nx != 112 else 707
    return gs.wire_grid(n, n, iters=args.iters, aa_m=20), f"wire mesh height field {n}x{n} quads"


def geom_cpu_baseline(args):
    """The REFERENCE's ALMGeometrySolver (oracle/_ref/ref_geom, compiled from its own sources) on
    the host cores, bounded sample: the same scene with a reduced iteration count."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import refio  # test infrastructure: the reference driver's file format
    # bounded sample (~10-30 s of CPU work): the 500k-point wire mesh costs ~0.6 s per reference
    # iteration plus two LDLT factorisations, so it gets fewer iterations than the PQ mesh
    iters = args.cpu_iters if args.config == "c3" else min(args.cpu_iters, 10)
    sc, _ = geom_scene(argparse.Namespace(**{**vars(args), "iters": iters}))
    drv = os.path.join(REPO, "oracle", "_ref", "ref_geom")
    threads = cpu_threads()
    if not os.path.exists(drv):
        return {"value": None, "error": "oracle/_ref/ref_geom not built"}
    with tempfile.TemporaryDirectory() as tmp:
        refio.write_geom_scene(sc, os.path.join(tmp, "s.bin"))
        r = run_logged([drv, "s.bin", "o.bin"], tmp, cpu_env(threads), 900)
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-500:])
        res = refio.read_geom_result(os.path.join(tmp, "o.bin"), sc.n_points)
    return {"value": round(len(res["comb"]) / res["loop_s"], 3), "unit": "ADMM iters/s", "cores": threads,
            "kind": "reference", "setup_s": round(res["setup_s"], 3),
            "host": {**host_info(), "OMP_NUM_THREADS": threads, "OMP_PROC_BIND": "close", "OMP_PLACES": "cores"},
            "sample": f"{sc.name}: one solve_ADMM of {iters} accepted iterations (m={sc.aa_m}), loop time "
                      f"(setup excluded, as ALMGeometrySolver.h:194-195)"}


MALL_BYTES = 256e6   # MI355X Infinity Cache: working sets below it are flagged cache-resident


def geom_line(args, world, rank, local, group):
    """configs[2] / configs[4]: one bench step = one solve_ADMM of `iters` accepted ALM iterations
    (inputs resident on the device after setup); value = accepted iterations / wall time.
    Returns the JSON line (rank 0) or None."""
    pkg = importlib.import_module("aa-admm_amd")
    capi = pkg.capi
    ctx = capi.Context(0 if args.same_device else local)
    sc, desc = geom_scene(args)
    comm, part = make_comm(pkg, ctx, args, world, rank, group)
    lib_first_use_ms = ctx.warm_dense()   # one-time rocBLAS / rocSOLVER load, outside setup_ms
    t0 = time.time()
    bind_phases = {}
    g = capi.geom_from_scene(ctx, sc, comm, bind_phases)   # add_*_constraint + setup_ADMM (rows, weights)
    bind_ms = (time.time() - t0) * 1e3
    eps = 2.0 * (1e-8 * sc.avg_edge_length() * sc.hard_cols()) ** 2   # ALMGeometrySolver.h:173 (commented stop)
    t1 = time.time()
    g.solve(sc.x0, 1e-8 * sc.avg_edge_length(), sc.iters, sc.aa_m)   # first solve also orders + factors
    first_ms = (time.time() - t1) * 1e3
    rt0 = g.runtime()
    t1 = time.time()
    for _ in range(max(1, args.warmup) - 1):
        g.solve(sc.x0, 1e-8 * sc.avg_edge_length(), sc.iters, sc.aa_m)
    warm_ms = (time.time() - t1) * 1e3
    # setup = what the reference's setup_ADMM does (rows + LDLT): binding/setup_ADMM here plus the
    # ordering, factorization and uploads done at the first solve; the first solve's loop (graph
    # capture, Anderson buffers) and the warm-up solves are reported beside it, not in it
    setup_ms = bind_ms + rt0.factor_ms
    setup_breakdown = {"bind_and_setup_admm_ms": round(bind_ms, 1), "bind_phases_ms": bind_phases,
                       "setup_admm_cpp_ms": round(rt0.setup_ms, 1),
                       "order_factor_upload_ms": round(rt0.factor_ms, 1),
                       "first_solve_loop_ms": round(first_ms - rt0.factor_ms, 1),
                       "warmup_solves_ms": round(warm_ms, 1), "warmup_solves": max(1, args.warmup) - 1,
                       "library_first_use_ms": round(lib_first_use_ms, 1)}
    print(f"[bench] {args.config} setup {setup_ms / 1e3:.2f} s ({setup_breakdown})", file=sys.stderr, flush=True)
    barrier(group, ctx)
    t0 = time.perf_counter()
    acc, xupd, tte, tte_rel = 0, 0, [], []
    for _ in range(args.steps):
        g.solve(sc.x0, 1e-8 * sc.avg_edge_length(), sc.iters, sc.aa_m)
        rt = g.runtime()
        acc += rt.accepted
        xupd += rt.iterations
        h = g.history()
        hit = np.nonzero(h["comb"] <= eps)[0]
        tte.append((int(hit[0]) + 1, float(h["time_s"][hit[0]] * 1e3)) if len(hit) else None)
        rel = {}
        for r in (1e-2, 1e-4, 1e-6):   # relative levels: comb <= r * comb_0 (the absolute stop is rarely met)
            hr = np.nonzero(h["comb"] <= r * h["comb"][0])[0] if len(h["comb"]) else []
            rel[str(r)] = {"iters": int(hr[0]) + 1, "ms": round(float(h["time_s"][hr[0]] * 1e3), 3)} if len(hr) else None
        tte_rel.append(rel)
    barrier(group, ctx)
    elapsed = time.perf_counter() - t0
    elapsed_max = allreduce(group, elapsed, "max")
    # replicas: independent copies (weak scaling); partitioned: one problem (strong scaling)
    acc_all = float(acc) if comm is not None else allreduce(group, float(acc), "sum")
    geps = geom_run_to_eps(g, sc, eps, args) if args.geom_eps_solves > 0 else None
    value = acc_all / elapsed_max
    roof, cpu, line = None, None, None
    if comm is not None:
        g.bench_iterations(min(sc.iters, 50))
    if rank == 0:
        if comm is None:
            g.bench_iterations(min(sc.iters, 50))
        stats = {k: g.kernel_stats(k) for k in ("z", "rhs", "solve", "u", "aa")}
        # roofline kernel: the global solve (HBM-bound triangular sweeps, 3 RHS). k_geo_z is
        # reported against its own bound below: a per-lane BVH traversal + 3xk SVDs is latency-
        # and divergence-bound, an HBM fraction would say nothing about it.
        st = stats["solve"]
        achieved = st["bytes"] / (st["avg_ms"] * 1e-3) / 1e9 if st["avg_ms"] > 0 else 0.0
        factor_b = 8.0 * rt0.nnz_factor
        roof = {"kernel": "global solve: multifrontal triangular solves (3 RHS)", "bound": "hbm",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "avg_launch_us": round(st["avg_ms"] * 1e3, 2), "bytes_per_launch": st["bytes"],
                "factor_bytes": factor_b, "cache_resident": bool(factor_b < MALL_BYTES),
                "note": ("factor fits the 256 MB Infinity Cache: the sweeps re-read it from MALL, so this "
                         "fraction of HBM peak overstates nothing but is not an HBM-bound figure either")
                        if factor_b < MALL_BYTES else "factor larger than the Infinity Cache: streamed from HBM",
                "phase_us_per_iter": {kk: round(v["avg_ms"] * 1e3, 2) for kk, v in stats.items()},
                "phase_bytes_per_iter": {kk: v["bytes"] for kk, v in stats.items()},
                "dominant_phase": max(stats, key=lambda kk: stats[kk]["avg_ms"])}
        try:
            cp = ctx.bench_read(2 << 30)
            roof["read_peak_measured"] = round(cp, 1)
            roof["frac_of_read_peak"] = round(achieved / cp, 4) if cp > 0 else None
        except Exception as e:
            roof["read_peak_measured"] = None
            roof["read_peak_error"] = str(e)[:120]
        z = stats["z"]
        ncon = int(rt0.n_constraints)
        roof["projections"] = {"kernel": "k_geo_z (constraint projections + rhs slot rows)",
                               "bound": "latency/divergence (per-lane BVH traversal, 3xk Jacobi SVDs)",
                               "avg_launch_us": round(z["avg_ms"] * 1e3, 2), "constraints": ncon,
                               "ns_per_constraint": round(z["avg_ms"] * 1e6 / max(ncon, 1), 3)}
        if world == 1 and not args.no_cpu_baseline:
            print(f"[bench] timing the reference CPU baseline ({args.config})", file=sys.stderr, flush=True)
            try:
                cpu = geom_cpu_baseline(args)
            except Exception as e:
                cpu = {"value": None, "error": str(e)[:200]}
        tt = [t[1] for t in tte if t is not None]
        line = {
            "metric": "ADMM iters/sec + time-to-eps (primal+dual residual)", "value": round(value, 2),
            "unit": "ADMM iters/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed_max * 1e3 / args.steps, 3), "higher_is_better": True,
            "scaling": "strong" if comm is not None else "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (generated height-field quad mesh)",
            "config": {"workload": f"{desc}, ALM + Anderson m={sc.aa_m}, {sc.iters} accepted iterations per solve "
                                   f"(BASELINE configs[{2 if args.config == 'c3' else 4}])",
                       "points": sc.n_points, "hard_cols": sc.hard_cols(), "anderson_m": sc.aa_m,
                       "parallelism": (f"mesh-partitioned{world} ({part})" if comm is not None else f"replicas{world}"),
                       "global_solve": "supernodal direct",
                       "nnz_factor": rt0.nnz_factor, "setup_ms": round(setup_ms, 1),
                       "factor_ms": round(rt0.factor_ms, 1), "setup_breakdown": setup_breakdown},
            "accepted_iters": int(acc_all), "x_updates": int(xupd),
            "time_to_eps_ms": all_steps_median([t[1] if t else None for t in tte]),
            "time_to_eps": {"eps_abs": eps, "criterion": "comb <= 2 (1e-8 avg_edge hard_cols)^2 (ALMGeometrySolver.h:173)",
                            "steps": len(tte), "reached": len(tt),
                            "iters_to_eps": [t[0] if t else None for t in tte],
                            "relative": {r: {"reached": sum(1 for x in tte_rel if x[r]),
                                             "median_ms": all_steps_median([x[r]["ms"] if x[r] else None for x in tte_rel]),
                                             "iters": [x[r]["iters"] if x[r] else None for x in tte_rel]}
                                         for r in ("0.01", "0.0001", "1e-06")},
                            "clock": "device wall_clock64 from the loop start (elapsed_time_)"},
            "run_to_eps": geps,
            "roofline": roof, "cpu_baseline": cpu,
        }
        if geps is not None:   # the headline time-to-eps: the run-to-eps leg (all solves, unreached = "> cap")
            line["time_to_eps_ms"] = geps["median_ms"]
    g.close()
    if comm is not None:
        comm.close()
    ctx.close()
    return line


def geom_run_to_eps(g, sc, eps, args):
    """Geometry run-to-epsilon leg: solves with a raised accepted-iteration cap that stop on the
    device at the reference's residual_eps (ALMGeometrySolver.h:172 -- computed there, its test
    commented out at :258-260). Relative levels (comb <= r comb_0) are read from the same curve."""
    rel_eps = 1e-8 * sc.avg_edge_length()
    g.set_stop(True, 0.0)
    runs = []
    try:
        for _ in range(args.geom_eps_solves):
            t0 = time.perf_counter()
            g.solve(sc.x0, rel_eps, args.geom_eps_cap, sc.aa_m)
            wall = (time.perf_counter() - t0) * 1e3
            rt = g.runtime()
            h = g.history()
            comb, ts = h["comb"], h["time_s"]
            hit = np.nonzero(comb < eps)[0]
            run = {"accepted": int(rt.accepted), "x_updates": int(rt.iterations), "solve_wall_ms": round(wall, 1),
                   "eps_abs": None if not len(hit) else {"iters": int(hit[0]) + 1, "ms": round(float(ts[hit[0]] * 1e3), 3)},
                   "final_comb": float(comb[-1]) if len(comb) else None,
                   "min_comb_over_eps": float(comb.min() / eps) if len(comb) else None}
            for r in (1e-4, 1e-6, 1e-8):
                hr = np.nonzero(comb <= r * comb[0])[0] if len(comb) else []
                run[f"rel_{r:g}"] = {"iters": int(hr[0]) + 1, "ms": round(float(ts[hr[0]] * 1e3), 3)} if len(hr) else None
            runs.append(run)
    finally:
        g.set_stop(False, 0.0)
    hit_ms = [r["eps_abs"]["ms"] for r in runs if r["eps_abs"]]
    out = {"criterion": "comb < 2 (1e-8 avg_edge hard_cols)^2 (ALMGeometrySolver.h:172; its stop is commented out "
                        "at :258-260, enabled here by aa_geom_set_stop)", "eps_abs": eps, "cap_accepted": args.geom_eps_cap,
           "solves": len(runs), "reached": len(hit_ms),
           "median_ms": all_steps_median([r["eps_abs"]["ms"] if r["eps_abs"] else None for r in runs]),
           "median_ms_reached_only": round(statistics.median(hit_ms), 3) if hit_ms else None,
           "clock": "device wall_clock64 from the loop start (elapsed_time_)", "per_solve": runs}
    if args.config == "c3" and sc.n_points == 101124:
        out["reference_regime"] = (
            "pinned (tests/golden/eps_pq317_ref.npz, test_gpu_c3_eps_regime_matches_reference): the reference run to "
            "1500 iterations reaches eps_abs at 1332 unperturbed and at 1145 when started 1e-13 off "
            "(profiles/r5_c3_ref_curve1500*.json): the curve branches at iteration ~1069 on rounding-level "
            "differences; the GPU follows the 1145 branch to 1e-4 relative, and both agree to 9e-11 comb_0 before it")
    if not hit_ms:
        out["note"] = (f"not reached in {len(runs)}/{len(runs)} solves with cap {args.geom_eps_cap} accepted iterations; "
                       f"min comb / eps_abs = {min(r['min_comb_over_eps'] for r in runs):.3g}")
    return out


def main_geom(args, world, rank, local, group, report):
    line = geom_line(args, world, rank, local, group)
    if line is not None:
        line["runtime_libs"] = report["bound"]
        print(json.dumps(line))
    group.close()


def elastic_scene(args, iters=None, n_steps=1):
    scenes = importlib.import_module("aa-admm_amd.scenes")
    it = args.iters if iters is None else iters
    if args.config == "c4" and args.mesh == "bunny":
        sc = scenes.bunny_drop(args.bunny_res, iters=it, n_steps=n_steps)
        return sc, (f"NeoHookean voxelised bunny free fall (bunny_closed.obj, {args.bunny_res} cells across, 5 "
                    f"make_tet_blocks tets per cell) {sc.n_elements()} tets, {sc.n_nodes} nodes, squashed 0.9 in y, "
                    f"z-AA (X order) m=6, {it} ADMM iters/step, dt=1/30 (BASELINE configs[3])")
    if args.config == "c4":
        cx, cy, cz = (int(v) for v in args.tets.split(","))
        sc = scenes.tet_drop(cx, cy, cz, iters=it, n_steps=n_steps)
        return sc, (f"NeoHookean block free fall make_tet_blocks({cx},{cy},{cz}) {sc.n_elements()} tets, "
                    f"{sc.n_nodes} nodes, squashed 0.9 in y, z-AA (X order) m=6, {it} ADMM iters/step, dt=1/30 "
                    f"(BASELINE configs[3])")
    sc = scenes.cloth(args.nx, args.nx, iters=it, n_steps=n_steps)
    return sc, (f"cloth drop make_tri_blocks({args.nx},{args.nx}) {sc.n_elements()} tris, (u,x)-AA m=6, "
                f"{it} ADMM iters/step, dt=1/30 (BASELINE configs[1])")


def elastic_cpu_baseline(args):
    scenes = importlib.import_module("aa-admm_amd.scenes")
    if args.config != "c4":
        return cpu_baseline(scenes.cloth(args.nx, args.nx, iters=args.cpu_iters, n_steps=3))
    # the reference cannot factor the 1M-tet system within a bench run (Eigen SimplicialLDLT of
    # ~633k dof, serial: tens of minutes). Two samples of the same recipe
    # (64k and 202k tets, 3 steps x 10 iterations each) give the per-iteration cost's growth
    # t(T) = a T^b; value = the fit at the workload's tet count.
    cx, cy, cz = (int(v) for v in args.tets.split(","))
    T = 5.0 * cx * cy * cz
    pts, notes = [], []
    for dims in ((40, 16, 20), (60, 24, 28)):
        sc = scenes.tet_drop(*dims, iters=10, n_steps=3)
        if pts and pts[-1]["wall_s"] > 90:   # a slow host: the larger sample would take > ~5 min
            notes.append(f"{sc.name} skipped (the smaller sample took {pts[-1]['wall_s']} s)")
            break
        print(f"[bench] reference CPU sample {sc.name} ({sc.n_elements()} tets)", file=sys.stderr, flush=True)
        raw, wall, kind, threads = cpu_sample(sc)
        pts.append({"sample": sc.name, "tets": sc.n_elements(), "iters_per_s": round(raw, 3), "wall_s": round(wall, 1)})
    if len(pts) >= 2:
        b = math.log(pts[0]["iters_per_s"] / pts[1]["iters_per_s"]) / math.log(pts[1]["tets"] / pts[0]["tets"])
        fit = f"per-iteration time ~ tets^{b:.3f} (fit through the two samples)"
    else:
        b, fit = 1.0, "linear in tets (one sample)"
    ref = pts[-1]
    value = ref["iters_per_s"] * (ref["tets"] / T) ** b
    # how far the same two-sample fit lands from a MEASURED larger point: the
    # reference at 512k tets, timed once in the build container (tools/ref_c4_points.py; its
    # 33-minute serial factorization does not fit a bench run)
    fit_check = None
    fc = os.path.join(REPO, "profiles", "r5_c4_ref_points.json")
    if os.path.exists(fc):
        d = json.load(open(fc))
        if "fit_check" in d:
            fit_check = {**d["fit_check"], "source": "profiles/r5_c4_ref_points.json", "host": d.get("host"),
                         "points": [{k: p[k] for k in ("sample", "tets", "iters_per_s")} for p in d["points"]],
                         "reading": "the two-sample power law over-predicts the reference's rate at the measured "
                                    "larger point (the per-iteration cost grows faster than the fit), so this "
                                    "extrapolated value is an upper bound on the reference's rate at 1M tets"}
    # the reference MEASURED at the full workload: the reference's own run that
    # made the configs[3] fixture -- the same 1M-tet scene (digest-checked by the parity test), one
    # time step of 10 ADMM iterations after its ~3 h serial factorization, in the build container
    measured = None
    fx = os.path.join(REPO, "tests", "golden", "full_c4_block_z_nh_aa6.npz")
    if os.path.exists(fx) and (cx, cy, cz) == (100, 40, 50):
        d = np.load(fx)
        its = int(d["nrec"].sum())
        ms = float(d["step_ms"].sum())
        measured = {"iters_per_s": round(its / (ms / 1e3), 4), "tets": int(T), "iters": its, "step_ms": round(ms, 1),
                    "threads": 6, "host": "build container: Intel(R) Xeon(R) Processor, 8 CPUs (not the GPU box)",
                    "source": "tests/golden/full_c4_block_z_nh_aa6.npz step_ms (oracle/_ref/ref_elastic_x, the reference "
                              "compiled from its sources; tests/golden/make_golden.py full_c4)",
                    "fit_over_prediction": ("the on-box two-sample fit above is the optimistic side: on the build "
                                            "container the same fit predicts 0.105 it/s at 1M tets and 8 threads (~0.079 "
                                            "scaled to 6) against the measured value here")}
    return {"value": round(value, 3), "unit": "ADMM iters/s", "cores": threads, "kind": kind,
            "value_kind": "extrapolated (two on-box samples, power law); the measured full-size point is in measured_1m",
            "measured_1m": measured,
            "host": {**host_info(), "OMP_NUM_THREADS": threads, "OMP_PROC_BIND": "close", "OMP_PLACES": "cores"},
            "samples": pts, "scaling_fit": fit, "exponent": round(b, 4), "fit_check": fit_check,
            "sample": f"reference X-order solver (admm_anderson_xzu) on make_tet_blocks drops of {', '.join(p['sample'] for p in pts)}"
                      f" (NeoHookean, z-AA m=6, 3 time steps x 10 ADMM iters, median of steps 2-3); value = the "
                      f"largest sample's iters/s x (sample tets / {int(T)})^{b:.3f}" + ("; " + "; ".join(notes) if notes else "")}


def eps_stats(comb, times_ms, eps):
    """(iterations, device ms) until comb <= eps * comb_0, or None."""
    if len(comb) == 0:
        return None
    hit = np.nonzero(comb <= eps * comb[0])[0]
    if len(hit) == 0:
        return None
    k = int(hit[0])
    return k + 1, (float(times_ms[k]) if k < len(times_ms) else None)


def run_to_eps(solver, args, state0):
    """Run-to-epsilon leg (after the timed steps): the reference's default cap of 500 ADMM
    iterations per step and a device-side stop once comb <= 1e-8 comb_0, on time steps 1..eps_steps
    of the drop (replayed from the initial state, like the timed steps). Time to epsilon is
    the device clock (wall_clock64) from the step's start (prologue included) to the end of the
    iteration that reached it."""
    solver.set_iterations(args.eps_cap, EPS_ELASTIC)
    solver.set_state(*state0)   # the same time steps as the timed region, from the initial state
    steps = []
    n_eps = args.steps if args.eps_steps < 0 else args.eps_steps
    for _ in range(n_eps):
        t0 = time.perf_counter()
        solver.step()
        wall = (time.perf_counter() - t0) * 1e3
        h, t = solver.history(), solver.times()
        st = {"iterations": int(solver.runtime().iterations), "step_wall_ms": round(wall, 2)}
        for e in (1e-4, 1e-6, EPS_ELASTIC):
            r = eps_stats(h["comb"], t, e)
            st[f"{e:g}"] = None if r is None else {"iters": r[0], "ms": round(r[1], 3)}
        steps.append(st)
    solver.set_iterations(args.iters, 0.0)
    key = f"{EPS_ELASTIC:g}"
    hit = [s[key]["ms"] for s in steps if s[key] is not None]
    its = [s[key]["iters"] for s in steps if s[key] is not None]
    out = {"eps_rel": EPS_ELASTIC, "cap": args.eps_cap, "steps": len(steps), "reached": len(hit),
           # the headline: median over ALL steps, an unreached step counted as "> cap" (null when more
           # than half of the steps are unreached -- the median is then itself "not reached")
           "median_ms": all_steps_median([s[key]["ms"] if s[key] is not None else None for s in steps]),
           "median_ms_reached_only": round(statistics.median(hit), 3) if hit else None,
           "p90_ms_reached_only": round(float(np.percentile(hit, 90)), 3) if hit else None,
           "iters_to_eps": [s[key]["iters"] if s[key] is not None else None for s in steps],
           "median_iters": all_steps_median([s[key]["iters"] if s[key] is not None else None for s in steps]),
           "not_reached_note": (None if len(hit) == len(steps) else
                                f"not reached in {len(steps) - len(hit)}/{len(steps)} steps with cap {args.eps_cap}"),
           "clock": "device wall_clock64 from the step's start (prologue included) to the end of the iteration "
                    "reaching comb <= eps_rel * comb_0",
           "reference_regime": ("pinned on the 64k-tet drop of the same recipe (profiles/r4_c4_eps_ref_drop40.json vs "
                                "r4_c4_eps_gpu_drop40.json, test_gpu_c4_eps_regime_matches_reference): the reference "
                                "reaches 1e-8 comb_0 in steps 1-5 only, stalls at 2e-7 / 6e-7 / 2e-5 comb_0 in steps 6-8 "
                                "and aborts in step 9 (LBFGS.hpp:192-199) -- the GPU at the same iterations and floors"),
           "per_step": steps}
    for e in (1e-4, 1e-6):
        k = f"{e:g}"
        v = [s[k]["ms"] if s[k] is not None else None for s in steps]
        out[f"median_ms_{k}"] = all_steps_median(v)
        out[f"reached_{k}"] = sum(1 for t in v if t is not None)
    return out


def all_steps_median(vals):
    """Median over every step, None (not reached) ranked above every reached value; None when the
    median itself falls on an unreached step."""
    if not vals:
        return None
    srt = sorted(vals, key=lambda t: (t is None, t if t is not None else 0.0))
    n = len(srt)
    lo, hi = srt[(n - 1) // 2], srt[n // 2]
    if lo is None or hi is None:
        return None
    return round((lo + hi) / 2.0, 3)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.rehearse > 1:   # a timing rehearsal is not a bench line: no baselines, no eps leg
        args.no_cpu_baseline, args.no_secondary, args.eps_steps, args.geom_eps_solves = True, True, 0, 0
    world, rank, local, group, report = dist_setup(args.gpus)
    if args.launch_check:
        # every rank's bound runtime objects and mapped copies, after the RCCL load (ncclGetUniqueId
        # itself needs a GPU: without one only the library load is exercised)
        pkg = importlib.import_module("aa-admm_amd")
        try:
            pkg.capi.Comm.unique_id()
        except pkg.capi.AAError:
            pass
        report = pkg.capi.check_runtime()
        part = args.partition if args.partition != "auto" else ("rccl" if world > 1 else "none")
        all_ranks = group.all_gather_json({"rank": rank, "local_rank": local, "torch_imported": "torch" in sys.modules,
                                           "runtime_bound": report["bound"], "runtime_mapped": report["mapped"]})
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": world, "ranks": all_ranks,
                              "runtime_expected": report["expected"],
                              "parallelism": f"mesh-partitioned{world} ({part})" if part != "none" else f"replicas{world}"}))
        group.close()
        return
    if args.config in ("c3", "c5"):
        return main_geom(args, world, rank, local, group, report)
    pkg = importlib.import_module("aa-admm_amd")
    capi = pkg.capi

    ctx = capi.Context(0 if args.same_device else local)
    sc, desc = elastic_scene(args)
    comm, part = make_comm(pkg, ctx, args, world, rank, group)
    solver = capi.solver_from_scene(ctx, sc, comm)
    if args.lq_stats:
        os.environ["AA_LQ_STATS"] = "1"
    # the process's one-time rocBLAS / rocSOLVER code-object load, timed on its own (it would
    # otherwise sit inside the first factorization: seconds on a fresh box's cold page cache)
    lib_first_use_ms = ctx.warm_dense()
    t0 = time.time()
    solver.initialize(capi.settings_from_scene(sc))
    setup_ms = (time.time() - t0) * 1e3
    setup_phases = solver.setup_phases()
    if os.environ.get("AA_DUMP_MAPS"):   # diagnostics: library map to resolve a crash's frames
        with open("/proc/self/maps") as fi, open(os.environ["AA_DUMP_MAPS"], "w") as fo:
            fo.write(fi.read())
    print(f"[bench] {args.config} setup {setup_ms / 1e3:.1f} s", file=sys.stderr, flush=True)
    for _ in range(args.warmup):
        solver.step()
    # the timed steps (and the run-to-epsilon leg) replay the drop from its initial state
    x0, v0 = np.asarray(sc.x, np.float64).reshape(-1, 3), np.zeros((sc.n_nodes, 3))
    solver.set_state(x0, v0)
    if args.lq_stats:
        solver.local_stats(reset=True)

    barrier(group, ctx)
    t0 = time.perf_counter()
    iters_run, tte, rejects = 0, [], 0
    for _ in range(args.steps):
        solver.step()
        rt = solver.runtime()
        iters_run += rt.iterations
        h = solver.history()
        rejects += int(np.sum(h["reject"]))
        tte.append(eps_stats(h["comb"], solver.times(), EPS_ELASTIC))
    barrier(group, ctx)
    elapsed = time.perf_counter() - t0
    elapsed_max = allreduce(group, elapsed, "max")
    # replicas: every rank ran its own copy of the scene (weak scaling); partitioned: all ranks
    # ran ONE scene together (strong scaling), its iterations count once
    iters_all = float(iters_run) if comm is not None else allreduce(group, float(iters_run), "sum")
    value = iters_all / elapsed_max

    lq = None
    if args.lq_stats:
        st = solver.local_stats(reset=True)
        h = st["hist"]
        its = float((h * np.arange(len(h))).sum())
        lq = {"elements": int(h.sum()), "mean_lbfgs_iters": round(its / max(1, h.sum()), 3),
              "hist": {str(i): int(c) for i, c in enumerate(h) if c},
              "trips": st["trips"], "refills": st["refills"], "waves": st["waves"],
              "lane_busy_frac": round(its / max(1, 64 * st["trips"]), 4)}
    # roofline of the dominant kernel class, timed live with HIP events on the solver's stream
    # (separate instrumented pass of the same iteration loop, after the timed region; every
    # rank of a partitioned run takes part -- the loop has collectives)
    roof = None
    if comm is not None:
        solver.bench_iterations(min(args.iters, 50))
    if rank == 0:
        if comm is None:
            solver.bench_iterations(min(args.iters, 50))
        names = ("local_z", "solve", "resid", "rhs", "aa") if sc.variant == 1 else \
                ("grad", "rhs", "solve", "solve1", "prim", "local_z", "aa", "comb", "reject", "copy")
        stats = {k: solver.kernel_stats(k) for k in names}
        per_iter = {k: v["avg_ms"] * v["launches"] for k, v in stats.items()}
        k = "solve"   # the global solve: the dominant HBM-bound phase (north_star roofline)
        st = stats[k]
        achieved = st["bytes"] / (st["avg_ms"] * 1e-3) / 1e9 if st["avg_ms"] > 0 else 0.0
        # Z variant + Anderson: the iteration's solve and the previous iteration's
        # combined-residual solve run as ONE two-set pass over the factor (6 RHS)
        pipelined = sc.variant != 1 and sc.accel and os.environ.get("AA_Z_PIPELINE", "1") != "0"
        roof = {"kernel": "global solve: multifrontal triangular solves, " +
                ("6 RHS = this iteration's solve + the previous iteration's combined-residual solve in one pass "
                 "(k_fwd*/k_bwd* per pass)" if pipelined else "3 RHS (k_fwd*/k_bwd* per solve)"),
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "avg_launch_us": round(st["avg_ms"] * 1e3, 2), "bytes_per_launch": st["bytes"],
                "phase_us_per_launch": {kk: round(v["avg_ms"] * 1e3, 2) for kk, v in stats.items()},
                "phase_bytes_per_launch": {kk: v["bytes"] for kk, v in stats.items()},
                "dominant_phase": max(per_iter, key=per_iter.get)}
        try:   # the measured HBM read ceiling (16-B/lane streaming read of 2 GiB) beside the spec
            cp = ctx.bench_read(2 << 30)
            roof["read_peak_measured"] = round(cp, 1)
            roof["frac_of_read_peak"] = round(achieved / cp, 4) if cp > 0 else None
        except Exception as e:
            roof["read_peak_measured"] = None
            roof["read_peak_error"] = str(e)[:120]
    if roof is not None:   # HBM bytes per solve from the committed PMC passes (tools/gpu.sh pmc)
        pmc = next((q for q in (os.path.join(REPO, "profiles", f"r{k}_{args.config}_pmc.json") for k in (6, 5, 4, 3, 2, 1))
                    if os.path.exists(q)), "")
        if pmc and comm is None:
            # the PMC group of the same solve the roofline times: two-set (6 RHS) when pipelined
            key = "solve2_per_launch" if pipelined else "solve_per_launch"
            sp = json.load(open(pmc)).get(key) or {}
            if sp.get("traffic_B"):
                roof["traffic"] = sp["traffic_B"]
                roof["traffic_source"] = (f"profiles/{os.path.basename(pmc)} {key}: FETCH_SIZE (x2, calibrated on "
                                          f"k_copy) + WRITE_SIZE over the solve's {sp['kernels']} kernels, separate "
                                          "--pmc passes")
    # run-to-epsilon leg (every rank: a partitioned loop has collectives)
    eps_leg = run_to_eps(solver, args, (x0, v0)) if args.eps_steps != 0 else None
    rt = solver.runtime()
    solver.close()
    if comm is not None:
        comm.close()
    ctx.close()

    # north_star's second target (BASELINE configs[2], the 100k-face PQ mesh) in the same line;
    # at N > 1 as independent replicas (the partitioned geometry path is exercised by the tests)
    secondary = None
    if args.config == "c4" and not args.no_secondary:
        a3 = argparse.Namespace(**{**vars(args), "config": "c3", "iters": 100, "nx": 112,
                                   "partition": "none" if world > 1 else args.partition})
        try:
            secondary = geom_line(a3, world, rank, local, group)
        except Exception as e:   # report, never lose the primary line
            secondary = {"config": "c3", "error": str(e)[:300]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        print("[bench] timing the reference CPU baseline", file=sys.stderr, flush=True)
        try:
            cpu = elastic_cpu_baseline(args)
        except Exception as e:  # report, never fail the GPU number on the baseline leg
            cpu = {"value": None, "error": str(e)[:200]}

    if rank == 0:
        tt = [t[1] for t in tte if t is not None]
        line = {
            "metric": "ADMM iters/sec + time-to-eps (primal+dual residual)", "value": round(value, 2),
            "unit": "ADMM iters/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed_max * 1e3 / args.steps, 3), "higher_is_better": True,
            "scaling": "strong" if comm is not None else "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": ("synthetic (generated make_tet_blocks mesh)" if args.mesh == "block" else
                     "voxelised reference mesh (bunny_closed.obj -> aa-admm_amd/data/bunny_vox%d.npz)" % args.bunny_res)
                    if args.config == "c4" else "synthetic (generated make_tri_blocks mesh)",
            "config": {"workload": desc, "nodes": sc.n_nodes, "elements": sc.n_elements(),
                       "admm_iters_per_step": args.iters, "anderson_m": sc.aa_m,
                       "parallelism": (f"mesh-partitioned{world} ({part})" if comm is not None else f"replicas{world}"),
                       "global_solve": "supernodal direct", "nnz_factor": rt.nnz_factor,
                       "setup_ms": round(setup_ms, 1),
                       # initialize()'s phases (Solver.cpp:373-498; their sum vs setup_ms: the binding's
                       # own overhead) and, outside setup_ms, the process's one-time library load
                       "setup_breakdown": {"phases_ms": setup_phases,
                                           "phases_sum_ms": round(sum(setup_phases.values()), 1),
                                           "library_first_use_ms": round(lib_first_use_ms, 1)}},
            "iters_executed": int(iters_all),
            # Anderson rejects in the timed steps (each re-runs a one-set solve: SURVEY App. B.11)
            "anderson_rejects": rejects,
            # run-to-epsilon leg (cap 500, stop at 1e-8 comb_0); null when no step reached it
            "time_to_eps_ms": eps_leg["median_ms"] if eps_leg else None, "eps_rel": EPS_ELASTIC,
            "time_to_eps": eps_leg,
            "eps_in_timed_steps": {"iters_cap": args.iters, "steps": len(tte), "reached": len(tt),
                                   "median_ms": all_steps_median([t[1] if t is not None else None for t in tte]),
                                   "median_ms_reached_only": round(statistics.median(tt), 3) if tt else None},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if comm is not None:
            line["config"]["partition"] = {"elements_rank0": rt.n_elements, "z_dim_rank0": rt.z_dim}
        if args.rehearse > 1:
            line["metric"] = f"REHEARSAL (not a result): one rank's share of a {args.rehearse}-GPU partition"
            line["rehearsal"] = {"P": args.rehearse, "rank": args.rehearse_rank,
                                 "us_per_iter": round(elapsed_max * 1e6 / max(1, iters_run), 2),
                                 "note": "collectives replaced by local stand-ins (aa_comm_create_solo); add the "
                                         "all-reduce cost for a P-GPU estimate"}
        if lq is not None:
            line["local_step_queue"] = lq
        if secondary is not None:
            line["secondary"] = secondary
        line["runtime_libs"] = report["bound"]
        print(json.dumps(line))
    group.close()


if __name__ == "__main__":
    main()
