"""bench.py's multi-rank launcher: `bench.py --gpus N` run without an outside
torch.distributed.run must start N ranks itself (as a child process, before any HIP call) so the
driver's 1/2/4/8-GPU line reports N ranks, and a WORLD_SIZE that disagrees with --gpus must fail.
Each rank reports the ROCm runtime it is bound to: never torch's bundled one.
The CPU test stops at --launch-check (no GPU); the GPU test runs a real 2-rank partitioned step
(host transport, both ranks on GPU 0)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bench_gpus2_launches_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                       timeout=300, env=_env(), cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2
    assert [q["rank"] for q in line["ranks"]] == [0, 1]
    assert [q["local_rank"] for q in line["ranks"]] == [0, 1]
    assert line["parallelism"] == "mesh-partitioned2 (rccl)"
    # each rank: no torch in the process, every runtime object (incl. the dlopened RCCL) from the
    # directory libaa_admm.so was linked against
    for q in line["ranks"]:
        assert q["torch_imported"] is False
        for name, path in q["runtime_bound"].items():
            assert os.path.dirname(path) == line["runtime_expected"], (q["rank"], name, path)
        for name, paths in q["runtime_mapped"].items():
            assert paths and all(os.path.dirname(p) == line["runtime_expected"] for p in paths), (name, paths)


def test_bench_single_gpu_default_is_one_rank():
    r = subprocess.run([sys.executable, BENCH, "--launch-check"], capture_output=True, text=True, timeout=120,
                       env=_env(), cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 1 and line["parallelism"] == "replicas1"


def test_bench_world_size_mismatch_fails():
    env = dict(_env(), WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-check"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=REPO)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in (r.stderr + r.stdout)


@pytest.mark.gpu
def test_bench_gpus2_partitioned_step_on_one_gpu():
    """Two ranks of one partitioned cloth (host transport, same GPU): the line says 2 ranks."""
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--partition", "host", "--same-device",
                        "--config", "c2", "--nx", "24", "--steps", "1", "--warmup", "1", "--iters", "20",
                        "--no-cpu-baseline", "--eps-steps", "0"],
                       capture_output=True, text=True, timeout=110, env=_env(), cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "mesh-partitioned2 (host)"
    assert line["iters_executed"] == 20 and line["value"] > 0


def test_time_to_eps_median_counts_unreached_steps():
    """The time-to-epsilon headline is the median over ALL steps with an unreached step ranked
    above every reached one ("> cap"), so a majority of unreached steps yields null instead of the
    median of the survivors."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    m = b.all_steps_median
    assert m([]) is None
    assert m([10.0, 30.0, 20.0]) == 20.0
    assert m([10.0, None, 20.0]) == 20.0            # 10, 20, >cap
    assert m([10.0, None, None]) is None            # the middle step is unreached
    assert m([10.0, 40.0, None, None]) is None      # even count: the upper middle is unreached
    assert m([10.0, 40.0, 30.0, None]) == 35.0
    assert m([None] * 13 + [5.0] * 7) is None       # round 3's 7/20 survivors no longer make a headline
