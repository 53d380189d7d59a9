#!/bin/bash
# Correctness first (all GPU tests), then C4/C2 bench variants. Each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
TESTS=${TESTS:-tests/}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_iter.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/pytest_iter.log | head -20; exit $rc; }
for v in ${VARIANTS:-"c4:"}; do
  cfg=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/iter_$cfg.log 2>&1; rc=$?
  echo "== $cfg [$envs] rc=$rc"
  python3 - "$cfg" <<'PY'
import json, sys
for l in open(f"gpurun_out/iter_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(" value", d["value"], "solve_us", r.get("avg_launch_us"), "frac", r["frac"], {k: v for k, v in (r.get("phase_us_per_launch") or r.get("phase_us_per_iter")).items()})
PY
  [ $rc -ne 0 ] && { tail -20 gpurun_out/iter_$cfg.log; exit $rc; }
done
exit 0
