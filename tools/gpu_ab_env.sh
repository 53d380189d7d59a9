#!/bin/bash
# A/B of library builds x environment settings on one box: "lib|ENV=V ENV2=V" per entry in CASES.
#   CASES="ab/lib_head.so| ab/lib_v1.so|AA_SOLVE_TILE=128" CFG=c4 bash tools/gpu_ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
CFG=${CFG:-c4}
i=0
for c in $CASES; do
  lib=${c%%|*}; envs=${c#*|}; envs=${envs//,/ }
  i=$((i+1)); tag="$i_$(basename "$lib" .so)"
  env AA_ADMM_LIB="$PWD/$lib" $envs timeout -k 10 ${T:-300} python -u bench.py --config $CFG --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --eps-steps 0 --no-secondary ${BENCH_ARGS} > gpurun_out/abe_${CFG}_$i.log 2>&1; rc=$?
  echo "== $i $lib [$envs] rc=$rc"
  case $rc in 0) ;; *) tail -5 gpurun_out/abe_${CFG}_$i.log; exit $rc;; esac
  python - gpurun_out/abe_${CFG}_$i.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "frac", r.get("frac"), "phases", r.get("phase_us_per_launch"))
PY
done
exit 0
