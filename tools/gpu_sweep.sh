#!/bin/bash
# C4 bench under a list of environment settings (one run each, own time limit), e.g.
#   SWEEP="AA_SOLVE_MIN_SUBTREES=256 AA_SOLVE_MIN_SUBTREES=512" bash tools/gpu_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
CFG=${CFG:-c4}
k=0
for kv in ${SWEEP}; do
  k=$((k+1))
  env $(echo "$kv" | tr ',' ' ') timeout -k 10 300 python -u bench.py --config $CFG --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/sweep_$k.log 2>&1; rc=$?
  v=$(grep -h '^{' gpurun_out/sweep_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline'].get('phase_us_per_launch'))")
  echo "$kv rc=$rc $v"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
