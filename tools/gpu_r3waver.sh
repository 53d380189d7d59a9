#!/bin/bash
# backward split-K threshold (AA_SOLVE_WAVER, R above it -> tiles) re-checked with the narrow tiles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for cfg in c4 c3; do
  echo "== $cfg"
  CFG=$cfg BENCH_ARGS="--eps-steps 0 --no-secondary" SWEEP="AA_SOLVE_WAVER=384 AA_SOLVE_WAVER=256 AA_SOLVE_WAVER=192 AA_SOLVE_WAVER=128 AA_SOLVE_WAVER=384 AA_SOLVE_WAVER=256" bash tools/gpu_sweep.sh || exit $?
done
