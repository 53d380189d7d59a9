#!/bin/bash
# Solve-geometry sweep: parity subset, then the C4 / C3 roofline solve time under several
# split-K settings (env: AA_SOLVE_MIN_TILES, AA_SOLVE_WAVEP, AA_SOLVE_WAVER, AA_SOLVE_TILE).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYK:-pipelined or full_drop40 or golden or full_size_c3}" > gpurun_out/pytest_sweep.log 2>&1; rc=$?
echo "pytest_rc=$rc"; tail -2 gpurun_out/pytest_sweep.log
[ $rc -ne 0 ] && exit $rc
i=0
while read -r cfg envs; do
  [ -z "$cfg" ] && continue
  i=$((i+1))
  env $envs AA_SOLVE_STATS=1 timeout -k 10 300 python -u bench.py --config $cfg --steps 2 --no-cpu-baseline --no-secondary --eps-steps 0 > gpurun_out/sweep_$i.log 2>&1; rc=$?
  echo "[$i] $cfg $envs rc=$rc"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/sweep_$i.log; exit $rc; }
  grep '^{' gpurun_out/sweep_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('   value', d['value'], 'solve_us', r['avg_launch_us'], 'frac', r['frac'])"
done < "${SWEEP:-tools/sweep_solve.txt}"
exit 0
