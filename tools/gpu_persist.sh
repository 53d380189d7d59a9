#!/bin/bash
# Persistent-sweep check: bit-identity tests, then C4 / C3 solve timings (persistent vs levels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "persistent or run_to_eps or full_drop40 or pipelined" > gpurun_out/pytest_persist.log 2>&1; rc=$?
echo "pytest_rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_persist.log | tail -20
[ $rc -ne 0 ] && exit $rc
for lv in 1 2 0; do
  AA_SOLVE_PERSIST=$(( lv > 0 ? 1 : 0 )) AA_SOLVE_PERSIST_ACQ=$(( lv == 2 ? 1 : 0 )) AA_SOLVE_STATS=1 timeout -k 10 300 python -u bench.py --config c4 --steps 3 --no-cpu-baseline --no-secondary --eps-steps 0 > gpurun_out/bench_persist_c4_$lv.log 2>&1; rc=$?
  echo "c4 mode=$lv rc=$rc"; grep -E "persistent sweeps" gpurun_out/bench_persist_c4_$lv.log | head -2
  grep '^{' gpurun_out/bench_persist_c4_$lv.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'solve_us', r['avg_launch_us'], 'frac', r['frac'], r['phase_us_per_launch'])"
  [ $rc -ne 0 ] && exit $rc
done
for lv in 1 2 0; do
  AA_SOLVE_PERSIST=$(( lv > 0 ? 1 : 0 )) AA_SOLVE_PERSIST_ACQ=$(( lv == 2 ? 1 : 0 )) timeout -k 10 300 python -u bench.py --config c3 --steps 3 --no-cpu-baseline > gpurun_out/bench_persist_c3_$lv.log 2>&1; rc=$?
  echo "c3 mode=$lv rc=$rc"
  grep '^{' gpurun_out/bench_persist_c3_$lv.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'solve_us', r['avg_launch_us'], 'frac', r['frac'])"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
