#!/bin/bash
# round 3 call m: XCD-aware tile placement A/B (AA_SOLVE_XCD), solve tests, kernel trace of one solve
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3m.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/pytest_r3m.log; [ $rc -ne 0 ] && exit $rc
B="--steps 5 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary"
for cfg in c4 c3 c2; do
for v in 1 0 1; do
  tag=xcd${v}_$cfg
  AA_SOLVE_XCD=$v timeout -k 10 300 python3 -u bench.py --config $cfg $B > gpurun_out/ab_r3m_$tag.log 2> gpurun_out/ab_r3m_$tag.err; rc=$?
  echo "$tag rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3m_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r.get('read_peak_measured'),r.get('phase_us_per_iter') or r.get('phase_us_per_launch'))")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3m_$tag.err; exit $rc; }
done; done
cd /tmp && export TMPDIR=/tmp
AA_ADMM_NO_GRAPH=1 AA_EAGER_SYNC=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3m" -o run -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/prof_r3m.log" 2>&1; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { grep -v "^ *@" "$R/gpurun_out/prof_r3m.log" | tail -5; exit $rc; }
f=$(find "$R/gpurun_out/prof_r3m" -name "*kernel_trace.csv" | head -1); python3 "$R/tools/solve_levels.py" "$f" 6 > "$R/gpurun_out/prof_r3m_levels.txt"; cat "$R/gpurun_out/prof_r3m_levels.txt"
exit 0
