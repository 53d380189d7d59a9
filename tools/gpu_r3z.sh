#!/bin/bash
# round 3 call z: C2 / C5 / C3 lines with their CPU baselines; C3 kernel-trace summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
for cfg in c2 c3 c5; do
  timeout -k 10 600 python3 -u bench.py --config $cfg --steps 10 --warmup 3 > gpurun_out/bench_r3z_$cfg.log 2> gpurun_out/bench_r3z_$cfg.err; rc=$?
  echo "bench $cfg rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_r3z_$cfg.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],(d.get('cpu_baseline') or {}).get('value'),d['config'].get('setup_ms'))")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r3z_$cfg.err; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
AA_ADMM_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3z_c3" -o run -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu-baseline --geom-eps-solves 0 > "$R/gpurun_out/prof_r3z_c3.log" 2>&1; rc=$?
echo "prof c3 rc=$rc"; [ $rc -ne 0 ] && { grep -v "^ *@" "$R/gpurun_out/prof_r3z_c3.log" | tail -5; exit $rc; }
f=$(find "$R/gpurun_out/prof_r3z_c3" -name "*kernel_stats.csv" | head -1); head -16 "$f" | cut -c1-160
exit 0
