#!/bin/bash
# round 3 call f: bunny golden test, tile depth A/B, bunny bench, graph-mode traces A/B lookahead
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_elastic.py -k "bunny40" -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r3f.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/pytest_r3f.log | tail -5; [ $rc -ne 0 ] && exit $rc
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 1 --no-cpu-baseline --eps-steps 0 --no-secondary > gpurun_out/ab_$tag.log 2> gpurun_out/ab_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/ab_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_us'],r['frac'],r['phase_us_per_launch'])")"
  return $rc
}
run f2b2 AA_TILE_DEPTH_F=2 AA_TILE_DEPTH_B=2 && run f4b3 AA_TILE_DEPTH_F=4 AA_TILE_DEPTH_B=3 && run f4b4 AA_TILE_DEPTH_F=4 AA_TILE_DEPTH_B=4 \
  && run f3b3 AA_TILE_DEPTH_F=3 AA_TILE_DEPTH_B=3 && run f2b2b AA_TILE_DEPTH_F=2 AA_TILE_DEPTH_B=2 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_geom.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3f_geom.log 2>&1; rc=$?
echo "geom pytest rc=$rc"; tail -3 gpurun_out/pytest_r3f_geom.log; [ $rc -ne 0 ] && exit $rc
for cfg in c3 c5; do for ss in 0 16; do
  AA_SURF_SORT=$ss timeout -k 10 300 python3 -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --geom-eps-solves 0 > gpurun_out/ab_${cfg}_sort$ss.log 2> gpurun_out/ab_${cfg}_sort$ss.err; rc=$?
  echo "$cfg sort=$ss rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_${cfg}_sort$ss.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['phase_us_per_iter'])")"
  [ $rc -ne 0 ] && exit $rc
done; done
timeout -k 10 400 python3 -u bench.py --mesh bunny --steps 5 --warmup 1 --no-cpu-baseline --eps-steps 5 --no-secondary > gpurun_out/bench_r3f_bunny.log 2> gpurun_out/bench_r3f_bunny.err; rc=$?
echo "bunny bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r3f_bunny.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for ah in 0 1; do
  AA_LQ_AHEAD=$ah timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3f_ah$ah" -o run -- python3 "$R/bench.py" --steps 3 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/prof_r3f_ah$ah.log" 2>&1; rc=$?
  echo "prof ahead=$ah rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/prof_r3f_ah$ah.log"; exit $rc; }
done
exit 0
