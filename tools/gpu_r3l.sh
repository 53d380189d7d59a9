#!/bin/bash
# round 3 call l: non-temporal factor loads (A/B builds), read ceiling forms, solve tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_elastic.py -k "streamed or lds_history or pipelined or drop40" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3l.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/pytest_r3l.log; [ $rc -ne 0 ] && exit $rc
B="--steps 5 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary"
for lib in ab/lib_nt1.so ab/lib_nt0.so ab/lib_nt1.so ab/lib_nt0.so; do
  tag=$(basename $lib .so)
  AA_ADMM_LIB="$R/$lib" timeout -k 10 300 python3 -u bench.py $B > gpurun_out/ab_r3l_$tag.log 2> gpurun_out/ab_r3l_$tag.err; rc=$?
  echo "$tag rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3l_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['read_peak_measured'],r['phase_us_per_launch'])")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3l_$tag.err; exit $rc; }
done
for cfg in c3 c2; do
for lib in ab/lib_nt1.so ab/lib_nt0.so; do
  tag=$(basename $lib .so)_$cfg
  AA_ADMM_LIB="$R/$lib" timeout -k 10 300 python3 -u bench.py --config $cfg $B > gpurun_out/ab_r3l_$tag.log 2> gpurun_out/ab_r3l_$tag.err; rc=$?
  echo "$tag rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3l_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r.get('phase_us_per_iter') or r.get('phase_us_per_launch'))")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3l_$tag.err; exit $rc; }
done; done
exit 0
