#!/bin/bash
# round 3 call o: fused-subtree phase clocks with start/end spread, C3 setup breakdown, bunny C4 line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
AA_SUB_TIMING=2 AA_ADMM_NO_GRAPH=1 timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > gpurun_out/subtiming_r3o.log 2>&1; rc=$?
echo "subtiming rc=$rc"; grep "sub timing" gpurun_out/subtiming_r3o.log | head -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --geom-eps-solves 0 > gpurun_out/c3_r3o.log 2> gpurun_out/c3_r3o.err; rc=$?
echo "c3 rc=$rc"; grep "setup" gpurun_out/c3_r3o.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u bench.py --mesh bunny --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/bunny_r3o.log 2> gpurun_out/bunny_r3o.err; rc=$?
echo "bunny rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bunny_r3o.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],d['config']['elements'],d['config']['setup_ms'],r['avg_launch_us'],r['frac'],d['time_to_eps']['reached'],d['time_to_eps']['median_ms'])")"
exit $rc
