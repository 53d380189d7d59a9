#!/bin/bash
# round 3 call w: full GPU suite with the size-dependent top amalgamation, then a short line per config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3w.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3w.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_r3w.log | head -20; exit $rc; }
B="--steps 4 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0"
for cfg in c2 c3 c4 c5; do
  timeout -k 10 300 python3 -u bench.py --config $cfg $B > gpurun_out/ab_r3w_$cfg.log 2> gpurun_out/ab_r3w_$cfg.err; rc=$?
  echo "$cfg rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3w_$cfg.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],'nnz',d['config']['nnz_factor'],'setup',d['config']['setup_ms'])")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3w_$cfg.err; exit $rc; }
done
exit 0
