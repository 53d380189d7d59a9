#!/bin/bash
# round 3 call x: split-K thresholds (forward rows p > WAVEP and backward columns R > WAVER tiled)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
B="--steps 4 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0"
for cfg in c4 c3 c2; do
for v in "AA_SOLVE_WAVEP=192" "AA_SOLVE_WAVEP=96" "AA_SOLVE_WAVEP=128" "AA_SOLVE_WAVEP=64" "AA_SOLVE_WAVEP=192" "AA_SOLVE_WAVEP=96"; do
  tag=$(echo "$v" | tr ' =' '__')_$cfg
  env $v timeout -k 10 300 python3 -u bench.py --config $cfg $B > gpurun_out/ab_r3x_$tag.log 2> gpurun_out/ab_r3x_$tag.err; rc=$?
  echo "$tag rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3x_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'])")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3x_$tag.err; exit $rc; }
done; done
exit 0
