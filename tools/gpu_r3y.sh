#!/bin/bash
# round 3 call y: warm closest-point queries over the sibling path -- geometry tests, A/B C3 / C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
AA_ADMM_LIB="$R/ab/lib_sib1.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_geom.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3y.log 2>&1; rc=$?
echo "geom tests rc=$rc"; tail -2 gpurun_out/pytest_r3y.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_r3y.log | head -20; exit $rc; }
for lib in sib0 sib1; do
  AA_ADMM_LIB="$R/ab/lib_$lib.so" timeout -k 10 200 python3 tools/ab_dump.py gpurun_out/dump_pq_$lib.npz pq > gpurun_out/dump_pq_$lib.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "dump $lib rc=$rc"; tail -5 gpurun_out/dump_pq_$lib.log; exit $rc; }
done
echo "pq sib0 vs sib1: $(python3 tools/ab_dump.py --compare gpurun_out/dump_pq_sib0.npz gpurun_out/dump_pq_sib1.npz)"
B="--steps 4 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0"
for cfg in c3 c5; do
for lib in sib0 sib1 sib0 sib1; do
  tag=${lib}_$cfg
  AA_ADMM_LIB="$R/ab/lib_$lib.so" timeout -k 10 300 python3 -u bench.py --config $cfg $B > gpurun_out/ab_r3y_$tag.log 2> gpurun_out/ab_r3y_$tag.err; rc=$?
  echo "$tag rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3y_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],'z',r['phase_us_per_iter']['z'])")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3y_$tag.err; exit $rc; }
done; done
exit 0
