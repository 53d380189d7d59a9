#!/bin/bash
# round 3 call p: row-loop unroll 8 / 12 / 16 (fused subtrees + row tasks) -- identity + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
for lib in u8 c8; do
  AA_ADMM_LIB="$R/ab/lib_$lib.so" timeout -k 10 200 python3 tools/ab_dump.py gpurun_out/dump_drop40_$lib.npz drop40 > gpurun_out/dump_drop40_$lib.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "dump $lib rc=$rc"; tail -5 gpurun_out/dump_drop40_$lib.log; exit $rc; }
done
echo "drop40 u8 vs c8: $(python3 tools/ab_dump.py --compare gpurun_out/dump_drop40_u8.npz gpurun_out/dump_drop40_c8.npz)"
B="--steps 4 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0"
for cfg in c4 c3 c2; do
for lib in u8 c8 c16 c4 c8 u8; do
  tag=${lib}_$cfg
  AA_ADMM_LIB="$R/ab/lib_$lib.so" timeout -k 10 300 python3 -u bench.py --config $cfg $B > gpurun_out/ab_r3q_$tag.log 2> gpurun_out/ab_r3q_$tag.err; rc=$?
  echo "$tag rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3q_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'])")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3q_$tag.err; exit $rc; }
done; done
AA_ADMM_LIB="$R/ab/lib_c8.so" AA_SUB_TIMING=2 AA_ADMM_NO_GRAPH=1 timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > gpurun_out/subtiming_r3q.log 2>&1; rc=$?
echo "subtiming c8 rc=$rc"; grep "sub timing" gpurun_out/subtiming_r3q.log | head -2
exit 0
