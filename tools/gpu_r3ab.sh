#!/bin/bash
# Round-3: two-phase closest-point schedule (AA_BVH_HOLD_PCT builds) -- bit-identity on a PQ scene,
# C3 / C5 A/B, and the SQ counters of the C5 z kernel (summarised on the box, raw CSVs dropped).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in 0 50 100; do
  AA_ADMM_LIB=$PWD/ab/lib_hold$v.so timeout -k 10 120 python -u tools/ab_dump.py gpurun_out/ab_pq_hold$v.npz pq > gpurun_out/ab_pq_hold$v.log 2>&1 || { echo "dump $v failed"; tail -5 gpurun_out/ab_pq_hold$v.log; exit 1; }
done
python tools/ab_dump.py --compare gpurun_out/ab_pq_hold0.npz gpurun_out/ab_pq_hold50.npz || exit 1
python tools/ab_dump.py --compare gpurun_out/ab_pq_hold0.npz gpurun_out/ab_pq_hold100.npz || exit 1
for cfg in c5 c3; do
  for v in ${HOLDS:-0 50 75 100 25}; do
    AA_ADMM_LIB=$PWD/ab/lib_hold$v.so timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0 > gpurun_out/ab_${cfg}_hold$v.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "bench $cfg $v rc=$rc"; tail -5 gpurun_out/ab_${cfg}_hold$v.log; exit $rc; }
    python - $cfg $v gpurun_out/ab_${cfg}_hold$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print(sys.argv[1], "hold", sys.argv[2], "value", d["value"], "phases", d["roofline"].get("phase_us_per_iter"))
PY
  done
done
exit 0
